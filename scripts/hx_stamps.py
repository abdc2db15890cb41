"""Phase stamps of hx_user_kernel (diagnostic build: HREC_HX_STAMPS, loaded
through HREC_LIB): per phase the mean / max s_memtime ticks over the blocks of
the last local() call at c2, and the slowest block's split.

    bash scripts/build_variants.sh "hxst:-DHREC_HX_STAMPS"
    HREC_LIB=.../lib/ab/libhrec_hxst.so python scripts/hx_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import hx_probe  # noqa: E402

from src import _hrec  # noqa: E402


def main():
    torch.cuda.set_device(0)
    rec, hu, uvec = hx_probe.setup(256, 2)
    lib = _hrec.lib()
    for wins in (False, True):
        rec.recommend(hu, uvec, wins, 5)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (1024 * 16 + 1024 * 32))()
        assert lib.hrec_debug_hx_stamps(buf) == 0
        arr = np.array(buf, dtype=np.int64)
        st = arr[:1024 * 16].reshape(1024, 16)[:256]
        ws = arr[1024 * 16:].reshape(1024, 8, 4)[:256]
        d = np.diff(st[:, :7], axis=1)
        names = ["rows+norms+approx extremes", "extremes sweep", "seeds", "top-k sweep", "merge", "tail"]
        n_ext, n_top, _ = rec.last_exact.counts()
        tot = st[:, 6] - st[:, 0]
        worst = int(np.argmax(tot))
        print(f"als_wins={wins}: total ticks mean {tot.mean():.0f} max {tot.max()} (block {worst}: "
              f"{int(n_ext[worst])} extreme groups, {int(n_top[worst])} live groups)")
        for k, nm in enumerate(names):
            print(f"  {nm:28s} mean {d[:, k].mean():9.0f}  max {d[:, k].max():9d}  worst-block {d[worst, k]:9d}")
        sub = {"stats->LDS start": (0, 12), "stats->LDS + rows (to barrier)": (12, 13), "barrier": (13, 14),
               "seed ub scan": (7, 8), "seed wave_best x2": (8, 9), "seed scan (1 pair)": (9, 10),
               "seed insert": (10, 11), "seed merge": (11, 3)}
        for nm, (x, y) in sub.items():
            dd = st[:, y] - st[:, x]
            print(f"    {nm:30s} mean {dd.mean():9.0f}  max {dd.max():9d}")
        ub_scan = ws[:, :, 1] - ws[:, :, 0]
        to_merge = ws[:, :, 2] - ws[:, :, 0]
        start_skew = ws[:, :, 0] - ws[:, :1, 0]
        print(f"    per wave: seed start skew vs wave 0 mean {start_skew.mean(0).round(0).tolist()}")
        print(f"    per wave: ub scan + wave_best + scan mean {ub_scan.mean(0).round(0).tolist()}")
        print(f"    per wave: to merge entry mean {to_merge.mean(0).round(0).tolist()}")
        b1 = (ctypes.c_ulonglong * (4096 * 4))()
        assert lib.hrec_debug_hx1_stamps(b1) == 0
        s1 = np.array(b1, dtype=np.int64).reshape(4096, 4)
        nb = int((s1[:, 0] > 0).sum())
        s1 = s1[:nb]
        t0 = s1[:, 0].min()
        print(f"  phase 1 ({nb} blocks): span {s1[:, 2:].max() - t0} ticks; per block staging mean "
              f"{(s1[:, 1] - s1[:, 0]).mean():.0f}, loop w0 mean {(s1[:, 2] - s1[:, 1]).mean():.0f} max "
              f"{(s1[:, 2] - s1[:, 1]).max()}; block start offsets max {s1[:, 0].max() - t0}")
        corr = np.corrcoef(n_top.cpu().numpy(), d[:, 3])[0, 1]
        print(f"  top-k sweep ticks vs live groups: corr {corr:.2f}, ticks per live group "
              f"{(d[:, 3] / np.maximum(n_top.cpu().numpy(), 1)).mean():.0f}")


if __name__ == "__main__":
    main()
