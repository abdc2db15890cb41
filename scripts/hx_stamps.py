"""Phase stamps of hx_pre_kernel and hx_stats_kernel (diagnostic build:
HREC_HX_STAMPS, loaded through HREC_LIB): per phase the mean / max s_memtime
ticks over the blocks of the last local() call at c2.

    bash scripts/build_variants.sh "hxst:-DHREC_HX_STAMPS"
    HREC_LIB=.../lib/variants/libhrec_hxst.so python scripts/hx_stamps.py
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
        buf = (ctypes.c_ulonglong * (1024 * 16))()
        assert lib.hrec_debug_hx_stamps(buf) == 0
        st = np.array(buf, dtype=np.int64).reshape(1024, 16)[:256]
        d = np.diff(st[:, :5], axis=1)
        names = ["stats->LDS + rows + norms", "extremes", "seeds + tau", "live count + queue"]
        n_ext, n_top, _ = rec.last_exact.counts()
        tot = st[:, 4] - st[:, 0]
        worst = int(np.argmax(tot))
        print(f"als_wins={wins}: 2a ticks mean {tot.mean():.0f} max {tot.max()} (block {worst}: "
              f"{int(n_ext[worst])} extreme groups, {int(n_top[worst])} live groups); "
              f"2a block start spread {st[:, 0].max() - st[:, 0].min()}")
        for k, nm in enumerate(names):
            print(f"  {nm:28s} mean {d[:, k].mean():9.0f}  max {d[:, k].max():9d}  worst-block {d[worst, k]:9d}")
        bp = (ctypes.c_ulonglong * (8192 * 4))()
        assert lib.hrec_debug_hx_pstamps(bp) == 0
        sp = np.array(bp, dtype=np.int64).reshape(8192, 4)
        sp = sp[sp[:, 0] > 0]
        dur = sp[:, 1] - sp[:, 0]
        busy = sp[sp[:, 2] > 0]
        print(f"  2b ({len(sp)} waves): span {sp[:, 1].max() - sp[:, 0].min()} ticks; start spread "
              f"{sp[:, 0].max() - sp[:, 0].min()}; pairs total {sp[:, 2].sum()} (max/wave {sp[:, 2].max()}), "
              f"exact items {sp[:, 3].sum()}; wave ticks mean {dur.mean():.0f} max {dur.max()}; "
              f"ticks per pair (busy waves) {((busy[:, 1] - busy[:, 0]) / busy[:, 2]).mean():.0f}")
        b1 = (ctypes.c_ulonglong * (4096 * 4))()
        assert lib.hrec_debug_hx1_stamps(b1) == 0
        s1 = np.array(b1, dtype=np.int64).reshape(4096, 4)
        nb = int((s1[:, 0] > 0).sum())
        s1 = s1[:nb]
        t0 = s1[:, 0].min()
        print(f"  phase 1 ({nb} blocks): span {s1[:, 2:].max() - t0} ticks; per block staging mean "
              f"{(s1[:, 1] - s1[:, 0]).mean():.0f}, loop w0 mean {(s1[:, 2] - s1[:, 1]).mean():.0f} max "
              f"{(s1[:, 2] - s1[:, 1]).max()}; block start offsets max {s1[:, 0].max() - t0}")


if __name__ == "__main__":
    main()
