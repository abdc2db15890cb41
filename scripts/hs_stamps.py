"""Diagnostic: phase split of the c5 GEMM launches (hyb_scores_kernel modes
HS_PRUNE and HS_FILTER) from a -DHREC_HS_STAMPS build (HREC_LIB): the last
launch's per-block s_memtime stamps (wave 0: entry, staged, main loop done,
end) and every wave's main-loop ticks; block start spread and percentiles."""
import ctypes
import runpy
import sys

import numpy as np

sys.argv = ["c5_probe.py", "1"]
sys.path.insert(0, "hybrid-als-twotower-recommender_amd")
from src import _hrec  # noqa: E402

lib = _hrec.lib()
lib.hrec_debug_hs_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
runpy.run_path("scripts/c5_probe.py", run_name="__main__")
buf = np.zeros((3, 1024, 8), np.uint64)
lib.hrec_debug_hs_stamps(buf.ctypes.data, 0)
for mode, name in ((1, "HS_PRUNE (phase 1)"), (2, "HS_FILTER (pass 2b)")):
    b = buf[mode].astype(np.int64)
    b = b[b[:, 0] > 0]
    t0 = b[:, 0].min()
    st, lp, ep = b[:, 1] - b[:, 0], b[:, 2] - b[:, 1], b[:, 3] - b[:, 2]
    wl = np.concatenate([(b[:, 4 + q] & 0xffffffff, b[:, 4 + q] >> 32) for q in range(4)])
    q = lambda x: "p10 %6d  p50 %6d  p90 %6d" % tuple(np.percentile(x, [10, 50, 90]))  # noqa: E731
    print(f"{name}: {len(b)} blocks; kernel span {b[:, 3].max() - t0} ticks; block start spread "
          f"{b[:, 0].max() - t0}\n  staging   {q(st)}\n  loop w0   {q(lp)}\n  epilogue  {q(ep)}\n  loop (all waves) {q(wl)}",
          flush=True)

# hp_bound_kernel / hp_cand_topk_kernel (-DHREC_HP_STAMPS): per block, ticks
# between its phase points
if hasattr(lib, "hrec_debug_hp_stamps"):
    lib.hrec_debug_hp_stamps.argtypes = [ctypes.c_void_p]
    hp = np.zeros((2, 1024, 8), np.uint64)
    lib.hrec_debug_hp_stamps(hp.ctypes.data)
    for kid, name, pts in ((0, "hp_bound", ["extremes", "setup", "slots", "seed MFMAs", "tau", "theta"]),
                           (1, "hp_cand_topk", ["loads", "survivors", "merge", "-", "-", "end"])):
        t = hp[kid].astype(np.int64)
        t = t[t[:, 0] > 0]
        print(f"{name}: {len(t)} blocks, span {t[:, 7].max() - t[:, 0].min()} ticks, block start spread "
              f"{t[:, 0].max() - t[:, 0].min()}")
        prev = t[:, 0]
        for i, nm in enumerate(pts, start=1):
            cur = np.where(t[:, i] > 0, t[:, i], prev)
            d = cur - prev
            print(f"  -> {nm:12s} p50 {np.percentile(d, 50):7.0f}  p90 {np.percentile(d, 90):7.0f}")
            prev = cur
        d = t[:, 7] - prev
        print(f"  -> {'(to end)':12s} p50 {np.percentile(d, 50):7.0f}  p90 {np.percentile(d, 90):7.0f}")
