"""Diagnostic: per-phase cycles of the rank-k wide half-sweep (HREC_WIDE_STAMPS
build at lib/variants/libhrec_stamps.so; wave 0 of every block, s_memtime)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["HREC_LIB"] = os.path.join(ROOT, "hybrid-als-twotower-recommender_amd", "lib", "variants", "libhrec_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "hybrid-als-twotower-recommender_amd"))
from src import _hrec, synthetic  # noqa: E402
from src.als_engine import DeviceALS  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    users, items = 100_000, 100_000
    csr = synthetic.generate(users, items, 0.005, False)
    csc = synthetic.generate(users, items, 0.005, True)
    eng = DeviceALS(users, items, k, 0.1, csr, csc)
    eng.init_user_factors(synthetic.SEED_INIT)
    lib = _hrec.lib()
    buf = (ctypes.c_ulonglong * 8)()
    fn = lib.hrec_debug_wide_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    eng.item_half_sweep()
    torch.cuda.synchronize()
    fn(buf, 1)
    for name, sweep, n in (("item", eng.item_half_sweep, items), ("user", eng.user_half_sweep, users)):
        sweep()
        torch.cuda.synchronize()
        fn(buf, 1)
        v = [buf[i] / n for i in range(8)]
        tot = sum(v)
        print(f"rank {k} {name}: cycles/row (s_memtime ticks) " +
              " ".join(f"{lbl}={x:.0f}" for lbl, x in zip(["gram", "trail+write", "panel", "p2tail", "xstore", "bs_chain", "bs_update", "bs_barrier"], v)) +
              f" total={tot:.0f}", flush=True)


if __name__ == "__main__":
    main()
