"""Diagnostic: per-phase cycle shares of the ALS half-sweep (stamped build).
Run with HREC_LIB pointing at a -DHREC_ALS_STAMPS build."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hybrid-als-twotower-recommender_amd"))
from src import _hrec, synthetic  # noqa: E402
from src.als_engine import DeviceALS  # noqa: E402

lib = _hrec.lib()
lib.hrec_debug_als_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()
n_users, n_items = 1_000_000, 100_000
csr = synthetic.generate(n_users, n_items, 0.005, False)
csc = synthetic.generate(n_users, n_items, 0.005, True)
eng = DeviceALS(n_users, n_items, 64, 0.1, csr, csc)
eng.init_user_factors(7)
eng.epoch()
torch.cuda.synchronize()
names = ["gramian", "b+layout", "factor", "solves", "-", "-", "-"]
for side, fn, rows in (("item", eng.item_half_sweep, n_items), ("user", eng.user_half_sweep, n_users)):
    lib.hrec_debug_als_stamps(buf, 1)
    fn()
    torch.cuda.synchronize()
    lib.hrec_debug_als_stamps(buf, 1)
    tot = sum(buf[i] for i in range(7))
    print(side, " ".join(f"{names[i]}={buf[i] / rows:.0f}cyc({100 * buf[i] / max(tot, 1):.0f}%)"
                         for i in range(7) if names[i] != "-"))
