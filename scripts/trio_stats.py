"""Diagnostic: producer slot waits and consumer busy share of the trio ALS
half-sweep (HREC_LIB -> a -DHREC_ALS_SPLIT=2 -DHREC_ALS_TRIO_STATS build)."""
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
for side, fn in (("item", eng.item_half_sweep), ("user", eng.user_half_sweep)):
    lib.hrec_debug_als_stamps(buf, 1)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize()
    lib.hrec_debug_als_stamps(buf, 1)
    wait, ptot, busy, ctot, rows = (buf[i] for i in range(5))
    print(f"{side}: {s.elapsed_time(e):.2f} ms; producer wait {100 * wait / max(ptot, 1):.1f}% of producer time; "
          f"consumer busy {100 * busy / max(ctot, 1):.1f}%, {busy / max(rows, 1):.0f} cyc/row, "
          f"producer {ptot / 2048:.0f} cyc/wave, consumer {ctot / 1024:.0f} cyc/wave, rows {rows}")
