"""Timing probe: one ALS epoch at c2 (1M x 100k, 0.5 %) for a given rank."""
import sys
import time

import torch

sys.path.insert(0, "hybrid-als-twotower-recommender_amd")
from src import synthetic  # noqa: E402
from src.als_engine import DeviceALS  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    users = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    items = int(sys.argv[3]) if len(sys.argv) > 3 else 100_000
    dens = 0.005
    csr = synthetic.generate(users, items, dens, False)
    csc = synthetic.generate(users, items, dens, True)
    eng = DeviceALS(users, items, k, 0.1, csr, csc)
    eng.init_user_factors(synthetic.SEED_INIT)
    eng.epoch()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record(s)
    eng.item_half_sweep()
    e[1].record(s)
    eng.user_half_sweep()
    e[2].record(s)
    torch.cuda.synchronize()
    it, ut = e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2])
    nnz = csr.nnz
    fl = 2 * (nnz * (k * (k + 1) + 2 * k)) + (users + items) * (k ** 3 / 3 + 2 * k * k)
    print(f"rank {k}: item {it:.1f} ms, user {ut:.1f} ms, epoch {it + ut:.1f} ms = {1e3 / (it + ut):.2f} epochs/s, "
          f"{fl / (it + ut) / 1e9:.1f} TFLOP/s algorithmic ({fl / (it + ut) / 1e9 / 78.6:.2f} of f64 peak)", flush=True)


if __name__ == "__main__":
    main()
