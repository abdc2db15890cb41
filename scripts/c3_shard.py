"""BASELINE configs[2] (c3: 10M users x 1M items, 1% density, rank 64, 8 GPUs)
measured per GPU: rank 0's shard of an 8-way row partition (1.25M user rows,
125k item rows, 2.5e10 ratings, ~200 GB of CSR + CSC) generated on ONE GPU and
swept by the same half-sweep kernel, against the full replicated factor
matrices. Reports per-GPU compute time per epoch and the implied 8-GPU
epochs/s without the all-gathers (their bytes are printed beside)."""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hybrid-als-twotower-recommender_amd"))
from src import _hrec, synthetic  # noqa: E402


def main():
    n_users, n_items, dens, k, W = 10_000_000, 1_000_000, 0.01, 64, 8
    u_per, i_per = math.ceil(n_users / W), math.ceil(n_items / W)
    t0 = time.perf_counter()
    csr = synthetic.generate(n_users, n_items, dens, False, 0, u_per)
    csc = synthetic.generate(n_users, n_items, dens, True, 0, i_per)
    torch.cuda.synchronize()
    print(f"generated rank-0 shard: user nnz {csr.nnz:.3e}, item nnz {csc.nnz:.3e} "
          f"in {time.perf_counter() - t0:.1f} s; device memory used {torch.cuda.memory_allocated() / 1e9:.1f} GB",
          flush=True)
    U = torch.empty((n_users, k), dtype=torch.float32, device="cuda")
    V = torch.empty((n_items, k), dtype=torch.float32, device="cuda")
    _hrec.als_init_factors(synthetic.SEED_INIT, 0, n_users, k, k, U)
    _hrec.als_init_factors(synthetic.SEED_INIT + 1, 0, n_items, k, k, V)
    Vloc = torch.empty((i_per, k), dtype=torch.float32, device="cuda")
    Uloc = torch.empty((u_per, k), dtype=torch.float32, device="cuda")

    def item():
        _hrec.als_half_sweep(csc.indptr, csc.indices, csc.values, U, k, 0.1, Vloc)

    def user():
        _hrec.als_half_sweep(csr.indptr, csr.indices, csr.values, V, k, 0.1, Uloc)

    item()
    user()
    torch.cuda.synchronize()
    reps = 2
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ti = tu = 0.0
    for _ in range(reps):
        e[0].record()
        item()
        e[1].record()
        user()
        e[2].record()
        torch.cuda.synchronize()
        ti += e[0].elapsed_time(e[1]) / reps
        tu += e[1].elapsed_time(e[2]) / reps
    nnz = csr.nnz + csc.nnz
    flops = nnz * (k * (k + 1) + 2 * k) + (u_per + i_per) * (k ** 3 / 3 + 2 * k * k)
    ep = (ti + tu) / 1e3
    print(f"c3 rank-0 shard of {W}: item half-sweep {ti:.1f} ms, user half-sweep {tu:.1f} ms, "
          f"{flops / ep / 1e12:.1f} TFLOP/s algorithmic = {flops / ep / 1e12 / 78.6:.3f} of f64 MFMA peak; "
          f"8-GPU compute-only bound {1 / ep:.3f} epochs/s; all-gathers per epoch "
          f"{(n_users + n_items) * k * 4 / 1e9:.2f} GB replicated", flush=True)


if __name__ == "__main__":
    main()
