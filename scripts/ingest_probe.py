"""Ingest step timings at the bench's c2 shape (GPU): encode_ids x2, the
CSR build (sorted-rows path) and the CSC build (the stable sort), each timed
on its own with HIP events.

python scripts/ingest_probe.py [--users 1000000] [--items 100000] [--density 0.005]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-als-twotower-recommender_amd"))

from src import _hrec, synthetic  # noqa: E402
from src.als_engine import RowLayout  # noqa: E402


def ev(fn, reps=3):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        out = fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--density", type=float, default=0.005)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    lay = RowLayout.equal(a.users, 1, 1)
    csr = synthetic.generate_layout(a.users, a.items, a.density, False, lay, 0)
    counts = csr.indptr[1:] - csr.indptr[:-1]
    uid = torch.repeat_interleave(torch.arange(a.users, dtype=torch.int64, device="cuda"), counts)
    iid = csr.indices.to(torch.int64)
    vals = csr.values
    nnz = int(csr.nnz)
    print("nnz", nnz)
    t, (_, urow, u_ord, u_ptr) = ev(lambda: _hrec.encode_ids(uid, (0, a.users - 1), order=True))
    print("encode users ms %.3f  (%.1f GB/s at 12 B/rating)" % (t, 12 * nnz / t / 1e6))
    t, (iu, irow, i_ord, _) = ev(lambda: _hrec.encode_ids(iid, (0, a.items - 1), order=True))
    print("encode items ms %.3f" % t)
    t, _ = ev(lambda: _hrec.coo_to_csr(urow, irow, vals, a.users, alias=True, rows_in_order=u_ord, indptr=u_ptr))
    print("csr (sorted rows, the codes aliased) ms %.3f" % t)
    t, out = ev(lambda: _hrec.coo_to_csr(irow, urow, vals, int(iu.numel()), rows_in_order=i_ord))
    print("csc (stable sort) ms %.3f  (%.1f GB/s at 20 B/rating)" % (t, 20 * nnz / t / 1e6))


if __name__ == "__main__":
    main()
