"""Kernel-shape probe (GPU, run under rocprofv3 --kernel-trace --stats):
dot_scores / dot_topk at one (B, N, dk) with random bf16 operands.

python scripts/dot_shape_probe.py [--users 256] [--items 100000] [--d 256]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-als-twotower-recommender_amd"))

from src import _hrec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=256)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    U = torch.randn(a.users, a.d, device="cuda", generator=g)
    V = torch.randn(a.items, a.d, device="cuda", generator=g)
    Ub, Vb = _hrec.dot_operand(U, torch.bfloat16), _hrec.dot_operand(V, torch.bfloat16)
    for _ in range(a.reps):
        _hrec.dot_scores(Ub, Vb)
    for _ in range(a.reps):
        _hrec.dot_topk(Ub, Vb, 5)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
