"""Timing probe of hrec_dot_filter at the c5 shape (run under rocprofv3
--kernel-trace --stats): no survivors, per-user bounds at the 99.9th
percentile, per-group bounds, clustered survivors.

python scripts/filter_probe.py [--users 256] [--items 100000] [--d 256]
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
    S = _hrec.dot_scores(Ub, Vb)
    q = torch.quantile(S[:, :20000], 0.999, dim=1)
    cases = {"none": torch.full((a.users,), float("inf"), device="cuda"), "q999": q}
    for name, thr in cases.items():
        for _ in range(a.reps):
            _, _, cn = _hrec.dot_filter(Ub, Vb, thr, 0)
        torch.cuda.synchronize()
        print(name, "survivors/user", float(cn.double().mean()))
    per = 784
    G = (a.items + per - 1) // per
    thr = q[:, None].expand(a.users, G).contiguous()
    for _ in range(a.reps):
        _, _, cn = _hrec.dot_filter(Ub, Vb, thr, per)
    torch.cuda.synchronize()
    print("group survivors/user", float(cn.double().mean()))


if __name__ == "__main__":
    main()
