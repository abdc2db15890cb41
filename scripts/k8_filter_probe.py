"""K8 bf16 filter (hrec_dot_filter) at the scoring shape (1024 users x 100k
items, dk 64): time vs the bound, to separate the GEMM from the survivor
appends."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hybrid-als-twotower-recommender_amd"))
from src import _hrec  # noqa: E402

B, N, dk = 1024, 100_000, 64
g = torch.Generator(device="cuda").manual_seed(3)
U = _hrec.dot_operand(torch.randn(B, dk, device="cuda", generator=g), torch.bfloat16, dk)
V = _hrec.dot_operand(torch.randn(N, dk, device="cuda", generator=g), torch.bfloat16, dk)
sc = _hrec.dot_scores(U, V)
for q in (None, 0.9999, 0.999, 0.9975, 0.99):
    if q is None:
        thr = torch.full((B,), 1e30, device="cuda")
    else:
        thr = torch.quantile(sc[:, :16384].float(), q, dim=1).contiguous()
    for _ in range(2):
        r = _hrec.dot_filter(U, V, thr, cap=4096)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        r = _hrec.dot_filter(U, V, thr, cap=4096)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    n = r[2].float() if len(r) > 2 else None
    print(f"q {q}: {ms * 1e3:7.1f} us  survivors/user mean {float(n.mean()) if n is not None else -1:.1f}", flush=True)
