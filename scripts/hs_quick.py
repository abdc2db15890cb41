"""Quick timing of the c5 score stage: hrec_hybrid_scores vs the old
dot_scores x2 + rows_minmax x2 (HIP events), at c5's shape (256 users x 100k
items, rank 256 / d 256, bf16). HREC_LIB selects a variant build."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hybrid-als-twotower-recommender_amd"))
from src import _hrec as h  # noqa: E402

B, N, dk = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 100_000, 256
g = torch.Generator(device="cuda").manual_seed(0)
U = torch.randn((1_000_000 if B <= 4096 else B, dk), device="cuda", generator=g) / 16
uv = torch.randn((B, dk), device="cuda", generator=g) / 16
va = h.dot_operand(torch.randn((N, dk), device="cuda", generator=g) / 16, torch.bfloat16)
vt = h.dot_operand(torch.randn((N, dk), device="cuda", generator=g) / 16, torch.bfloat16)
rows = torch.randint(0, U.shape[0], (B,), device="cuda", generator=g)


def t(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def old():
    ua = h.dot_operand(U.index_select(0, rows), torch.bfloat16, dk)
    ut = h.dot_operand(uv, torch.bfloat16, dk)
    a, b = h.dot_scores(ua, va), h.dot_scores(ut, vt)
    return h.rows_minmax(a), h.rows_minmax(b)


us_new = t(lambda: h.hybrid_scores(U, rows, uv, va, vt))
us_old = t(old)
gb = (2 * 4.0 * B * N + 2 * 2.0 * dk * N) / 1e9
print(f"B={B}: hybrid_scores {us_new:.1f} us ({gb / us_new * 1e6 / 1e3:.2f} TB/s, "
      f"{4.0 * dk * B * N / us_new / 1e6:.0f} TF/s); old chain {us_old:.1f} us")
