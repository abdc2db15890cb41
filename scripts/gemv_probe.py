"""Timing probe of hrec_dot_scores / hrec_dot_topk for 1-4 users (the GEMV,
csrc/dot_gemv.hip) at BASELINE c4 (50M x 128 f32); HREC_LIB picks a variant."""
import os
import sys

import torch

sys.path.insert(0, "hybrid-als-twotower-recommender_amd")
from src import _hrec as h  # noqa: E402


def t_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


N = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
g = torch.Generator(device="cuda").manual_seed(0)
for d in (128, 64, 256):
    n = N if d <= 128 else N // 2
    V = torch.randn((n, d), device="cuda", generator=g)
    U = torch.randn((4, d), device="cuda", generator=g)
    for B in (1, 4):
        Ub = U[:B].contiguous()
        out = torch.empty((B, n), device="cuda")
        ms = t_ms(lambda: h.dot_scores(Ub, V))
        mk = t_ms(lambda: h.dot_topk(Ub, V, 5))
        print(f"{os.path.basename(os.environ.get('HREC_LIB', 'default'))} d={d} B={B} N={n}: scores {ms:.3f} ms "
              f"({n * d * 4 / ms / 1e6:.0f} GB/s)  topk5 {mk:.3f} ms ({n * d * 4 / mk / 1e6:.0f} GB/s)", flush=True)
    del V
    torch.cuda.empty_cache()
