"""c4 B = 1 (the reference's one-user call): hrec_dot_topk of one user over
50M x 128 items, f32 and bf16, HIP-event time per call and the HBM rate of
the item operand read once; HREC_LIB selects a variant build."""
import sys

import torch

sys.path.insert(0, "hybrid-als-twotower-recommender_amd")
from src import _hrec as h  # noqa: E402

N, d = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000, 128
g = torch.Generator(device="cuda").manual_seed(0)
V = torch.randn((N, d), device="cuda", generator=g)
U = torch.randn((4, d), device="cuda", generator=g)
for dt in (torch.float32, torch.bfloat16):
    Vd = h.dot_operand(V, dt)
    for B in (1, 2, 4):
        Ud = h.dot_operand(U[:B].contiguous(), dt)
        h.dot_topk(Ud, Vd, 5)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            h.dot_topk(Ud, Vd, 5)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        gb = N * d * Vd.element_size() / 1e9
        print(f"{str(dt)[6:]:9s} B={B}: {ms:.3f} ms  {gb / ms:.2f} TB/s  frac {gb / ms / 8:.3f}", flush=True)
    del Vd
    torch.cuda.empty_cache()
