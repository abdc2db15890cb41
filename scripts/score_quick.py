"""Timing probe of hrec_als_score_topk (JVM-exact ALS scoring + top-5) at the
bench's c2 size: 1024 users x 100k items, rank 64."""
import sys

import torch

sys.path.insert(0, "hybrid-als-twotower-recommender_amd")
from src import _hrec as h  # noqa: E402


def t_ms(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    n_users, n_items, k = 1_000_000, 100_000, 64
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    g = torch.Generator(device="cuda").manual_seed(0)
    U = torch.randn((n_users, k), device="cuda", generator=g) * 0.3
    V = torch.randn((n_items, k), device="cuda", generator=g) * 0.3
    Vt = h.transpose(V)
    users = torch.arange(B, dtype=torch.int64, device="cuda") * (n_users // B)
    ms = t_ms(lambda: h.als_score_topk(U, users, Vt, n_items, k, 5, check_overflow=False))
    ms2 = t_ms(lambda: h.als_score_topk(U, users, Vt, n_items, k, 5))
    print(f"score_topk B={B}: {ms*1e3:.1f} us/batch (no host sync), {ms2*1e3:.1f} us with overflow check, "
          f"{B*n_items/ms/1e9:.3e} pairs/s x1e12->, VALU {B*n_items*2*k/ms/1e9/78.6:.3f} of 78.6", flush=True)
    i, v = h.als_score_topk(U, users, Vt, n_items, k, 5)
    s = h.als_score(U, users, Vt, None, n_items, k)
    i2, v2 = h.topk(s, 5)
    assert torch.equal(i, i2) and torch.equal(v, v2), "score_topk != full scores + topk"
    print("score-quick-ok", flush=True)


if __name__ == "__main__":
    main()
