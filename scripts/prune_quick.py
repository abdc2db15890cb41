"""Timing probe of hrec_als_score_topk_pruned (the bench's scoring line: 1024
users x 100k items, rank 64, top-5) with a per-kernel split from HIP events
around the whole call; HREC_LIB picks a variant build."""
import os
import sys

import torch

sys.path.insert(0, "hybrid-als-twotower-recommender_amd")
from src import _hrec as h  # noqa: E402


def t_ms(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


n_users, n_items, k = 1_000_000, 100_000, 64
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
g = torch.Generator(device="cuda").manual_seed(0)
U = torch.randn((n_users, k), device="cuda", generator=g) * 0.3
V = torch.randn((n_items, k), device="cuda", generator=g) * 0.3
Vt = h.transpose(V)
ops = h.als_items_bf16(V, k)
users = torch.arange(B, dtype=torch.int64, device="cuda") * (n_users // B)
ws = torch.empty(int(h.lib().hrec_als_score_topk_pruned_workspace_bytes(B, n_items, 5, k)), dtype=torch.uint8,
                 device="cuda")
flag = torch.zeros(1, dtype=torch.int32, device="cuda")
f = lambda: h.als_score_topk_pruned(U, users, Vt, V, ops, n_items, k, 5, check_overflow=False,  # noqa: E731
                                    overflow_out=flag, workspace=ws)
for _ in range(3):
    ms = t_ms(f)
    print(f"{os.path.basename(os.environ.get('HREC_LIB', 'default'))} pruned B={B}: {ms * 1e3:.1f} us/batch "
          f"({B * n_items / ms / 1e9:.3e} pairs/s)", flush=True)
i, v = f()
i2, v2 = h.als_score_topk(U, users, Vt, n_items, k, 5)
assert int(flag.item()) == 0 and torch.equal(i, i2) and torch.equal(v, v2), "pruned != fused"
print("prune-quick-ok", flush=True)

# the bench's call: overflow checked on the host after every batch (one sync per call)
import time  # noqa: E402


def wall(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


f_sync = lambda: h.als_score_topk_pruned(U, users, Vt, V, ops, n_items, k, 5, workspace=ws)  # noqa: E731
print(f"checked call (host sync each): {wall(f_sync) * 1e3:.1f} us; unchecked: {wall(f) * 1e3:.1f} us", flush=True)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    f()
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    gi, gv = f()
def f_graph():  # noqa: E302
    g.replay()
    return int(flag.item())
print(f"graph replay + flag check: {wall(f_graph) * 1e3:.1f} us", flush=True)
assert torch.equal(gi, i2) and torch.equal(gv, v2)
