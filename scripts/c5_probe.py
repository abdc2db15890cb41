"""BASELINE c5's pruned hybrid batch alone (the bench's data: rank-256 ALS
factors from hrec_als_init_factors, a d = 256 two-tower on c2's tables; 256
users x 100k items): HIP-event time per one-shard call (both phases), for
kernel traces / PMC passes of just these launches."""
import sys

import torch

sys.path.insert(0, "hybrid-als-twotower-recommender_amd")
from src import _hrec, synthetic  # noqa: E402
from src.recommend import ShardedRecommender  # noqa: E402
from src.tt_engine import DeviceTwoTower  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n_users, n_items, k5, d5, B5 = 1_000_000, 100_000, 256, 256, 256
torch.cuda.set_device(0)
U5 = torch.zeros((n_users, k5), dtype=torch.float32, device="cuda")
_hrec.als_init_factors(synthetic.SEED_INIT, 0, n_users, k5, k5, U5)
V5 = torch.zeros((n_items, k5), dtype=torch.float32, device="cuda")
_hrec.als_init_factors(synthetic.SEED_INIT + 1, 0, n_items, k5, k5, V5)
tt5 = DeviceTwoTower(n_users, n_items, 2651, 255, d5, seed=2)
g5 = torch.Generator().manual_seed(6)
items5 = torch.arange(0, n_items, dtype=torch.int32)
man5 = torch.randint(0, 2651, (n_items,), generator=g5, dtype=torch.int32)
cat5 = torch.randint(0, 255, (n_items,), generator=g5, dtype=torch.int32)
num5 = torch.rand((n_items, 2), generator=g5).contiguous()
iv5 = tt5.item_vectors(items5.cuda(), man5.cuda(), cat5.cuda(), num5.cuda())
rec5 = ShardedRecommender(U5, None, iv5, 0, k5, precision="bf16", V_local=V5)
hu5 = (torch.arange(B5, dtype=torch.int64) * (n_users // B5)).cuda()
uv5 = tt5.user_vectors(hu5.to(torch.int32))
for _ in range(3):
    i, v = rec5.recommend(hu5, uv5, False, 5)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    rec5.recommend(hu5, uv5, False, 5)
e.record()
torch.cuda.synchronize()
sv = rec5.last_prune.survivors().double()
q = torch.quantile(sv.cpu(), torch.tensor([0.5, 0.9, 0.99], dtype=torch.float64)).tolist()
print(f"c5 batch {s.elapsed_time(e) / reps * 1e3:.1f} us, fallback {rec5.last_prune.fallback_taken()}, "
      f"survivors mean {sv.mean().item():.0f} (p50 {q[0]:.0f}, p90 {q[1]:.0f}, p99 {q[2]:.0f}, "
      f"max {sv.max().item():.0f})", flush=True)
