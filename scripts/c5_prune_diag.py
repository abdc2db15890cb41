"""c5 pruned-hybrid diagnostics (GPU): how many items survive the heavy-model
filter of hrec_hybrid_prune_topk on the bench's c5 data, against what an
exact-tau heavy-only filter would keep and how crowded the fused top is.

python scripts/c5_prune_diag.py [--users 256] [--items 100000]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-als-twotower-recommender_amd"))
sys.path.insert(0, ROOT)

from src import _hrec, synthetic  # noqa: E402
from src.recommend import ShardedRecommender  # noqa: E402
from src.tt_engine import DeviceTwoTower  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=256)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--n-users", type=int, default=1_000_000)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    k5 = d5 = 256
    n_users, n_items = a.n_users, a.items
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
    rec = ShardedRecommender(U5, None, iv5, 0, k5, precision="bf16", V_local=V5)
    B = a.users
    hu = (torch.arange(B, dtype=torch.int64) * (n_users // B)).cuda()
    uv = tt5.user_vectors(hu.to(torch.int32))
    o = rec.ops
    hp = o.hybrid_prune(rec.U, hu, uv, rec.V_op, rec.iv_op, 5)
    a_mm, t_mm = hp.minmax()
    hp.topk(a_mm, t_mm, False, 0)
    surv = hp.survivors().double()
    print("fallback_taken", hp.fallback_taken())
    print("survivors/user mean %.1f median %.1f max %.0f min %.0f" % (
        surv.mean(), surv.median(), surv.max(), surv.min()))
    als, tt, am, tm = o.hybrid_scores(rec.U, hu, uv, rec.V_op, rec.iv_op)
    als, tt = als.double(), tt.double()
    an = (als - als.min(1, keepdim=True).values) / (als.max(1, keepdim=True).values - als.min(1, keepdim=True).values)
    tn = (tt - tt.min(1, keepdim=True).values) / (tt.max(1, keepdim=True).values - tt.min(1, keepdim=True).values)
    f = 0.2 * an + 0.8 * tn
    f5 = f.topk(5, dim=1).values[:, -1:]
    ideal = (0.8 * tn + 0.2 >= f5).sum(1).double()
    print("exact-tau heavy-only filter: mean %.1f max %.0f" % (ideal.mean(), ideal.max()))
    for eps in (0.0, 0.01, 0.05, 0.1):
        c = (f >= f5 - eps).sum(1).double()
        print("fused >= f5-%.2f: mean %.1f" % (eps, c.mean()))
    for q in (0.5, 0.9, 0.99, 0.999):
        print("tn quantile %.3f: %.4f" % (q, torch.quantile(tn[:16].flatten().float(), q)))
    print("an at fused top-5 mean %.3f; tn at fused top-5 mean %.3f" % (
        an.gather(1, f.topk(5, 1).indices).mean(), tn.gather(1, f.topk(5, 1).indices).mean()))
    # per-group light max bound: groups of the hs slice layout are not exposed;
    # emulate 128 contiguous groups
    G = 128
    gs = (n_items + G - 1) // G
    anp = torch.nn.functional.pad(an, (0, G * gs - n_items), value=0.0).view(B, G, gs).max(2).values
    lb = anp.repeat_interleave(gs, 1)[:, :n_items]
    grp = (0.8 * tn + 0.2 * lb >= f5).sum(1).double()
    print("exact tau + per-group(%d) light max: mean %.1f max %.0f" % (G, grp.mean(), grp.max()))
    # the bound kernel's theta [B][G] (workspace after part / argpos / uop,
    # each rounded to 256 B: csrc/hybrid_prune.hip hp_layout)
    Gk = min(max((n_items + 255) // 256, 1), 128)
    r256 = lambda x: (x + 255) // 256 * 256  # noqa: E731
    off = r256(2 * Gk * 2 * B * 4) + r256(2 * Gk * B * 4) + r256(2 * B * rec.V_op.shape[1] * 2)
    th = hp.ws[off: off + B * Gk * 4].view(torch.float32).view(B, Gk)
    live = torch.isfinite(th)
    print("theta live (user, group) pairs %d of %d (%.2f%%); live groups/user mean %.1f max %d" % (
        live.sum(), B * Gk, 100.0 * live.float().mean(), live.sum(1).float().mean(), live.sum(1).max()))
    ch = live.view(-1, 64, Gk).any(1) if B % 64 == 0 else None
    if ch is not None:
        print("live (64-user chunk, group) tiles %d of %d" % (ch.sum(), ch.numel()))
    print("groups live for any user %d of %d" % (live.any(0).sum(), Gk))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        hp.topk(a_mm, t_mm, False, 0)
    torch.cuda.synchronize()
    print("topk ms %.3f" % ((time.perf_counter() - t0) / 20 * 1e3))


if __name__ == "__main__":
    main()
