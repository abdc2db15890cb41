"""c2 hybrid probe (GPU): the bench's hybrid_top5 inputs — c2's ALS factors
after a few epochs, random-init towers (d = 64) — through the exact pruned
path (hrec_hybrid_exact_*) and the materialised one, checked bit for bit;
prints per-call times (HIP events, eager and one HIP graph) and how many
32-item groups the bounds left per user.

    python scripts/hx_probe.py [--users 256] [--epochs 2] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-als-twotower-recommender_amd"))
sys.path.insert(0, ROOT)

from src import _hrec, synthetic  # noqa: E402
from src.als_engine import DeviceALS  # noqa: E402
from src.recommend import CapturedRecommend, ShardedRecommender  # noqa: E402
from src.tt_engine import DeviceTwoTower  # noqa: E402


def ev_ms(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def setup(B, epochs, n_users=1_000_000, n_items=100_000, pruned=True):
    """The bench's hybrid_top5 inputs: (recommender, user rows, user vectors)."""
    k, d = 64, 64
    csr = synthetic.generate(n_users, n_items, 0.005, False)
    csc = synthetic.generate(n_users, n_items, 0.005, True)
    eng = DeviceALS(n_users, n_items, k, 0.1, csr, csc)
    eng.init_user_factors(synthetic.SEED_INIT)
    eng.fit(epochs)
    tt = DeviceTwoTower(n_users, n_items, 2651, 255, d, seed=1)
    g = torch.Generator().manual_seed(5)
    items = torch.arange(n_items, dtype=torch.int32)
    man = torch.randint(0, 2651, (n_items,), generator=g, dtype=torch.int32)
    cat = torch.randint(0, 255, (n_items,), generator=g, dtype=torch.int32)
    num = torch.rand((n_items, 2), generator=g).contiguous()
    ivec = tt.item_vectors(items.cuda(), man.cuda(), cat.cuda(), num.cuda())
    Vt = _hrec.transpose(eng.item_factor_rows(0, n_items).contiguous())
    hu_ids = (torch.arange(B, dtype=torch.int64) * (n_users // B)).cuda()
    hu = eng.user_rows(hu_ids)
    uvec = tt.user_vectors(hu_ids.to(torch.int32))
    rec = ShardedRecommender(eng.U, Vt, ivec, 0, k, pruned=pruned)
    rec.materialised = ShardedRecommender(eng.U, Vt, ivec, 0, k, pruned=False)
    return rec, hu, uvec


def analyze(pr, hu, uvec, wins=False, k=5):
    """How many 32-item groups the bounds could leave at best: the groups
    whose upper bound (phase-1 records + E) reaches the FINAL k-th best fused
    score, against the groups the kernel rescored (tau from the seeds)."""
    import numpy as np

    idx, val = pr.recommend(hu, uvec, wins, k)
    hx = pr.last_exact
    B, N, dk = hx.B, hx.N, hx.dk
    G = -(-N // 32)
    r256 = lambda n: -(-n // 256) * 256  # noqa: E731  (hx_layout: uop, uf, uok, then the records)
    off = r256(2 * B * 2 * dk * 2) + r256(2 * B * dk * 4) + r256(B * 4)
    st = hx.ws[off: off + B * G * 16].view(torch.float32).view(B, G, 4).double().cpu().numpy()
    a_mm, t_mm = hx.minmax()
    a_mm, t_mm = a_mm.double().cpu().numpy(), t_mm.double().cpu().numpy()
    U = pr.U[hu][:, :pr.k].double()
    un = torch.linalg.vector_norm(U, dim=1).cpu().numpy()
    tn = torch.linalg.vector_norm(uvec.double(), dim=1).cpu().numpy()
    nrm = hx.items.buf[-256:].view(torch.float32)[:2].double().cpu().numpy()
    Ea, Et = 2.0 ** -13 * un * nrm[0], 2.0 ** -13 * tn * nrm[1]
    w0, w1 = (0.8, 0.2) if wins else (0.2, 0.8)
    ar = np.maximum(a_mm[1] - a_mm[0], 1e-300)
    trr = np.maximum(t_mm[1] - t_mm[0], 1e-30)
    ub = (w0 * (st[:, :, 0] + Ea[:, None] - a_mm[0][:, None]) / ar[:, None]
          + w1 * (st[:, :, 2] + Et[:, None] - t_mm[0][:, None]) / trr[:, None])
    kth = val[:, k - 1].cpu().numpy()
    ideal = (ub >= kth[:, None] - 1e-9).sum(1)
    _, n_top, _ = hx.counts()
    n_top = n_top.cpu().numpy()
    worst = int(np.argmax(n_top))
    return {"live_groups_mean": float(n_top.mean()), "live_groups_max": int(n_top.max()),
            "ideal_groups_mean": float(ideal.mean()), "ideal_groups_max": int(ideal.max()),
            "worst_user": worst, "worst_user_live": int(n_top[worst]), "worst_user_ideal": int(ideal[worst])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n-users", type=int, default=1_000_000)
    ap.add_argument("--n-items", type=int, default=100_000)
    ap.add_argument("--analyze", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    B, n_items = args.users, args.n_items
    pr, hu, uvec = setup(B, args.epochs, args.n_users, n_items)
    mt = pr.materialised
    out = {"users": B, "items": n_items}
    for wins in (False, True):
        a = pr.recommend(hu, uvec, wins, 5)
        b = mt.recommend(hu, uvec, wins, 5)
        same = bool(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]))
        n_ext, n_top, every = pr.last_exact.counts()
        r = {"bit_identical": same, "every_group_rescored": every,
             "groups_extremes": {"mean": float(n_ext.double().mean()), "max": int(n_ext.max())},
             "groups_topk": {"mean": float(n_top.double().mean()), "max": int(n_top.max())},
             "groups_total": -(-n_items // 32)}
        r["pruned_eager_ms"] = ev_ms(lambda: pr.recommend(hu, uvec, wins, 5), args.reps)
        r["materialised_eager_ms"] = ev_ms(lambda: mt.recommend(hu, uvec, wins, 5), args.reps)
        cp = CapturedRecommend(pr, hu, uvec, wins, 5)
        r["pruned_graph_ms"] = ev_ms(lambda: cp(), args.reps)
        cm = CapturedRecommend(mt, hu, uvec, wins, 5)
        r["materialised_graph_ms"] = ev_ms(lambda: cm(), args.reps)
        cp()
        n_ext, n_top, every = pr.last_exact.counts()
        r["after_graph"] = {"every": every, "groups_topk_max": int(n_top.max())}
        out["als_wins" if wins else "tt_wins"] = r
        print(json.dumps({("als_wins" if wins else "tt_wins"): r}), flush=True)
    hx = pr.last_exact
    if args.analyze:
        out["bound_analysis"] = analyze(pr, hu, uvec)
    out["stage_ms"] = {"local (3 launches)": ev_ms(lambda: hx.local(False), args.reps),
                       "minmax (ops + stats + extremes)": ev_ms(lambda: hx.minmax(), args.reps)}
    a_mm, t_mm = hx.minmax()
    out["stage_ms"]["topk (given extremes)"] = ev_ms(lambda: hx.topk(a_mm, t_mm, False), args.reps)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
