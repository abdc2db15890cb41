"""Diagnostics for tests/test_gpu_trained_ranking.py: how far the GPU-trained
two-tower / hybrid scores sit from the oracle-trained ones, relative to the
stated tolerances, and how many users' top-k are decided (no assertions)."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "hybrid-als-twotower-recommender_amd"), ROOT]

import test_gpu_trained_ranking as T  # noqa: E402
from parity_rules import decided_positions  # noqa: E402

from oracle import als as oals  # noqa: E402
from oracle import fusion as ofus  # noqa: E402
from oracle import two_tower as ott  # noqa: E402


def tt_stats(d, epochs=2):
    rng = np.random.default_rng(40 + d)
    df, cat = T.c1_frame(rng)
    tt, p = T._tt_pair(df, (8000, 9964, 2651, 255), d, 256, epochs, seed=d)
    for name in list(ott.DENSE) + ["user_emb", "item_emb", "man_emb", "cat_emb"]:
        a, b = tt.model.tensors[name].cpu().numpy(), p[name]
        bad = np.abs(a - b) > 1e-4 * np.abs(b) + 2e-6
        print(f"  d={d} {name:14s} mismatched {int(bad.sum())}/{a.size} max|diff| {np.abs(a - b).max():.3g}")
    users = np.random.default_rng(3).choice(8000, 64, replace=False)
    ratios, full = [], 0
    for uid in users:
        preds = tt.predict_for_user(int(uid), cat)
        s = np.array([x for _, x in preds], np.float64)
        o, t = T._tt_oracle_scores(tt, p, int(uid), cat)
        ratios.append(np.max(np.abs(s - o) / t))
        rel = np.abs(s - o) / (np.abs(o) + 1e-3)
        _, dec = decided_positions(o, t, 10)
        full += bool(dec.all())
    print(f"  d={d} score err / tol: max {max(ratios):.3g} median {np.median(ratios):.3g}; fully decided {full}/64")


def hybrid_stats(als_wins=True):
    rng = np.random.default_rng(77)
    n_users, n_items = 1500, 1200
    df, cat = T.c1_frame(rng, n_users=n_users, n_items=n_items, per_user=12)
    als, u_ids, i_ids, U, V = T._als_pair(df, 20, 10, seed=5)
    tt, p = T._tt_pair(df, (n_users, n_items, 2651, 255), 50, 256, 1, seed=6)
    known = set(int(i) for i in i_ids)
    cand = cat[cat["itemId"].isin(known)].reset_index(drop=True)
    cand_ids = cand["itemId"].tolist()
    col = np.searchsorted(i_ids, cand["itemId"].to_numpy())
    f1 = (0.5, 0.1) if als_wins else (0.1, 0.5)
    w = (0.8, 0.2) if als_wins else (0.2, 0.8)
    Ug, Vg = als.model.U[:, :20].cpu().numpy(), als.model.V[:, :20].cpu().numpy()
    users = np.random.default_rng(9).choice(len(u_ids), 64, replace=False)
    ra, rt, full, gaps = [], [], 0, []
    for r in users:
        uid = int(u_ids[r])
        a = oals.score_matrix(U[r: r + 1], V[col])[0].astype(np.float64)
        ag = oals.score_matrix(Ug[r: r + 1], Vg[col])[0].astype(np.float64)
        ta = T._als_tol(U[r], V[col])
        ra.append(np.max(np.abs(ag - a) / ta))
        o_t, t_t = T._tt_oracle_scores(tt, p, uid, cand)
        s_t = np.array([x for _, x in tt.predict_for_user(uid, cand)], np.float64)
        rt.append(np.max(np.abs(s_t - o_t) / t_t))
        fused = ofus.adaptive_fusion(list(zip(cand_ids, a.tolist())), list(zip(cand_ids, o_t.astype(np.float32))),
                                     *f1, legacy=True)
        fd = dict(fused)
        o = np.array([fd[i] for i in cand_ids], np.float64)
        t = w[0] * T._minmax_tol(a, ta) + w[1] * T._minmax_tol(o_t, t_t)
        order, dec = decided_positions(o, t, 5)
        full += bool(dec.all())
        gaps.append(np.min(-np.diff(o[order[:6]])) / np.max(t))
    print(f"  hybrid als_wins={als_wins}: ALS err/tol max {max(ra):.3g}; TT err/tol max {max(rt):.3g}; "
          f"fully decided {full}/64; median min-gap/tol {np.median(gaps):.3g}")


if __name__ == "__main__":
    for d in (16, 50):
        tt_stats(d)
    hybrid_stats(True)
    hybrid_stats(False)
