"""GPU parity of the exact hybrid top-k without score matrices
(csrc/hybrid_exact.hip, hrec_hybrid_exact_*) — get_hybrid_recommendations
(/root/reference/src/hybrid_system.py:57-75, :95-116) for a batch of users at
the reference's numerics: the JVM-exact ALS dot (Spark ALSModel.transform,
src/als_model.py:75) and the f32 Keras Dot (src/two_tower_model.py:80).

Tolerance: BIT-EXACT. Every assertion compares ids, fused f64 scores and both
models' [min; max] rows with torch.equal (NaN positions with
np.testing.assert_array_equal) against the materialised path the recommender
used before — hrec_als_score + hrec_tt_score + hrec_rows_minmax_f32 +
hrec_fuse_rows_topk — on the same inputs. The pruned path only decides WHICH
items are scored exactly; every score it ranks is computed by the same
arithmetic, so nothing weaker than bit equality is acceptable.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _h():
    from src import _hrec

    return _hrec


def _kp(k):
    return 64 if k <= 64 else 128


def _case(device, B, N, ka, kt, seed, n_users=None, same_items=False, tt_scale=0.25):
    rng = np.random.default_rng(seed)
    n_users = n_users or B + 7
    kp = _kp(ka)
    U = np.zeros((n_users, kp), np.float32)
    U[:, :ka] = rng.normal(size=(n_users, ka))
    V = np.zeros((N, kp), np.float32)
    V[:, :ka] = np.tile(rng.normal(size=(1, ka)), (N, 1)) if same_items else rng.normal(size=(N, ka))
    iv = rng.normal(size=(N, kt)).astype(np.float32)
    uv = (rng.normal(size=(B, kt)) * tt_scale).astype(np.float32)
    rows = rng.integers(0, n_users, B)
    t = lambda x: torch.as_tensor(x, device=device)  # noqa: E731
    return t(U), t(V), t(iv), t(uv), t(rows.astype(np.int64))


def _materialised(h, U, rows, Vt, N, ka, uv, iv, wins, k, offset=0):
    als = h.als_score(U, rows, Vt, None, N, ka)
    tt = h.tt_score(uv, iv)
    a_mm, t_mm = h.rows_minmax(als), h.rows_minmax(tt)
    ei, ev = h.fuse_rows_topk(als, tt, a_mm, t_mm, wins, k, offset)
    return ei, ev, a_mm, t_mm


def _same(x, y):
    np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())  # NaN == NaN position-wise


@pytest.mark.parametrize("B,N,ka,kt,k", [(256, 100_003, 64, 64, 5), (70, 20_000, 50, 32, 8), (130, 40_001, 100, 128, 1),
                                         (33, 5_000, 10, 64, 3), (300, 777, 64, 64, 5), (8, 9, 64, 64, 8),
                                         (8, 1, 64, 64, 5), (40, 33, 16, 32, 4),
                                         # G > 8192 groups (records read from memory, not LDS)
                                         (16, 300_007, 64, 64, 5),
                                         # batches of < 8 users (hrec_tt_score's GEMV: the same bits)
                                         (3, 50_000, 32, 32, 2), (1, 30_000, 64, 64, 5), (2, 20_000, 16, 32, 1),
                                         (4, 40_000, 64, 128, 3), (7, 25_000, 100, 64, 8)])
def test_hybrid_exact_equals_materialised(device, B, N, ka, kt, k):
    """K9x == the materialised exact path bit for bit — ids, fused scores and
    both min / max rows — for both weight orders, through the two-phase calls
    (the multi-shard sequence) and the one-shard call; on random data no user
    rescored every group."""
    h = _h()
    U, V, iv, uv, rows = _case(device, B, N, ka, kt, B * 3 + N)
    Vt = h.transpose(V)
    items = h.HybridExactItems(Vt, N, ka, iv)
    for wins in (True, False):
        ei, ev, ea, et = _materialised(h, U, rows, Vt, N, ka, uv, iv, wins, k, 11)
        hx = h.HybridExact(U, rows, uv, items, k)
        a_mm, t_mm = hx.minmax()
        assert torch.equal(a_mm, ea) and torch.equal(t_mm, et)
        gi, gv = hx.topk(a_mm, t_mm, wins, 11)
        assert torch.equal(gi, ei), (wins, (gi != ei).nonzero()[:5])
        assert torch.equal(gv, ev)
        li, lv, la, lt = hx.local(wins, 11)
        assert torch.equal(li, ei) and torch.equal(lv, ev)
        assert torch.equal(la, ea) and torch.equal(lt, et)
        n_ext, n_top, every = hx.counts()
        if N >= 1000:
            assert not every
            G = -(-N // 32)
            # the bounds decide: a minority of the groups per user, not the shard
            mt, me = float(n_top.double().mean()), float(n_ext.double().mean())
            assert mt < G / 4 and me < G / 4, (mt, me, G)


def test_hybrid_exact_fallback_cases(device):
    """Users the bounds cannot help — every ALS item identical (all fused
    scores tie on the ALS side), an unknown ALS row (NaN scores: the first k
    items, NaN values), a NaN two-tower vector, a huge user vector (no bound:
    every group rescored) — get the materialised path's bits."""
    h = _h()
    B, N, ka, kt = 40, 30_000, 64, 64
    U, V, iv, uv, rows = _case(device, B, N, ka, kt, 12, n_users=60, same_items=True)
    uv_bad = uv.clone()
    uv_bad[5, 3] = float("nan")
    uv_huge = uv.clone()
    uv_huge[7] *= 1e30
    rows_bad = rows.clone()
    rows_bad[3] = -1
    Vt = h.transpose(V)
    items = h.HybridExactItems(Vt, N, ka, iv)
    for r, u, wins in ((rows, uv, True), (rows_bad, uv, True), (rows_bad, uv_bad, False), (rows, uv_huge, False)):
        ei, ev, ea, et = _materialised(h, U, r, Vt, N, ka, u, iv, wins, 5)
        hx = h.HybridExact(U, r, u, items, 5)
        a_mm, t_mm = hx.minmax()
        _same(a_mm, ea)
        _same(t_mm, et)
        gi, gv = hx.topk(a_mm, t_mm, wins)
        assert torch.equal(gi, ei)
        _same(gv, ev)
        li, lv, _, _ = hx.local(wins)
        assert torch.equal(li, ei)
        _same(lv, ev)


def test_hybrid_exact_ties_and_duplicates(device):
    """Items repeated across group boundaries (equal fused scores: ties ->
    the smaller item id) and a constant two-tower side (range 0 -> scale 1)."""
    h = _h()
    rng = np.random.default_rng(5)
    B, N, ka, kt = 24, 4_000, 64, 64
    base = rng.normal(size=(50, ka)).astype(np.float32)
    V = np.zeros((N, 64), np.float32)
    V[:, :ka] = base[rng.integers(0, 50, N)]
    iv = np.tile(rng.normal(size=(1, kt)).astype(np.float32), (N, 1))
    U = np.zeros((B, 64), np.float32)
    U[:, :ka] = rng.normal(size=(B, ka))
    uv = rng.normal(size=(B, kt)).astype(np.float32)
    t = lambda x: torch.as_tensor(x, device=device)  # noqa: E731
    U, V, iv, uv = t(U), t(V), t(iv), t(uv)
    rows = torch.arange(B, device=device)
    items = h.HybridExactItems(h.transpose(V), N, ka, iv)
    for wins in (True, False):
        ei, ev, _, _ = _materialised(h, U, rows, h.transpose(V), N, ka, uv, iv, wins, 8)
        hx = h.HybridExact(U, rows, uv, items, 8)
        li, lv, _, _ = hx.local(wins)
        assert torch.equal(li, ei) and torch.equal(lv, ev)


def test_recommender_exact_paths_agree(device):
    """ShardedRecommender precision "exact": pruned (default for >= 8 users)
    and materialised (pruned=False) give the same ids and scores, eagerly and
    replayed as one HIP graph."""
    from src import _hrec
    from src.recommend import CapturedRecommend, ShardedRecommender

    rng = np.random.default_rng(45)
    n_users, n_items, k, d, B = 600, 50_000, 64, 64, 64
    U = torch.as_tensor(rng.normal(size=(n_users, k)).astype(np.float32), device=device)
    V = torch.as_tensor(rng.normal(size=(n_items, k)).astype(np.float32), device=device)
    iv = torch.as_tensor(rng.normal(size=(n_items, d)).astype(np.float32), device=device)
    uv = torch.as_tensor(rng.normal(size=(B, d)).astype(np.float32), device=device)
    rows = torch.as_tensor(rng.choice(n_users, B, replace=False), device=device)
    Vt = _hrec.transpose(V)
    pr = ShardedRecommender(U, Vt, iv, 0, k)
    mt = ShardedRecommender(U, Vt, iv, 0, k, pruned=False)
    assert pr.pruned_exact and not mt.pruned_exact
    for wins in (True, False):
        a = pr.recommend(rows, uv, wins, 5)
        b = mt.recommend(rows, uv, wins, 5)
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
        cap = CapturedRecommend(pr, rows, uv, wins, 5)
        g = cap()
        assert torch.equal(g[0], b[0]) and torch.equal(g[1], b[1])
    assert not pr.last_exact.counts()[2]


@pytest.mark.parametrize("B", [8, 40])
def test_hybrid_exact_many_live_groups(device, B):
    """The first half of the items nearly tie at the top for every user (the
    two-tower vectors along one direction, the ALS side flat), the second
    half scores far below: every user keeps about half of the groups live,
    more than 2a's LDS list holds (> 2 x pair cap). Their pairs are written
    window by window into the shared queue while it has room; the users it
    has no room for rescore every group in 2c. Both give the materialised
    path's bits."""
    h = _h()
    rng = np.random.default_rng(B)
    N, ka, kt = 100_003, 64, 64
    U, V, _, _, rows = _case(device, B, N, ka, kt, 77, same_items=True)
    e = rng.normal(size=kt)
    sign = np.where(np.arange(N) < N // 2, 1.0, -1.0)[:, None]
    iv = sign * e + 1e-4 * rng.normal(size=(N, kt))
    uv = e + 0.01 * rng.normal(size=(B, kt))
    iv = torch.as_tensor(iv.astype(np.float32), device=device)
    uv = torch.as_tensor(uv.astype(np.float32), device=device)
    Vt = h.transpose(V)
    items = h.HybridExactItems(Vt, N, ka, iv)
    G = -(-N // 32)
    for wins in (True, False):
        ei, ev, ea, et = _materialised(h, U, rows, Vt, N, ka, uv, iv, wins, 5)
        hx = h.HybridExact(U, rows, uv, items, 5)
        li, lv, la, lt = hx.local(wins)
        assert torch.equal(li, ei) and torch.equal(lv, ev)
        assert torch.equal(la, ea) and torch.equal(lt, et)
        n_live = hx.counts()[1].cpu().numpy()
        assert ((n_live > 1024) & (n_live < G)).any(), n_live  # the windowed queue path ran
