"""GPU parity of the matrix-core dot-product scoring + fused top-k
(csrc/dot_topk.hip, hrec_dot_scores / hrec_dot_topk) — the two-tower
candidate scoring of src/two_tower_model.py:80,136-146 ranked like
src/hybrid_system.py:108 (stable sort, ties keep candidate order).

Tolerances (written here, per north_star "float scores within 1e-4 rtol"):
* f32 operands: every score is an exact f32 fma chain (the MFMA's k order),
  so |score - f64 dot| <= 1e-6 * sum_k |u_k v_k| (the guide's measured
  0.75-1.5e-7 per unit of sum|ab| at K <= 1024, with margin);
* bf16 operands: products are exact in f32, accumulation f32 -> the same
  bound against the f64 dot of the bf16-ROUNDED vectors;
* top-k: BIT-EXACT (indices and values) against a stable sort of the same
  kernel's full score matrix (the filter pass computes identical values), and
  against the f64 oracle ranking wherever the k-th and (k+1)-th oracle scores
  are separated by more than the score tolerance (SURVEY App. A.3 rule).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _h():
    from src import _hrec

    return _hrec


def _vecs(n, d, seed, scale=1.0):
    g = np.random.default_rng(seed)
    return (g.standard_normal((n, d)) * scale).astype(np.float32)


def _bf16_round(x):
    """f32 -> nearest-even bf16 -> f32 (numpy, the oracle of the device cast)."""
    b = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((b + 0x7FFF + ((b >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def _mfma_scores(h, U, V):
    """hrec_dot_scores (every batch size issues the same MFMA sequence per
    score: the GEMV of B <= 4 users included)."""
    return h.dot_scores(U, V)


def _stable_topk(scores, k):
    """Python's sorted(..., reverse=True)[:k] order on each row: larger first,
    ties -> smaller index."""
    idx = np.argsort(-scores.astype(np.float64), axis=1, kind="stable")[:, :k]
    return idx, np.take_along_axis(scores, idx, 1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,N,d", [(1, 1, 8), (5, 300, 50), (130, 1000, 64), (257, 777, 128), (64, 513, 256),
                                   (3, 40, 32)])
def test_dot_scores_vs_f64(device, dtype, B, N, d):
    h = _h()
    U = _vecs(B, d, 1)
    V = _vecs(N, d, 2)
    Ud = h.dot_operand(torch.from_numpy(U).to(device), dtype)
    Vd = h.dot_operand(torch.from_numpy(V).to(device), dtype)
    got = h.dot_scores(Ud, Vd).cpu().numpy()
    if dtype == torch.bfloat16:
        U, V = _bf16_round(U), _bf16_round(V)
        np.testing.assert_array_equal(Ud.float().cpu().numpy()[:, :d], U)  # device RNE cast is bit-exact
    ref = U.astype(np.float64) @ V.astype(np.float64).T
    bound = 1e-6 * (np.abs(U).astype(np.float64) @ np.abs(V).astype(np.float64).T) + 1e-30
    assert np.all(np.abs(got - ref) <= bound), np.max(np.abs(got - ref) / bound)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,d", [(1, 32), (1, 64), (1, 128), (1, 256), (2, 50), (2, 128), (3, 32), (4, 64)])
def test_few_user_scores_and_topk(device, dtype, B, d):
    """K8v (csrc/dot_gemv.hip: B <= 4 users, the reference's one-user call
    shape; the streaming GEMV where its per-lane partials fit, the matrix-core
    kernel otherwise): scores within the f32 bound of the f64 dot on a ragged
    catalogue (not a multiple of the 64-row tile), and the sampled-bound top-k
    (N > 16384) bit-exact against the same path's full score matrix."""
    h = _h()
    N = 70_001
    U = _vecs(B, d, 40 + B)
    V = _vecs(N, d, 41)
    Ud = h.dot_operand(torch.from_numpy(U).to(device), dtype)
    Vd = h.dot_operand(torch.from_numpy(V).to(device), dtype)
    got = h.dot_scores(Ud, Vd).cpu().numpy()
    if dtype == torch.bfloat16:
        U, V = _bf16_round(U), _bf16_round(V)
    ref = U.astype(np.float64) @ V.astype(np.float64).T
    bound = 1e-6 * (np.abs(U).astype(np.float64) @ np.abs(V).astype(np.float64).T) + 1e-30
    assert np.all(np.abs(got - ref) <= bound), np.max(np.abs(got - ref) / bound)
    for k in (1, 5, 64):
        ei, ev = _stable_topk(got, k)
        gi, gv = h.dot_topk(Ud, Vd, k)
        np.testing.assert_array_equal(gi.cpu().numpy(), ei)
        np.testing.assert_array_equal(gv.cpu().numpy(), ev)


def test_dot_topk_batch_of_four_vs_five(device):
    """f32 batches of 1-4 users take the GEMV and >= 5 users
    the matrix-core tiles; both issue the same MFMA sequence per score, so a
    user's top-k ids AND score bits are the same from a batch of 4 and from a
    batch of 5 — on quantised vectors with many exact ties too."""
    h = _h()
    N, d, k = 50_000, 64, 10
    for quant in (False, True):
        U = _vecs(5, d, 71)
        V = _vecs(N, d, 72)
        if quant:  # few distinct score values: ties at the k-th place
            U, V = np.round(U), np.round(V * 0.5)
        Ud = h.dot_operand(torch.from_numpy(U).to(device), torch.float32)
        Vd = h.dot_operand(torch.from_numpy(V).to(device), torch.float32)
        for kk in (k, 64):
            i4, v4 = h.dot_topk(Ud[:4].contiguous(), Vd, kk)
            i5, v5 = h.dot_topk(Ud, Vd, kk)
            np.testing.assert_array_equal(i4.cpu().numpy(), i5.cpu().numpy()[:4])
            np.testing.assert_array_equal(v4.cpu().numpy().view(np.int32), v5.cpu().numpy()[:4].view(np.int32))
        full = h.dot_scores(Ud, Vd).cpu().numpy()
        ei, ev = _stable_topk(full, k)
        np.testing.assert_array_equal(i5.cpu().numpy()[:, :k], ei)


@pytest.mark.parametrize("d", [32, 64, 128, 256])
def test_dot_scores_bits_independent_of_batch(device, d):
    """hrec_dot_scores (f32): the rows of a batch of 9 users, bit for bit,
    from calls of 1 .. 9 users (GEMV for <= 4, resident / tile kernels above)
    on a ragged catalogue (not a multiple of any kernel's item tile)."""
    h = _h()
    N = 20_011
    U = torch.from_numpy(_vecs(9, d, 80 + d)).to(device)
    V = torch.from_numpy(_vecs(N, d, 81 + d)).to(device)
    ref = h.dot_scores(U, V).cpu().numpy().view(np.int32)
    for B in range(1, 9):
        got = h.dot_scores(U[:B].contiguous(), V).cpu().numpy().view(np.int32)
        np.testing.assert_array_equal(got, ref[:B], err_msg=f"B={B}")
        got = h.dot_scores(U[9 - B:].contiguous(), V).cpu().numpy().view(np.int32)
        np.testing.assert_array_equal(got, ref[9 - B:], err_msg=f"last B={B}")


@pytest.mark.parametrize("d", [16, 32, 50, 64, 100, 128, 256])
def test_tt_score_bits_independent_of_batch(device, d):
    """hrec_tt_score (the Keras Dot of every two-tower ranking): a user's
    scores have the same bits at every batch size (1, 2, 3, 4, 5, 7, 8, 9, 16
    users), from 16-B-misaligned operands (the scalar kernel's fmaf chain in
    the same k order: the MFMA == fmaf-chain identity) and from
    hrec_tt_pair_score on the same (user, item) pairs; within the f32 bound
    of the f64 dot."""
    h = _h()
    N = 9_001
    Un = _vecs(16, d, 90 + d)
    Vn = _vecs(N, d, 91 + d)
    U = torch.from_numpy(Un).to(device)
    V = torch.from_numpy(Vn).to(device)
    ref = h.tt_score(U, V).cpu().numpy()
    f64 = Un.astype(np.float64) @ Vn.astype(np.float64).T
    bound = 1e-6 * (np.abs(Un).astype(np.float64) @ np.abs(Vn).astype(np.float64).T) + 1e-30
    assert np.all(np.abs(ref - f64) <= bound)
    for B in (1, 2, 3, 4, 5, 7, 8, 9):
        got = h.tt_score(U[:B].contiguous(), V).cpu().numpy()
        np.testing.assert_array_equal(got.view(np.int32), ref[:B].view(np.int32), err_msg=f"B={B}")
    # misaligned copies (one float in): the scalar kernel, same k order
    for B in (1, 9, 16):
        ub = torch.empty(B * d + 1, dtype=torch.float32, device=device)
        ub[1:].copy_(U[:B].reshape(-1))
        vb = torch.empty(N * d + 1, dtype=torch.float32, device=device)
        vb[1:].copy_(V.reshape(-1))
        got = h.tt_score(ub[1:].view(B, d), vb[1:].view(N, d)).cpu().numpy()
        np.testing.assert_array_equal(got.view(np.int32), ref[:B].view(np.int32), err_msg=f"misaligned B={B}")
    # pair scores: user b against item j
    j = torch.arange(N, device=device) % 997
    b = torch.arange(N, device=device) % 16
    pair = h.tt_pair_score(U[b].contiguous(), V[j].contiguous()).cpu().numpy()
    np.testing.assert_array_equal(pair.view(np.int32), ref[b.cpu().numpy(), j.cpu().numpy()].view(np.int32))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,N,d,k", [(7, 5000, 64, 5), (130, 40000, 128, 5), (3, 100003, 64, 10),
                                     (1, 20000, 256, 1), (200, 17000, 32, 64), (2, 3, 64, 5)])
def test_dot_topk_bit_exact_vs_full_scores(device, dtype, B, N, d, k):
    """Sample-threshold + fused filter (N > 16384) and the small exact path
    return exactly the stable top-k of the full score matrix."""
    h = _h()
    Ud = h.dot_operand(torch.from_numpy(_vecs(B, d, 3)).to(device), dtype)
    Vd = h.dot_operand(torch.from_numpy(_vecs(N, d, 4)).to(device), dtype)
    full = h.dot_scores(Ud, Vd).cpu().numpy()
    ei, ev = _stable_topk(full, min(k, N))
    gi, gv = h.dot_topk(Ud, Vd, k)
    np.testing.assert_array_equal(gi.cpu().numpy(), ei)
    np.testing.assert_array_equal(gv.cpu().numpy(), ev)


@pytest.mark.parametrize("dtype,d,B,N,per", [(torch.bfloat16, 256, 256, 100_003, 784), (torch.bfloat16, 64, 70, 5000, 0),
                                             (torch.float32, 128, 33, 20_000, 300), (torch.bfloat16, 128, 300, 777, 16)])
def test_dot_filter_per_group_bounds(device, dtype, d, B, N, per):
    """hrec_dot_filter: exactly the items with score >= the bound of their
    (user, item group) survive (a NaN bound admits the group), each with its
    hrec_dot_scores value (bit-exact); the count of an overflowing list is
    still exact. Survivors cluster on the same items for every user (as the
    pruned hybrid's do): one shared direction dominates the user vectors."""
    h = _h()
    rng = np.random.default_rng(7)
    common = rng.standard_normal(d).astype(np.float32)
    U = (_vecs(B, d, 8, 0.3) + common).astype(np.float32)
    Ud = h.dot_operand(torch.from_numpy(U).to(device), dtype)
    Vd = h.dot_operand(torch.from_numpy(_vecs(N, d, 9)).to(device), dtype)
    S = h.dot_scores(Ud, Vd).cpu().numpy()
    G = (N + per - 1) // per if per else 1
    grp = (np.arange(N) // per) if per else np.zeros(N, dtype=np.int64)
    hi = S.max(1, keepdims=True)
    lo = np.quantile(S, 0.99, axis=1, keepdims=True)
    thr = (lo + (hi - lo) * rng.random((B, G))).astype(np.float32)
    thr[5] = np.inf  # admits nothing (the kernel skips such users' chunks)
    if per:
        thr[3, G // 2] = np.nan  # admits the whole group
        thr[7:, 1::2] = np.inf  # dead groups
    cap = 512
    cv, ci, cn = h.dot_filter(Ud, Vd, torch.from_numpy(thr), per, cap)
    cv, ci, cn = cv.cpu().numpy(), ci.cpu().numpy(), cn.cpu().numpy()
    tf = thr[:, grp]
    want = np.where(np.isnan(tf), True, S >= tf)
    np.testing.assert_array_equal(cn, want.sum(1))  # no list here overflows a block's staging buffer
    for b in range(B):
        if cn[b] > cap:
            continue
        order = np.argsort(ci[b, : cn[b]])
        ids = ci[b, : cn[b]][order]
        np.testing.assert_array_equal(ids, np.nonzero(want[b])[0])
        np.testing.assert_array_equal(cv[b, : cn[b]][order], S[b, ids])


def test_dot_filter_staging_overflow_keeps_lists_valid(device):
    """More survivors in one tile than a block's LDS staging buffer holds
    (every score admitted): every such user is marked overflowing (count >
    cap) and every list slot still holds an entry — a real survivor with its
    exact score, or the (-inf, INT64_MAX - 1) filler — so the list's k-th best
    stays a valid lower bound."""
    h = _h()
    B, N, d, cap = 256, 5000, 256, 512
    Ud = h.dot_operand(torch.from_numpy(_vecs(B, d, 10)).to(device), torch.bfloat16)
    Vd = h.dot_operand(torch.from_numpy(_vecs(N, d, 11)).to(device), torch.bfloat16)
    S = h.dot_scores(Ud, Vd).cpu().numpy()
    thr = torch.full((B,), float("nan"))
    cv, ci, cn = h.dot_filter(Ud, Vd, thr, 0, cap)
    cv, ci, cn = cv.cpu().numpy(), ci.cpu().numpy(), cn.cpu().numpy()
    assert np.all(cn > cap)
    filler = ci == np.iinfo(np.int64).max - 1
    assert np.all(cv[filler] == -np.inf)
    for b in range(B):
        ids = ci[b][~filler[b]]
        assert np.all((ids >= 0) & (ids < N)) and len(np.unique(ids)) == len(ids)
        np.testing.assert_array_equal(cv[b][~filler[b]], S[b, ids])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_dot_topk_infinite_scores(device, dtype):
    """k or more items scoring +inf (overflowing dots) put +inf in
    the sample's k-th best, i.e. the filter bound; hrec_dot_topk must still
    admit scores >= +inf (the +inf items, smaller index first), as the full
    score matrix's stable top-k says."""
    h = _h()
    N, d, k = 20_000, 64, 5
    rng = np.random.default_rng(31)
    U = np.abs(rng.standard_normal((3, d))).astype(np.float32) + 0.5
    V = rng.standard_normal((N, d)).astype(np.float32)
    hot = np.arange(100, 1100, 100)  # 10 items on the sample's stride (even ids)
    V[hot] = 3e38
    Ud = h.dot_operand(torch.from_numpy(U).to(device), dtype)
    Vd = h.dot_operand(torch.from_numpy(V).to(device), dtype)
    full = h.dot_scores(Ud, Vd).cpu().numpy()
    assert np.all(np.isposinf(full[:, hot]))
    ei, ev = _stable_topk(full, k)
    gi, gv = h.dot_topk(Ud, Vd, k)
    np.testing.assert_array_equal(gi.cpu().numpy(), ei)
    np.testing.assert_array_equal(gi.cpu().numpy(), np.tile(hot[:k], (3, 1)))
    np.testing.assert_array_equal(gv.cpu().numpy(), ev)


def test_dot_topk_ties_keep_candidate_order(device):
    """Duplicated item vectors score identically: the reference's stable sort
    keeps candidate (index) order among them."""
    h = _h()
    base = _vecs(50, 64, 5)
    V = np.concatenate([base] * 600)  # 30000 items, every score repeated 600 times
    Ud = h.dot_operand(torch.from_numpy(_vecs(9, 64, 6)).to(device))
    Vd = h.dot_operand(torch.from_numpy(V).to(device))
    gi, gv = h.dot_topk(Ud, Vd, 5)
    full = h.dot_scores(Ud, Vd).cpu().numpy()
    ei, ev = _stable_topk(full, 5)
    np.testing.assert_array_equal(gi.cpu().numpy(), ei)
    np.testing.assert_array_equal(gv.cpu().numpy(), ev)
    best = np.argmax(full[:, :50], axis=1)
    np.testing.assert_array_equal(gi.cpu().numpy()[:, :5], best[:, None] + 50 * np.arange(5)[None, :])


def test_dot_topk_overflow_falls_back_exactly(device):
    """Every item scores the same -> every item survives every threshold: the
    overflow flag triggers the refinement round and then the exact chunked
    path, which returns the first k items (stable order)."""
    h = _h()
    V = np.tile(_vecs(1, 32, 7), (70000, 1))
    Ud = h.dot_operand(torch.from_numpy(_vecs(4, 32, 8)).to(device))
    Vd = h.dot_operand(torch.from_numpy(V).to(device))
    gi, gv = h.dot_topk(Ud, Vd, 6)
    np.testing.assert_array_equal(gi.cpu().numpy(), np.tile(np.arange(6), (4, 1)))
    full = h.dot_scores(Ud, Vd[:1]).cpu().numpy()
    np.testing.assert_array_equal(gv.cpu().numpy(), np.repeat(full, 6, axis=1))


def test_dot_topk_offset_and_shards_merge(device):
    """Item shards with idx_offset + a keyed merge == the unsharded top-k
    (the per-rank step of the sharded c4 scoring)."""
    h = _h()
    U = _vecs(33, 128, 9)
    V = _vecs(50000, 128, 10)
    Ud = h.dot_operand(torch.from_numpy(U).to(device))
    Vd = h.dot_operand(torch.from_numpy(V).to(device))
    ei, ev = h.dot_topk(Ud, Vd, 5)
    parts_i, parts_v = [], []
    for lo, hi in ((0, 17000), (17000, 17001), (17001, 50000)):
        i, v = h.dot_topk(Ud, Vd[lo:hi].contiguous(), 5, idx_offset=lo)
        parts_i.append(i)
        parts_v.append(v.double())
    mi, mv = h.topk_keyed(torch.cat(parts_v, 1).contiguous(), torch.cat(parts_i, 1).contiguous(), 5)
    np.testing.assert_array_equal(mi.cpu().numpy(), ei.cpu().numpy())
    np.testing.assert_array_equal(mv.float().cpu().numpy(), ev.cpu().numpy())


def test_dot_topk_matches_f64_ranking_outside_ties(device):
    """Against the f64 oracle ranking: indices equal wherever the oracle's
    k-th and (k+1)-th scores differ by more than the score tolerance."""
    h = _h()
    B, N, d, k = 64, 60000, 128, 5
    U, V = _vecs(B, d, 11), _vecs(N, d, 12)
    gi, gv = h.dot_topk(h.dot_operand(torch.from_numpy(U).to(device)),
                        h.dot_operand(torch.from_numpy(V).to(device)), k)
    ref = U.astype(np.float64) @ V.astype(np.float64).T
    order = np.argsort(-ref, axis=1, kind="stable")
    tol = 1e-6 * (np.abs(U).astype(np.float64) @ np.abs(V).astype(np.float64).T).max()
    gi = gi.cpu().numpy()
    checked = 0
    for b in range(B):
        r = ref[b, order[b]]
        if r[k - 1] - r[k] > 2 * tol and np.all(r[:k - 1] - r[1:k] > 2 * tol):
            np.testing.assert_array_equal(gi[b], order[b, :k])
            checked += 1
        np.testing.assert_allclose(gv.cpu().numpy()[b], r[:k], rtol=1e-4, atol=tol)
    assert checked >= B // 2


@pytest.mark.parametrize("n_items", [3000, 120_000])
def test_hybrid_bf16_mode_matches_f64_fusion(device, n_items):
    """BASELINE c5 numerics: rank-200 ALS factors (kp 256) and d = 256 tower
    vectors in bf16, both score matrices on the bf16 matrix cores, then the
    reference fusion (per-model min-max, 0.2/0.8 weights, stable top-5).
    Checked against the f64 fusion of the bf16-ROUNDED operands: fused
    scores within 1e-4, indices equal wherever the oracle's consecutive
    top-6 scores are separated by more than 1e-4. 120k items: the pruned
    path's per-group bounds and survivor filter over more than the 16,384
    items below which it scores everything (the path c5 serves)."""
    from src.recommend import ShardedRecommender

    rng = np.random.default_rng(21)
    n_users, k, kp, d = 40, 200, 256, 256
    U = np.zeros((n_users, kp), np.float32)
    U[:, :k] = rng.normal(size=(n_users, k)) / np.sqrt(k)
    V = np.zeros((n_items, kp), np.float32)
    V[:, :k] = rng.normal(size=(n_items, k)) / np.sqrt(k)
    uv = (rng.normal(size=(8, d)) / 16).astype(np.float32)
    iv = (rng.normal(size=(n_items, d)) / 16).astype(np.float32)
    rows = np.array([0, 3, 5, 7, 11, 13, 17, 39])
    rec = ShardedRecommender(torch.from_numpy(U).to(device), None, torch.from_numpy(iv).to(device), 0, k,
                             precision="bf16", V_local=torch.from_numpy(V).to(device))
    gi, gv = rec.recommend(torch.from_numpy(rows).to(device), torch.from_numpy(uv).to(device), False, 5)
    if n_items > 16384:
        assert not rec.last_prune.fallback_taken()  # the pruned path itself answered
    als = _bf16_round(U[rows]).astype(np.float64) @ _bf16_round(V).astype(np.float64).T
    tt = _bf16_round(uv).astype(np.float64) @ _bf16_round(iv).astype(np.float64).T

    def mm(x):
        lo, hi = x.min(1, keepdims=True), x.max(1, keepdims=True)
        return (x - lo) / (hi - lo)

    fused = 0.2 * mm(als) + 0.8 * mm(tt)
    order = np.argsort(-fused, axis=1, kind="stable")
    gi, gv = gi.cpu().numpy(), gv.cpu().numpy()
    for b in range(len(rows)):
        f = fused[b, order[b, :6]]
        np.testing.assert_allclose(gv[b], f[:5], atol=1e-4)
        for j in range(5):
            if (j == 0 or f[j - 1] - f[j] > 1e-4) and f[j] - f[j + 1] > 1e-4:
                assert gi[b, j] == order[b, j], (b, j)


@pytest.mark.parametrize("dk,B,N,ka,kt", [(256, 256, 100_003, 256, 256), (256, 300, 1000, 200, 250),
                                          (128, 70, 4097, 100, 50), (64, 1, 17, 64, 33), (64, 513, 2000, 48, 64),
                                          (256, 5, 1, 256, 7)])
def test_hybrid_scores_equals_dot_scores_and_minmax(device, dk, B, N, ka, kt):
    """hrec_hybrid_scores (user gather + bf16 conversion + both score GEMMs
    + per-row min/max in one launch) == hrec_f32_to_bf16 operands through
    hrec_dot_scores and hrec_rows_minmax_f32, bit for bit: odd widths and
    row strides, several user tiles (B > 256 at dk 256), tiny and ragged
    item counts, repeated user rows."""
    h = _h()
    rng = np.random.default_rng(B * 7 + N)
    n_users = max(B, 9)
    U = torch.as_tensor(rng.normal(size=(n_users, ka)).astype(np.float32), device=device)
    uv = torch.as_tensor(rng.normal(size=(B, kt)).astype(np.float32) / 4, device=device)
    va = h.dot_operand(torch.as_tensor(rng.normal(size=(N, ka)).astype(np.float32), device=device), torch.bfloat16, dk)
    vt = h.dot_operand(torch.as_tensor(rng.normal(size=(N, kt)).astype(np.float32), device=device), torch.bfloat16, dk)
    rows = torch.as_tensor(rng.integers(0, n_users, B), dtype=torch.int64, device=device)
    als, tt, a_mm, t_mm = h.hybrid_scores(U, rows, uv, va, vt)
    ua = h.dot_operand(U.index_select(0, rows), torch.bfloat16, dk)
    ut = h.dot_operand(uv, torch.bfloat16, dk)
    ref_a, ref_t = _mfma_scores(h, ua, va), _mfma_scores(h, ut, vt)
    assert torch.equal(als, ref_a) and torch.equal(tt, ref_t)
    assert torch.equal(a_mm, h.rows_minmax(ref_a)) and torch.equal(t_mm, h.rows_minmax(ref_t))


def test_hybrid_scores_unknown_rows_are_nan(device):
    """an ALS row outside [0, n) (the -1 of an unknown user, or a
    stale row) is never read: its score row is NaN (as hrec_als_score gives
    for -1) and its min / max +inf / -inf; the other rows are unchanged."""
    h = _h()
    rng = np.random.default_rng(3)
    U = torch.as_tensor(rng.normal(size=(10, 64)).astype(np.float32), device=device)
    uv = torch.as_tensor(rng.normal(size=(4, 64)).astype(np.float32), device=device)
    v = h.dot_operand(torch.as_tensor(rng.normal(size=(300, 64)).astype(np.float32), device=device), torch.bfloat16)
    rows = torch.tensor([2, -1, 10, 1 << 40], dtype=torch.int64, device=device)
    als, tt, a_mm, _ = h.hybrid_scores(U, rows, uv, v, v)
    assert torch.isnan(als[1:]).all() and not torch.isnan(als[0]).any()
    ref = _mfma_scores(h, h.dot_operand(U[2:3], torch.bfloat16), v)
    assert torch.equal(als[0:1], ref)
    assert torch.all(a_mm[0, 1:] == float("inf")) and torch.all(a_mm[1, 1:] == -float("inf"))
    assert not torch.isnan(tt).any()


def test_hybrid_scores_empty_catalogue(device):
    h = _h()
    U = torch.ones((4, 64), device=device)
    v = torch.empty((0, 64), dtype=torch.bfloat16, device=device)
    als, tt, a_mm, t_mm = h.hybrid_scores(U, torch.arange(4, device=device), U, v, v)
    assert als.shape == (4, 0) and torch.all(a_mm[0] == float("inf")) and torch.all(t_mm[1] == -float("inf"))


@pytest.mark.parametrize("precision", ["exact", "bf16"])
def test_captured_recommend_matches_eager(device, precision):
    """CapturedRecommend (HIP graph replay of one recommend batch) returns the
    eager results bit for bit, for new user batches copied into the
    captured inputs."""
    from src import _hrec
    from src.recommend import CapturedRecommend, ShardedRecommender

    rng = np.random.default_rng(41)
    n_users, n_items, k, d, B = 500, 20_000, 32, 48, 64
    U = torch.as_tensor(rng.normal(size=(n_users, k)).astype(np.float32), device=device)
    V = torch.as_tensor(rng.normal(size=(n_items, k)).astype(np.float32), device=device)
    iv = torch.as_tensor(rng.normal(size=(n_items, d)).astype(np.float32), device=device)
    if precision == "exact":
        rec = ShardedRecommender(U, _hrec.transpose(V), iv, 0, k)
    else:
        rec = ShardedRecommender(U, None, iv, 0, k, precision="bf16", V_local=V)
    rows = [torch.as_tensor(rng.choice(n_users, B, replace=False), device=device) for _ in range(3)]
    vecs = [torch.as_tensor(rng.normal(size=(B, d)).astype(np.float32), device=device) for _ in range(3)]
    for wins in (True, False):
        cap = CapturedRecommend(rec, rows[0], vecs[0], wins, 5)
        for r, v in zip(rows, vecs):
            gi, gv = cap(r, v)
            ei, ev = rec.recommend(r, v, wins, 5)
            assert torch.equal(gi, ei) and torch.equal(gv, ev)


def _unfused_bf16(h, U, rows, uv, va, vt, als_wins, k, offset=0):
    als, tt, a_mm, t_mm = h.hybrid_scores(U, rows, uv, va, vt)
    return h.fuse_rows_topk(als, tt, a_mm, t_mm, als_wins, k, offset), (a_mm, t_mm)


@pytest.mark.parametrize("dk,B,N,ka,kt,k", [(256, 256, 100_003, 256, 256, 5), (256, 70, 20_000, 200, 250, 8),
                                            (128, 130, 40_001, 100, 64, 1), (64, 33, 5_000, 48, 64, 3),
                                            (64, 300, 777, 64, 33, 5), (256, 5, 9, 256, 7, 8), (128, 2, 1, 128, 128, 5)])
def test_hybrid_prune_equals_unfused(device, dk, B, N, ka, kt, k):
    """K9p (csrc/hybrid_prune.hip: no score matrix; bound from the group
    maxima, heavy-model survivor filter, light scores of the survivors) ==
    hrec_hybrid_scores + hrec_fuse_rows_topk bit for bit — ids, fused scores
    and both min / max rows — for both weight orders, and on random data the
    pruned path itself answered (no fallback)."""
    h = _h()
    rng = np.random.default_rng(B * 3 + N)
    n_users = B + 7
    U = torch.as_tensor(rng.normal(size=(n_users, ka)).astype(np.float32), device=device)
    uv = torch.as_tensor(rng.normal(size=(B, kt)).astype(np.float32) / 4, device=device)
    va = h.dot_operand(torch.as_tensor(rng.normal(size=(N, ka)).astype(np.float32), device=device), torch.bfloat16, dk)
    vt = h.dot_operand(torch.as_tensor(rng.normal(size=(N, kt)).astype(np.float32), device=device), torch.bfloat16, dk)
    rows = torch.as_tensor(rng.integers(0, n_users, B), dtype=torch.int64, device=device)
    for wins in (True, False):
        (ei, ev), (ea, et) = _unfused_bf16(h, U, rows, uv, va, vt, wins, k, 11)
        hp = h.HybridPrune(U, rows, uv, va, vt, k)
        a_mm, t_mm = hp.minmax()
        assert torch.equal(a_mm, ea) and torch.equal(t_mm, et)
        gi, gv = hp.topk(a_mm, t_mm, wins, 11)
        assert torch.equal(gi, ei), (wins, (gi != ei).nonzero()[:5])
        assert torch.equal(gv, ev)
        if N >= 1000:
            assert not hp.fallback_taken()
        # one shard: both phases in one call (the bound kernel folds the extremes)
        li, lv, la, lt = hp.local(wins, 11)
        assert torch.equal(li, ei) and torch.equal(lv, ev)
        assert torch.equal(la, ea) and torch.equal(lt, et)


def test_hybrid_prune_fallback_cases(device):
    """The exact path (inside the survivor kernel, per user) answers with the
    same bits as the unfused path when the pruned one cannot: every item
    identical (all fused scores tie: the survivor list overflows), an unknown
    ALS row (NaN scores) and a catalogue with tied maxima — through both the
    two-phase calls and the one-shard call."""
    h = _h()
    rng = np.random.default_rng(12)
    B, N, dk = 40, 30_000, 128
    U = torch.as_tensor(rng.normal(size=(60, 128)).astype(np.float32), device=device)
    uv = torch.as_tensor(rng.normal(size=(B, 128)).astype(np.float32), device=device)
    same = np.tile(rng.normal(size=(1, 128)).astype(np.float32), (N, 1))
    va = h.dot_operand(torch.as_tensor(same, device=device), torch.bfloat16, dk)
    vt = h.dot_operand(torch.as_tensor(rng.normal(size=(N, 128)).astype(np.float32), device=device), torch.bfloat16, dk)
    rows = torch.as_tensor(rng.integers(0, 60, B), dtype=torch.int64, device=device)
    rows_bad = rows.clone()
    rows_bad[3] = -1
    for r, a_items, wins in ((rows, va, True), (rows_bad, vt, True), (rows_bad, vt, False)):
        (ei, ev), _ = _unfused_bf16(h, U, r, uv, a_items, vt, wins, 5)
        hp = h.HybridPrune(U, r, uv, a_items, vt, 5)
        gi, gv = hp.topk(*hp.minmax(), wins)
        assert hp.fallback_taken()
        assert torch.equal(gi, ei)
        np.testing.assert_array_equal(gv.cpu().numpy(), ev.cpu().numpy())  # NaN == NaN position-wise
        li, lv, _, _ = hp.local(wins)
        assert hp.fallback_taken()
        assert torch.equal(li, ei)
        np.testing.assert_array_equal(lv.cpu().numpy(), ev.cpu().numpy())


def test_recommender_bf16_paths_agree(device):
    """ShardedRecommender precision "bf16": pruned (default) and unfused
    (pruned=False) return the same ids and scores."""
    from src.recommend import ShardedRecommender

    rng = np.random.default_rng(44)
    n_users, n_items, k, d, B = 400, 50_000, 200, 256, 64
    U = torch.as_tensor(rng.normal(size=(n_users, 256)).astype(np.float32), device=device)
    V = torch.as_tensor(rng.normal(size=(n_items, k)).astype(np.float32), device=device)
    iv = torch.as_tensor(rng.normal(size=(n_items, d)).astype(np.float32), device=device)
    uv = torch.as_tensor(rng.normal(size=(B, d)).astype(np.float32), device=device)
    rows = torch.as_tensor(rng.choice(n_users, B, replace=False), device=device)
    recs = [ShardedRecommender(U, None, iv, 0, k, precision="bf16", V_local=V, **kw)
            for kw in ({}, {"pruned": False})]
    for wins in (True, False):
        outs = [r.recommend(rows, uv, wins, 5) for r in recs]
        for i, v in outs[1:]:
            assert torch.equal(outs[0][0], i) and torch.equal(outs[0][1], v)
    assert not recs[0].last_prune.fallback_taken()


def _f64_topk_chunked(U, V, k, chunk=1 << 20):
    vs, is_ = [], []
    for j0 in range(0, V.shape[0], chunk):
        s = U.double() @ V[j0: j0 + chunk].double().T
        v, i = torch.topk(s, k + 1, dim=1)
        vs.append(v)
        is_.append(i + j0)
    v, i = torch.cat(vs, 1), torch.cat(is_, 1)
    o = torch.argsort(-v, dim=1, stable=True)[:, : k + 1]
    return v.gather(1, o), i.gather(1, o)


@pytest.mark.parametrize("dtype,d", [(torch.float32, 128), (torch.bfloat16, 256)])
def test_dot_topk_beyond_4gib_operands(device, dtype, d):
    """Item operands larger than the 4 GiB a buffer resource spans (20M x 128
    f32 = 10 GB; 10M x 256 bf16 = 5 GB): the per-tile re-based resources read
    every row (round 2's single resource wrapped at row 2^32 / row bytes and
    ranked the first rows again). Top-5 of 8 users vs the f64 ranking."""
    h = _h()
    n = 20_000_000 if dtype == torch.float32 else 10_000_000
    g = torch.Generator(device=device).manual_seed(3)
    V = torch.randn((n, d), device=device, generator=g) * 0.1
    U = torch.randn((8, d), device=device, generator=g)
    Vd, Ud = h.dot_operand(V, dtype), h.dot_operand(U, dtype)
    del V
    gi, gv = h.dot_topk(Ud, Vd, 5)
    rv, ri = _f64_topk_chunked(Ud, Vd, 5)
    assert int(gi.max()) > (1 << 32) // (d * Vd.element_size())  # winners past the old wrap point exist
    for b in range(8):
        gaps = (rv[b, :-1] - rv[b, 1:]).min().item()
        if gaps > 1e-3:
            assert gi[b].tolist() == ri[b, :5].tolist(), b
        np.testing.assert_allclose(gv[b].double().cpu().numpy(), rv[b, :5].cpu().numpy(), rtol=1e-5, atol=1e-4)


def test_hybrid_paths_beyond_4gib_operands(device):
    """The c5 kernels on item operands past 4 GiB (9M items x dk 256 bf16 =
    4.6 GB per model): pruned == unfused bit for bit, and the unfused scores
    of the last items equal a direct dot of those rows."""
    h = _h()
    n, B = 9_000_000, 8
    g = torch.Generator(device=device).manual_seed(4)
    va = h.dot_operand(torch.randn((n, 256), device=device, generator=g) * 0.1, torch.bfloat16)
    vt = h.dot_operand(torch.randn((n, 256), device=device, generator=g) * 0.1, torch.bfloat16)
    U = torch.randn((16, 256), device=device, generator=g)
    uv = torch.randn((B, 256), device=device, generator=g)
    rows = torch.arange(B, dtype=torch.int64, device=device) * 2
    als, tt, a_mm, t_mm = h.hybrid_scores(U, rows, uv, va, vt)
    tail = slice(n - 1000, n)
    ua = h.dot_operand(U.index_select(0, rows), torch.bfloat16)
    assert torch.equal(als[:, tail], h.dot_scores(ua, va[tail].contiguous()))
    for wins in (True, False):
        ei, ev = h.fuse_rows_topk(als, tt, a_mm, t_mm, wins, 5)
        hp = h.HybridPrune(U, rows, uv, va, vt, 5)
        gi, gv = hp.topk(*hp.minmax(), wins)
        assert torch.equal(gi, ei) and torch.equal(gv, ev)
