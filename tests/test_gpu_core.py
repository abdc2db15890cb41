"""GPU parity of the HIP kernels through the C-ABI vs the CPU oracle.

Tolerances: integer/index/byte work (synthetic CSR, init factors, ALS
scoring — a JVM-exact f32 chain —, top-k, fusion) is compared BIT-EXACT.
The ALS half-sweep accumulates the Gramian in f64 in a different summation
order than Spark/the oracle, so factors are compared at rtol 1e-5 (one
half-sweep) and rtol 1e-4 after several epochs (north_star: "float scores
within 1e-4 rtol").
"""
import numpy as np
import pytest
import torch
from conftest import dec_pairs, load_golden

from oracle import als as oals
from oracle import build as obuild
from oracle import fusion as ofus
from oracle import synth as osyn

pytestmark = pytest.mark.gpu


def _hrec():
    from src import _hrec

    return _hrec


def _csr_to_dev(indptr, indices, values, device):
    return (torch.as_tensor(indptr, dtype=torch.int64, device=device),
            torch.as_tensor(indices, dtype=torch.int32, device=device),
            torch.as_tensor(values, dtype=torch.float32, device=device))


# ------------------------------------------------------------------ synth
@pytest.mark.parametrize("transposed", [0, 1])
@pytest.mark.parametrize("row_begin,n_rows", [(0, 300), (37, 50), (280, 40)])
def test_synth_bit_exact(device, transposed, row_begin, n_rows):
    from src import synthetic

    n_users, n_items, dens = 300, 260, 0.04
    got = synthetic.generate(n_users, n_items, dens, bool(transposed), row_begin, n_rows, seed=99, seed2=98)
    exp = obuild.synth_csr(n_users, n_items, dens, transposed, row_begin, n_rows, 99, 98)
    np.testing.assert_array_equal(got.indptr.cpu().numpy(), exp[0])
    np.testing.assert_array_equal(got.indices.cpu().numpy(), exp[1])
    np.testing.assert_array_equal(got.values.cpu().numpy(), exp[2])


def test_synth_empty_and_dense(device):
    from src import synthetic

    z = synthetic.generate(50, 40, 0.0, False)
    assert z.nnz == 0 and int(z.indptr[-1]) == 0
    d = synthetic.generate(20, 70, 0.999, False)
    exp = obuild.synth_csr(20, 70, 0.999, 0, 0, 20, synthetic.SEED, synthetic.SEED2)
    np.testing.assert_array_equal(d.indices.cpu().numpy(), exp[1])


@pytest.mark.parametrize("k,kp", [(10, 16), (16, 16), (20, 32), (50, 64), (64, 64)])
def test_init_factors_bit_exact(device, k, kp):
    h = _hrec()
    out = torch.full((33, kp), 7.0, device=device)
    h.als_init_factors(5, 1000, 33, k, kp, out)
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got[:, :k], osyn.init_factors(5, 1000, 33, k))
    assert (got[:, k:] == 0).all()


# ------------------------------------------------------------ ALS sweep
def _problem(seed, n_rows, n_src, k, max_deg, kp):
    rng = np.random.default_rng(seed)
    deg = rng.integers(0, max_deg, n_rows)
    deg[0] = 0          # empty row
    deg[1] = 1          # single rating
    if n_rows > 2:
        deg[2] = 3 * 64 + 5  # several pipeline chunks
    indptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    indices = rng.integers(0, n_src, indptr[-1]).astype(np.int32)
    values = rng.integers(0, 19, indptr[-1]).astype(np.float32)
    src = np.zeros((n_src, kp), np.float32)
    src[:, :k] = rng.normal(size=(n_src, k)).astype(np.float32)
    return indptr, indices, values, src


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("k,kp", [(8, 16), (16, 16), (20, 32), (32, 32), (50, 64), (64, 64)])
def test_half_sweep_matches_oracle(device, k, kp, mode):
    h = _hrec()
    indptr, indices, values, src = _problem(k, 70, 90, k, 150, kp)
    d_ip, d_ix, d_v = _csr_to_dev(indptr, indices, values, device)
    d_src = torch.as_tensor(src, device=device)
    dst = torch.full((70, kp), 3.0, device=device)
    h.als_half_sweep(d_ip, d_ix, d_v, d_src, k, 0.1, dst, accum_mode=mode)
    got = dst.cpu().numpy()
    exp = obuild.half_sweep(indptr, indices, values, src[:, :k], k, 0.1)
    # mode 0 accumulates in f64 like Spark; mode 1 rounds to f32 inside
    # 16-rating chunks (relative Gramian error ~1e-7), hence the looser bound
    rtol, atol = (1e-5, 1e-6) if mode == 0 else (1e-4, 1e-5)
    np.testing.assert_allclose(got[:, :k], exp, rtol=rtol, atol=atol)
    assert (got[:, k:] == 0).all(), "padding columns must stay zero"
    assert (got[0] == 0).all(), "a row without ratings has no factor"


@pytest.mark.parametrize("mode", [0, 1])
def test_half_sweep_window_boundaries(device, mode):
    """Row lengths around every pipeline boundary of the kp=64 kernel (steps of
    4 ratings, windows of 64, prefetch distance) and gathers of the first and
    last source rows (the structured-buffer range check must keep them)."""
    h = _hrec()
    k, kp, n_src = 64, 64, 301
    deg = np.array([0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 63, 64, 65, 66, 67, 95, 96, 97,
                    127, 128, 129, 130, 191, 192, 193, 255, 256, 257, 1000, 1023, 1024, 1025])
    rng = np.random.default_rng(11)
    indptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    indices = rng.integers(0, n_src, indptr[-1]).astype(np.int32)
    indices[::7] = n_src - 1
    indices[3::11] = 0
    values = rng.integers(0, 19, indptr[-1]).astype(np.float32)
    src = rng.normal(size=(n_src, kp)).astype(np.float32)
    d_ip, d_ix, d_v = _csr_to_dev(indptr, indices, values, device)
    dst = torch.full((len(deg), kp), 3.0, device=device)
    h.als_half_sweep(d_ip, d_ix, d_v, torch.as_tensor(src, device=device), k, 0.1, dst, accum_mode=mode)
    exp = obuild.half_sweep(indptr, indices, values, src, k, 0.1)
    rtol, atol = (1e-5, 1e-6) if mode == 0 else (1e-4, 1e-5)
    np.testing.assert_allclose(dst.cpu().numpy(), exp, rtol=rtol, atol=atol)


def test_half_sweep_src64_equals_f32_sources(device):
    """hrec_als_half_sweep_src64 (source factors pre-converted to f64, the
    user side's path at c2) returns the f32-source kernel's factors bit for
    bit (the gather converts exactly either way), across the pipeline's
    window boundaries and the first/last source rows; and matches the C
    oracle."""
    h = _hrec()
    k, kp, n_src = 64, 64, 301
    deg = np.array([0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 63, 64, 65, 66, 67, 95, 96, 97,
                    127, 128, 129, 130, 191, 192, 193, 255, 256, 257, 1000, 1023, 1024, 1025])
    rng = np.random.default_rng(12)
    indptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    indices = rng.integers(0, n_src, indptr[-1]).astype(np.int32)
    indices[::7] = n_src - 1
    indices[3::11] = 0
    values = rng.integers(0, 19, indptr[-1]).astype(np.float32)
    src = rng.normal(size=(n_src, kp)).astype(np.float32)
    d_ip, d_ix, d_v = _csr_to_dev(indptr, indices, values, device)
    d_src = torch.as_tensor(src, device=device)
    a = torch.full((len(deg), kp), 3.0, device=device)
    b = torch.full((len(deg), kp), 5.0, device=device)
    h.als_half_sweep(d_ip, d_ix, d_v, d_src, k, 0.1, a)
    s64 = h.f32_to_f64(d_src)
    assert torch.equal(s64, d_src.double())
    h.als_half_sweep(d_ip, d_ix, d_v, d_src, k, 0.1, b, src64=s64)
    assert torch.equal(a, b)
    np.testing.assert_allclose(b.cpu().numpy(), obuild.half_sweep(indptr, indices, values, src, k, 0.1),
                               rtol=1e-5, atol=1e-6)


def test_engine_uses_src64_for_cached_sources(device):
    """DeviceALS gathers sources of at most SRC64_MAX_BYTES from an f64 copy
    and larger ones in f32: the fit is the same either way."""
    from src import als_engine, synthetic
    from src.als_engine import DeviceALS

    n_users, n_items, dens, k = 600, 300, 0.05, 64
    fits = []
    for limit in (1 << 40, 0):
        old = als_engine.SRC64_MAX_BYTES
        als_engine.SRC64_MAX_BYTES = limit
        try:
            csr = synthetic.generate(n_users, n_items, dens, False)
            csc = synthetic.generate(n_users, n_items, dens, True)
            eng = DeviceALS(n_users, n_items, k, 0.1, csr, csc)
            eng.init_user_factors(synthetic.SEED_INIT)
            eng.fit(3)
            assert (eng._s64 is not None) == (limit > 0)
            fits.append((eng.user_factors.clone(), eng.item_factors.clone()))
        finally:
            als_engine.SRC64_MAX_BYTES = old
    assert torch.equal(fits[0][0], fits[1][0]) and torch.equal(fits[0][1], fits[1][1])


def test_half_sweep_spark_literal_small(device):
    h = _hrec()
    indptr, indices, values, src = _problem(7, 12, 20, 10, 20, 16)
    d_ip, d_ix, d_v = _csr_to_dev(indptr, indices, values, device)
    dst = torch.zeros((12, 16), device=device)
    h.als_half_sweep(d_ip, d_ix, d_v, torch.as_tensor(src, device=device), 10, 0.5, dst)
    exp = oals.half_sweep_spark(indptr, indices, values, src[:, :10], 10, 0.5)
    np.testing.assert_allclose(dst.cpu().numpy()[:, :10], exp, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode", [0, 1])
def test_engine_fit_matches_oracle(device, mode):
    from src import synthetic
    from src.als_engine import DeviceALS

    n_users, n_items, dens, k = 500, 350, 0.06, 32
    csr = synthetic.generate(n_users, n_items, dens, False)
    csc = synthetic.generate(n_users, n_items, dens, True)
    eng = DeviceALS(n_users, n_items, k, 0.1, csr, csc, accum_mode=mode)
    eng.init_user_factors(synthetic.SEED_INIT)
    U0 = eng.user_factors.cpu().numpy().copy()
    eng.fit(5)
    ucsr = obuild.synth_csr(n_users, n_items, dens, 0, 0, n_users, synthetic.SEED, synthetic.SEED2)
    icsc = obuild.synth_csr(n_users, n_items, dens, 1, 0, n_items, synthetic.SEED, synthetic.SEED2)
    U, V = oals.fit(ucsr, icsc, U0, k, 0.1, 5, sweep=obuild.half_sweep)
    atol = 1e-5 if mode == 0 else 3e-5
    np.testing.assert_allclose(eng.user_factors.cpu().numpy(), U, rtol=1e-4, atol=atol)
    np.testing.assert_allclose(eng.item_factors.cpu().numpy(), V, rtol=1e-4, atol=atol)


# ---------------------------------------------------------------- scoring
@pytest.mark.parametrize("k,kp", [(10, 16), (64, 64), (45, 64)])
def test_als_score_bit_exact(device, k, kp):
    h = _hrec()
    rng = np.random.default_rng(k)
    U = np.zeros((40, kp), np.float32)
    V = np.zeros((600, kp), np.float32)
    U[:, :k] = rng.normal(size=(40, k))
    V[:, :k] = rng.normal(size=(600, k))
    Vt = h.transpose(torch.as_tensor(V, device=device))
    users = np.array([3, 0, -1, 39, 17] + list(range(20)), np.int64)
    items = rng.integers(-1, 600, 333).astype(np.int64)
    out = h.als_score(torch.as_tensor(U, device=device), torch.as_tensor(users, device=device), Vt,
                      torch.as_tensor(items, device=device), len(items), k).cpu().numpy()
    exp = oals.score_matrix(U[np.maximum(users, 0), :k], V[np.maximum(items, 0), :k])
    exp[users < 0, :] = np.nan
    exp[:, items < 0] = np.nan
    np.testing.assert_array_equal(out, exp)
    # all items, identity map
    full = h.als_score(torch.as_tensor(U, device=device), torch.as_tensor(users[:3], device=device), Vt,
                       None, 600, k).cpu().numpy()
    e2 = oals.score_matrix(U[np.maximum(users[:3], 0), :k], V[:, :k])
    e2[users[:3] < 0] = np.nan
    np.testing.assert_array_equal(full, e2)


# ------------------------------------------------------------------ top-k
def _stable_topk(row, k):
    order = sorted(range(len(row)), key=lambda i: (np.isnan(row[i]), -row[i] if not np.isnan(row[i]) else 0, i))
    return order[:k]


@pytest.mark.parametrize("n,k", [(1, 1), (7, 5), (4096, 10), (4097, 10), (70000, 5), (300, 64), (20, 30)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_topk_stable(device, n, k, dtype):
    h = _hrec()
    rng = np.random.default_rng(n + k)
    vals = np.round(rng.normal(size=(3, n)), 1)  # many ties
    idx, v = h.topk(torch.as_tensor(vals, dtype=dtype, device=device), k)
    for r in range(3):
        exp = _stable_topk(vals[r].astype(np.float32 if dtype == torch.float32 else np.float64), min(k, n))
        assert idx[r].cpu().tolist() == exp


@pytest.mark.parametrize("n", [1, 64, 65, 2048, 8192, 8193])
@pytest.mark.parametrize("k", [1, 2, 3, 8, 16, 17])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_topk_wave_path_ties_nan(device, n, k, dtype):
    """kk <= 16 over rows of <= 8192 run the wave-per-row kernel (csrc/score.hip
    topk_wave_kernel); kk = 17 and n = 8193 the block kernel: same order
    (larger first, ties -> smaller index, NaN last) either way."""
    h = _hrec()
    rng = np.random.default_rng(7 * n + k)
    vals = np.round(rng.normal(size=(9, n)), 1)
    vals[1, ::3] = np.nan
    vals[2, :] = 0.5  # one big tie
    vals[3, :] = np.nan
    npdt = np.float32 if dtype == torch.float32 else np.float64
    vals = vals.astype(npdt)
    idx, v = h.topk(torch.as_tensor(vals, device=device), k)
    kk = min(k, n)
    for r in range(vals.shape[0]):
        row = vals[r]
        exp = np.lexsort((np.arange(n), -np.nan_to_num(row, nan=0.0), np.isnan(row)))[:kk]
        assert idx[r].cpu().tolist() == exp.tolist(), r
        np.testing.assert_array_equal(v[r].cpu().numpy(), row[exp])


# ----------------------------------------------------------------- fusion
def _fuse_gpu(device, als_scores, tt_scores, als_wins, top_k):
    h = _hrec()
    a = torch.as_tensor(np.asarray(als_scores, np.float64), device=device)
    t = torch.as_tensor(np.asarray(tt_scores), device=device)
    idx, sc, fused = h.fuse_topk(a, t, als_wins, top_k)
    return idx.cpu().numpy(), sc.cpu().numpy(), fused.cpu().numpy()


@pytest.mark.parametrize("case", load_golden("fusion.json")["cases"], ids=lambda c: c["name"])
def test_fusion_gpu_vs_oracle_legacy(device, case):
    als = dec_pairs(case["als"])
    tt = dec_pairs(case["tt"])
    combined = ofus.adaptive_fusion(als, tt, case["als_f1"], case["tt_f1"], legacy=True)
    items = [i for i, _ in combined]
    ad, td = dict(als), dict(tt)
    a_arr = np.array([ad.get(i, 0) for i in items]).astype(np.float64)
    t_arr = np.array([td.get(i, 0) for i in items])
    if t_arr.dtype.kind in "iub":
        t_arr = t_arr.astype(np.float64)
    idx, sc, fused = _fuse_gpu(device, a_arr, t_arr, case["als_f1"] > case["tt_f1"], case["top_k"])
    np.testing.assert_array_equal(fused, np.array([s for _, s in combined], np.float64))
    top = ofus.top_k(combined, case["top_k"])
    assert [items[i] for i in idx] == [i for i, _ in top]
    np.testing.assert_array_equal(sc, np.array([s for _, s in top], np.float64))


def test_fusion_gpu_large_random(device):
    rng = np.random.default_rng(5)
    n = 100_000
    a = np.round(rng.normal(size=n) * 3, 2)
    t = rng.normal(size=n).astype(np.float32)
    pairs_a = list(zip(range(n), a.tolist()))
    pairs_t = list(zip(range(n), t))
    comb = ofus.adaptive_fusion(pairs_a, pairs_t, 0.0, 0.0, legacy=True)
    items = np.array([i for i, _ in comb])
    idx, sc, fused = _fuse_gpu(device, a[items], t[items], False, 10)
    np.testing.assert_array_equal(fused, np.array([s for _, s in comb]))
    assert items[idx].tolist() == [i for i, _ in ofus.top_k(comb, 10)]


@pytest.mark.parametrize("mode", [0, 1])
def test_engine_c2_shaped_fit_matches_oracle(device, mode):
    """Rank 64 on a c2-like matrix (long item rows ~ 900 ratings, user rows
    ~ 90), 5 epochs, against the C oracle: the tolerance the bench's
    accumulation mode must hold (rtol 1e-4)."""
    from src import synthetic
    from src.als_engine import DeviceALS

    n_users, n_items, dens, k = 10000, 1000, 0.09, 64
    csr = synthetic.generate(n_users, n_items, dens, False)
    csc = synthetic.generate(n_users, n_items, dens, True)
    eng = DeviceALS(n_users, n_items, k, 0.1, csr, csc, accum_mode=mode)
    eng.init_user_factors(synthetic.SEED_INIT)
    U0 = eng.user_factors.cpu().numpy().copy()
    eng.fit(5)
    ucsr = obuild.synth_csr(n_users, n_items, dens, 0, 0, n_users, synthetic.SEED, synthetic.SEED2)
    icsc = obuild.synth_csr(n_users, n_items, dens, 1, 0, n_items, synthetic.SEED, synthetic.SEED2)
    U, V = oals.fit(ucsr, icsc, U0, k, 0.1, 5, sweep=obuild.half_sweep)
    Ug, Vg = eng.user_factors.cpu().numpy(), eng.item_factors.cpu().numpy()
    np.testing.assert_allclose(Vg, V, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(Ug, U, rtol=1e-4, atol=1e-5)
    # predictions (what the API serves): rtol 1e-4 with an absolute floor of
    # 1e-6 x the largest score (scores near zero have no meaningful rtol)
    pred_g = (Ug[:200].astype(np.float64) @ Vg.T.astype(np.float64))
    pred_o = (U[:200].astype(np.float64) @ V.T.astype(np.float64))
    np.testing.assert_allclose(pred_g, pred_o, rtol=1e-4, atol=1e-6 * np.abs(pred_o).max())


def _np_stable_topk(scores, k):
    out = []
    for row in scores:
        order = np.lexsort((np.arange(len(row)), -row.astype(np.float64)))
        out.append(order[:k])
    return np.array(out)


@pytest.mark.parametrize("n_items,quant", [(100_000, False), (1500, False), (30_000, True)])
def test_als_score_topk_fused_matches_full(device, n_items, quant):
    """Fused threshold-filtered top-k == stable top-k of the full JVM-exact
    score matrix (bit-exact indices and values); quantised factors create
    massive ties and exercise the overflow fallback."""
    h = _hrec()
    rng = np.random.default_rng(n_items)
    k, kp, B = 64, 64, 40
    U = np.zeros((B, kp), np.float32)
    V = np.zeros((n_items, kp), np.float32)
    U[:, :k] = rng.normal(size=(B, k))
    V[:, :k] = rng.normal(size=(n_items, k))
    if quant:
        U[:, :k] = np.round(U[:, :k])
        V[:, :k] = np.round(V[:, :k] * 0.5)
    dU = torch.as_tensor(U, device=device)
    Vt = h.transpose(torch.as_tensor(V, device=device))
    users = torch.arange(B, dtype=torch.int64, device=device)
    idx, val = h.als_score_topk(dU, users, Vt, n_items, k, 10)
    full = oals.score_matrix(U[:, :k], V[:, :k])
    exp_i = _np_stable_topk(full, 10)
    np.testing.assert_array_equal(idx.cpu().numpy(), exp_i)
    np.testing.assert_array_equal(val.cpu().numpy(), np.take_along_axis(full, exp_i, 1))


def test_als_score_topk_overflow_flag(device):
    """The filter kernel raises the overflow flag itself when a user's
    survivors exceed the candidate list (constant scores: every item ties
    with the sampled bound) and leaves it 0 on random factors; the wrapper's
    fallback then still returns the exact stable top-k."""
    h = _hrec()
    n_items, k, kp, B = 100_000, 64, 64, 8
    rng = np.random.default_rng(3)
    U = np.zeros((B, kp), np.float32)
    U[:, :k] = rng.normal(size=(B, k))
    users = torch.arange(B, dtype=torch.int64, device=device)
    flag = torch.full((1,), 7, dtype=torch.int32, device=device)
    V = np.zeros((n_items, kp), np.float32)
    V[:, :k] = rng.normal(size=(n_items, k))
    Vt = h.transpose(torch.as_tensor(V, device=device))
    h.als_score_topk(torch.as_tensor(U, device=device), users, Vt, n_items, k, 5, check_overflow=False,
                     overflow_out=flag)
    assert int(flag.item()) == 0
    Vc = np.zeros((n_items, kp), np.float32)
    Vc[:, :k] = 0.25
    Vt = h.transpose(torch.as_tensor(Vc, device=device))
    idx, val = h.als_score_topk(torch.as_tensor(U, device=device), users, Vt, n_items, k, 5,
                                overflow_out=flag)
    assert int(flag.item()) == 1
    full = oals.score_matrix(U[:, :k], Vc[:, :k])
    exp_i = _np_stable_topk(full, 5)
    np.testing.assert_array_equal(idx.cpu().numpy(), exp_i)
    np.testing.assert_array_equal(val.cpu().numpy(), np.take_along_axis(full, exp_i, 1))


@pytest.mark.parametrize("n_items,k,kp,B,top_k,case", [
    (100_003, 64, 64, 40, 5, "normal"), (100_000, 64, 64, 17, 10, "quant"), (30_000, 16, 16, 9, 1, "normal"),
    (50_000, 100, 128, 12, 100, "normal"), (40_000, 200, 256, 8, 8, "scaled"), (3000, 64, 64, 5, 5, "normal"),
    (60_000, 64, 64, 10, 5, "unknown"), (60_000, 64, 64, 10, 5, "nan_item"), (60_000, 64, 64, 10, 5, "const"),
    (3000, 16, 16, 4, 1, "round_up"), (40_000, 16, 16, 4, 1, "round_up"), (40_000, 64, 64, 6, 3, "round_up"),
    (60_000, 64, 64, 10, 8, "const"), (60_000, 64, 64, 10, 3, "nan_item")])
def test_als_score_topk_pruned_matches_fused(device, n_items, k, kp, B, top_k, case):
    """hrec_als_score_topk_pruned (bf16 matrix-core bound, exact chain only
    for the pairs it keeps) returns the fused path's (ids, scores) bit for
    bit, and both equal the stable top-k of the full JVM-exact matrix:
    odd n, rank 16 / 64 / 100 (kp 128) / 200 (kp 256), top_k 1 .. 100,
    quantised factors (ties), factors scaled by 1e6, an unknown user row
    (the fused path's empty candidate list), a NaN item (no finite bound:
    overflow -> the exact fallback), constant items (list overflow) and
    components whose bf16 roundings all go the same way (the bound's worst
    case: 2^-8 relative per operand)."""
    h = _hrec()
    rng = np.random.default_rng(n_items + k)
    U = np.zeros((B, kp), np.float32)
    V = np.zeros((n_items, kp), np.float32)
    U[:, :k] = rng.normal(size=(B, k))
    V[:, :k] = rng.normal(size=(n_items, k))
    if case == "quant":
        U[:, :k] = np.round(U[:, :k])
        V[:, :k] = np.round(V[:, :k] * 0.5)
    if case == "scaled":
        U *= np.float32(1e6)
    if case == "nan_item":
        V[777, 3] = np.nan
    if case == "const":
        V[:, :k] = 0.25
    if case == "round_up":  # every bf16 rounding error aligned: 1 + 2^-8 + 2^-20 -> 1 + 2^-7,
        # so s~ of the best items overshoots their chain by ~2^-7 ||u|| ||v|| (the sample bound then sits
        # right at the kk-th chain); four tied best items in distinct sample tiles (the last past the
        # 32768-item sample), the rest far below
        x = np.float32(1 + 2.0 ** -8 + 2.0 ** -20)
        U[:, :k] = x
        V[:, :k] = 0.5
        V[[0, 100, 200, min(33_000, n_items - 1)], :k] = x
    dU = torch.as_tensor(U, device=device)
    dV = torch.as_tensor(V, device=device)
    Vt = h.transpose(dV)
    rows = np.arange(B, dtype=np.int64)
    if case == "unknown":
        rows[3] = -1
    users = torch.as_tensor(rows, device=device)
    ops = h.als_items_bf16(dV, k)
    flag_p = torch.full((1,), 7, dtype=torch.int32, device=device)
    flag_f = torch.full((1,), 7, dtype=torch.int32, device=device)
    pi, pv = h.als_score_topk_pruned(dU, users, Vt, dV, ops, n_items, k, top_k, check_overflow=False,
                                     overflow_out=flag_p)
    fi, fv = h.als_score_topk(dU, users, Vt, n_items, k, top_k, check_overflow=False, overflow_out=flag_f)
    fp, ff = int(flag_p.item()), int(flag_f.item())
    known = rows >= 0
    full = oals.score_matrix(U[known, :k], V[:, :k])
    exp_i = _np_stable_topk(full, min(top_k, n_items))
    if case in ("nan_item", "const"):
        assert fp == 1
    else:
        assert fp == ff == 0, (fp, ff)
        np.testing.assert_array_equal(pi.cpu().numpy(), fi.cpu().numpy())
        np.testing.assert_array_equal(pv.cpu().numpy().view(np.int32), fv.cpu().numpy().view(np.int32))
    if min(top_k, n_items) <= 8:  # resolved on the device inside the call, whatever the flag says
        np.testing.assert_array_equal(pi.cpu().numpy()[known], exp_i)
        np.testing.assert_array_equal(pv.cpu().numpy()[known].view(np.int32),
                                      np.take_along_axis(full, exp_i, 1).view(np.int32))
        if not known.all():
            assert (pi.cpu().numpy()[~known] == -1).all()
    # with the fallback resolved, both equal the full matrix's stable top-k
    pi, pv = h.als_score_topk_pruned(dU, users, Vt, dV, ops, n_items, k, top_k)
    got_i, got_v = pi.cpu().numpy()[known], pv.cpu().numpy()[known]
    np.testing.assert_array_equal(got_i, exp_i)
    np.testing.assert_array_equal(got_v.view(np.int32), np.take_along_axis(full, exp_i, 1).view(np.int32))


# ------------------------------------------------ multi-rank on one device
def _chunked_worker(rank, world, port, chunks, q, balanced=False):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src import synthetic
    from src.als_engine import DeviceALS, shard_chunks

    n_u, n_i, dens, k = 700, 300, 0.05, 32
    if balanced:  # nnz-balanced parts: padded shards, ids remapped on the device (hrec_remap_i32)
        from src.als_engine import RowLayout

        ul = RowLayout.balanced(synthetic.row_counts(n_u, n_i, dens, False).cpu().numpy(), world, chunks)
        il = RowLayout.balanced(synthetic.row_counts(n_u, n_i, dens, True).cpu().numpy(), world, 2)
        assert not ul.identity and not il.identity
        eng = DeviceALS(n_u, n_i, k, 0.1, synthetic.generate_layout(n_u, n_i, dens, False, ul, rank),
                        synthetic.generate_layout(n_u, n_i, dens, True, il, rank), world=world, rank=rank,
                        group=dist.group.WORLD, chunks=chunks, item_chunks=2, user_layout=ul, item_layout=il)
    else:
        ur, _ = shard_chunks(n_u, world, rank, chunks)
        ir, _ = shard_chunks(n_i, world, rank, 2)
        eng = DeviceALS(n_u, n_i, k, 0.1, synthetic.generate_ranges(n_u, n_i, dens, False, ur),
                        synthetic.generate_ranges(n_u, n_i, dens, True, ir), world=world, rank=rank,
                        group=dist.group.WORLD, chunks=chunks, item_chunks=2)
    eng.init_user_factors(synthetic.SEED_INIT)
    eng.fit(3)
    torch.cuda.synchronize()
    q.put((rank, eng.user_factors.cpu().numpy(), eng.item_factors.cpu().numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("balanced", [False, True])
def test_chunked_overlapped_allgather_on_device(device, balanced):
    """Two ranks on one GPU (gloo carries the all-gathers of device tensors):
    the chunk-interleaved shards (equal-count, or nnz-balanced with padded
    parts and device-remapped ids), HIP half-sweeps on the compute stream and
    per-chunk all-gathers on the side stream reproduce the single-rank fit
    bit for bit."""
    import socket

    import torch.multiprocessing as mp
    from src import synthetic
    from src.als_engine import DeviceALS

    n_u, n_i, dens, k = 700, 300, 0.05, 32
    ref = DeviceALS(n_u, n_i, k, 0.1, synthetic.generate(n_u, n_i, dens, False),
                    synthetic.generate(n_u, n_i, dens, True))
    ref.init_user_factors(synthetic.SEED_INIT)
    ref.fit(3)
    U, V = ref.user_factors.cpu().numpy(), ref.item_factors.cpu().numpy()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_chunked_worker, args=(r, 2, port, 3, q, balanced)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for _, Ur, Vr in res:
        np.testing.assert_array_equal(Ur, U)
        np.testing.assert_array_equal(Vr, V)
