"""CPU: pin the oracle against the reference's golden vectors and cross-check
its numpy / C restatements (no GPU)."""
import numpy as np
import pytest
from conftest import dec_pairs, dec_score, load_golden

from oracle import als as oals
from oracle import build as obuild
from oracle import fusion as ofus
from oracle import synth as osyn
from oracle import two_tower as ott


def _same(a, b):
    """Bit-exact scalar equality that also checks the numpy scalar kind."""
    return float(a) == float(b) and type(a) is type(b)


# ------------------------------------------------------------ fusion golden
@pytest.mark.parametrize("case", load_golden("fusion.json")["cases"], ids=lambda c: c["name"])
def test_fusion_oracle_matches_reference(case):
    meta = load_golden("fusion.json")["meta"]
    legacy = int(meta["numpy"].split(".")[0]) < 2  # fixtures record the numpy they ran under
    als = dec_pairs(case["als"])
    tt = dec_pairs(case["tt"])
    combined = ofus.adaptive_fusion(als, tt, case["als_f1"], case["tt_f1"], legacy=legacy)
    exp = dec_pairs(case["combined"])
    assert [i for i, _ in combined] == [i for i, _ in exp]
    for (_, a), (_, b) in zip(combined, exp):
        assert float(a) == float(b)
    top = ofus.top_k(combined, case["top_k"])
    assert [(i, float(s)) for i, s in top] == [(i, float(s)) for i, s in dec_pairs(case["top"])]


def test_f1_oracle_matches_reference():
    for rec in load_golden("f1.json")["cases"]:
        actual = {int(i): s for i, s in rec["actual"]}
        pred = {int(i): s for i, s in rec["pred"]}
        got = ofus.compute_f1_score(actual, pred, k=rec["k"])  # TT copy: guarded k > 0
        assert float(got) == rec["tt"]
        if rec["als"] != "ZeroDivisionError":
            assert float(got) == rec["als"]


def test_similar_items_oracle_matches_reference():
    for case in load_golden("similar_items.json")["cases"]:
        feats = {int(i): {"features": np.asarray(f, dtype=np.float64), "rating": r}
                 for i, f, r in case["item_features"]}
        for q in case["queries"]:
            assert ofus.find_similar_items(feats, q) == case["similar"][str(q)]


def test_als_fallback_oracle_matches_reference():
    for case in load_golden("als_fallback.json")["cases"]:
        feats = {int(i): {"features": np.asarray(f, dtype=np.float64), "rating": r}
                 for i, f, r in case["item_features"]}
        spark = {int(i): (np.nan if p is None else p) for i, p in case["spark_predictions"]}
        got = ofus.als_predict_with_fallback(spark, feats, case["global_mean"], case["query"])
        exp = dec_pairs(case["result"])
        assert len(got) == len(exp)
        for (gi, gs), (ei, es) in zip(got, exp):
            assert gi == ei and _same(gs, es)


def test_tt_numeric_inputs_oracle_matches_reference():
    for case in load_golden("tt_inputs.json")["cases"]:
        tr = np.column_stack([case["train"]["price"], case["train"]["average_review_rating"]])
        scale, min_, dmin, dmax = ott.scaler_fit(tr)
        assert dmin.tolist() == case["scaler_min"] and dmax.tolist() == case["scaler_max"]
        assert ott.scaler_transform(tr, scale, min_).tolist() == case["prepare_numeric_in"]
        cand = np.column_stack([case["candidates"]["price"], case["candidates"]["average_review_rating"]])
        assert ott.scaler_transform(cand, scale, min_).tolist() == case["inputs"]["numeric_in"]
        assert case["inputs"]["user_in"] == [31] * len(case["candidates"]["itemId"])
        assert case["inputs"]["item_id_in"] == case["candidates"]["itemId"]


def test_utils_known_answers():
    u = load_golden("utils.json")["cases"]
    assert u["scale_ratings_to_5"][0][1] == [1.0, 2.0, 3.0, 4.0, 5.0]
    items, exp = u["normalize_predictions"][0]
    got = ofus.minmax(np.array([s for _, s in items]))
    assert got.tolist() == [s for _, s in exp]


# ------------------------------------------------------------------ synth
def test_synth_numpy_matches_c():
    for transposed in (0, 1):
        a = osyn.csr_rows(300, 200, 0.05, transposed, 7, 40, 11, 12)
        b = obuild.synth_csr(300, 200, 0.05, transposed, 7, 40, 11, 12)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)


def test_synth_csr_csc_are_transposes():
    U, I = 120, 90
    csr = obuild.synth_csr(U, I, 0.08, 0, 0, U, 3, 4)
    csc = obuild.synth_csr(U, I, 0.08, 1, 0, I, 3, 4)
    dense_r = np.zeros((U, I), np.float32)
    mask_r = np.zeros((U, I), bool)
    for u in range(U):
        c = csr[1][csr[0][u]:csr[0][u + 1]]
        dense_r[u, c] = csr[2][csr[0][u]:csr[0][u + 1]]
        mask_r[u, c] = True
    mask_c = np.zeros((U, I), bool)
    dense_c = np.zeros((U, I), np.float32)
    for i in range(I):
        c = csc[1][csc[0][i]:csc[0][i + 1]]
        dense_c[c, i] = csc[2][csc[0][i]:csc[0][i + 1]]
        mask_c[c, i] = True
    assert (mask_r == mask_c).all() and (dense_r == dense_c).all()
    assert 0.04 < mask_r.mean() < 0.12
    assert set(np.unique(csr[2])) <= set(range(19))


def test_init_factors_unit_norm():
    f = osyn.init_factors(7, 5, 6, 10)
    np.testing.assert_allclose(np.linalg.norm(f.astype(np.float64), axis=1), 1.0, rtol=1e-6)


# -------------------------------------------------------------------- ALS
def _small_problem(seed=0, n_rows=25, n_src=30, k=8):
    rng = np.random.default_rng(seed)
    deg = rng.integers(0, 12, n_rows)
    indptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    indices = rng.integers(0, n_src, indptr[-1]).astype(np.int32)
    values = rng.integers(0, 19, indptr[-1]).astype(np.float32)
    src = rng.normal(size=(n_src, k)).astype(np.float32)
    return indptr, indices, values, src


def test_als_spark_restatement_variants_agree():
    indptr, indices, values, src = _small_problem()
    a = oals.half_sweep_spark(indptr, indices, values, src, 8, 0.1)
    b = oals.half_sweep_blas(indptr, indices, values, src, 8, 0.1)
    c = obuild.half_sweep(indptr, indices, values, src, 8, 0.1)
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(a, c, rtol=1e-5, atol=1e-6)
    empty = np.diff(indptr) == 0
    assert (a[empty] == 0).all() and (c[empty] == 0).all()


def test_als_rank1_known_answer():
    # k = 1: x = sum(r v) / (sum(v^2) + reg * n), in closed form.
    indptr = np.array([0, 3], np.int64)
    indices = np.array([0, 1, 1], np.int32)  # duplicate rating counts twice (Spark keeps both)
    values = np.array([4.0, 0.0, 2.0], np.float32)
    src = np.array([[0.5], [2.0]], np.float32)
    x = oals.half_sweep_spark(indptr, indices, values, src, 1, 0.1)
    expect = (4 * 0.5 + 0 * 2.0 + 2 * 2.0) / (0.25 + 4 + 4 + 0.1 * 3)
    assert abs(float(x[0, 0]) - expect) < 1e-7
    assert float(obuild.half_sweep(indptr, indices, values, src, 1, 0.1)[0, 0]) == float(x[0, 0])


def test_als_normal_equation_residual():
    indptr, indices, values, src = _small_problem(seed=3, k=16)
    x = obuild.half_sweep(indptr, indices, values, src, 16, 0.05)
    for r in range(len(indptr) - 1):
        b, e = indptr[r], indptr[r + 1]
        if b == e:
            continue
        V = src[indices[b:e]].astype(np.float64)
        A = V.T @ V + 0.05 * (e - b) * np.eye(16)
        rhs = V.T @ values[b:e].astype(np.float64)
        np.testing.assert_allclose(A @ x[r].astype(np.float64), rhs, rtol=1e-5, atol=1e-5)


def test_als_score_matrix_matches_scalar_predict():
    rng = np.random.default_rng(1)
    U = rng.normal(size=(4, 12)).astype(np.float32)
    V = rng.normal(size=(9, 12)).astype(np.float32)
    m = oals.score_matrix(U, V)
    users = np.repeat(np.arange(4), 9)
    items = np.tile(np.arange(9), 4)
    np.testing.assert_array_equal(m.reshape(-1), oals.predict(U, V, users, items))


# -------------------------------------------------------------- two-tower
def test_tt_oracle_gradcheck():
    """The two-tower backward restatement against central finite differences."""
    rng = np.random.default_rng(2)
    d, B = 6, 5
    p = {
        "user_emb": rng.normal(size=(4, d)), "item_emb": rng.normal(size=(5, d)),
        "man_emb": rng.normal(size=(3, 8)), "cat_emb": rng.normal(size=(2, 8)),
        "w1": rng.normal(size=(2, 16)), "b1": rng.normal(size=16),
        "w2": rng.normal(size=(d + 32, d)) * 0.3, "b2": rng.normal(size=d),
        "ln_user_gamma": 1 + 0.2 * rng.normal(size=d), "ln_user_beta": rng.normal(size=d),
        "ln_item_gamma": 1 + 0.2 * rng.normal(size=d), "ln_item_beta": rng.normal(size=d),
    }
    user = np.array([0, 1, 1, 3, 2])
    item = np.array([4, 0, 4, 2, 1])
    man = np.array([0, 2, 1, 1, 0])
    cat = np.array([1, 0, 1, 1, 0])
    x = rng.uniform(0, 1, (B, 2))
    y = rng.integers(0, 19, B).astype(np.float64)

    def loss(q):
        c = ott.forward(q, user, item, man, cat, x)
        return float(((c["yhat"] - y) ** 2).mean())

    c = ott.forward(p, user, item, man, cat, x)
    grads, rows, _, _ = ott.backward(p, c, y)
    # scatter the per-sample rows into dense table grads
    for name, idx in (("user_emb", user), ("item_emb", item), ("man_emb", man), ("cat_emb", cat)):
        g = np.zeros_like(p[name])
        np.add.at(g, idx, rows[name])
        grads[name] = g
    h = 1e-6
    for name in p:
        it = np.nditer(p[name], flags=["multi_index"])
        for _ in it:
            ix = it.multi_index
            q1 = {k: v.copy() for k, v in p.items()}
            q2 = {k: v.copy() for k, v in p.items()}
            q1[name][ix] += h
            q2[name][ix] -= h
            fd = (loss(q1) - loss(q2)) / (2 * h)
            assert abs(fd - grads[name][ix]) <= 1e-5 * max(1.0, abs(fd)), (name, ix, fd, grads[name][ix])


def test_c_score_topk_matches_jvm_predict():
    """oracle_score_topk (bench's scoring cpu_baseline): the JVM-exact f32 dot
    of oracle/als.score_matrix + Python's stable sorted(reverse=True)[:k],
    ties included."""
    obuild.build()
    rng = np.random.default_rng(4)
    U = rng.normal(size=(40, 24)).astype(np.float32)
    V = rng.normal(size=(517, 24)).astype(np.float32)
    V[200] = V[7]  # exact tie: the earlier item wins
    rows = np.array([0, 3, 39, 17])
    idx, val = obuild.score_topk(U, rows, V, 24, 9)
    S = oals.score_matrix(U[rows], V)
    for r in range(len(rows)):
        order = sorted(range(V.shape[0]), key=lambda j: S[r, j], reverse=True)[:9]
        assert idx[r].tolist() == order
        assert np.array_equal(val[r], S[r, order])


def test_cpu_baseline_keras_step_matches_oracle():
    """The torch-CPU Keras train step timed as bench's tt_train cpu_baseline
    computes what the f64 two-tower oracle computes (3 steps, rtol 1e-4)."""
    import torch

    from oracle import cpu_baseline as cb

    d, sizes = 16, (30, 25, 6, 5)
    g = torch.Generator().manual_seed(2)
    p = cb._init(sizes, d, g)
    p["gi"] += 0.1 * torch.rand(d, generator=g)
    p["b2"] += 0.1 * torch.rand(d, generator=g)
    names = {"gi": "ln_item_gamma", "bi": "ln_item_beta", "gu": "ln_user_gamma", "bu": "ln_user_beta"}
    po = {names.get(n, n): t.numpy().astype(np.float32).copy() for n, t in p.items()}
    slots = {n: (torch.zeros_like(t), torch.zeros_like(t)) for n, t in p.items()}
    so = {n: (np.zeros_like(t), np.zeros_like(t)) for n, t in po.items()}
    rng = np.random.default_rng(3)
    for it in range(3):
        B = 12
        u, i = rng.integers(0, sizes[0], B), rng.integers(0, sizes[1], B)
        m, c = rng.integers(0, sizes[2], B), rng.integers(0, sizes[3], B)
        u[1] = u[0]  # a duplicated row (IndexedSlices dedup)
        x = rng.random((B, 2)).astype(np.float32)
        y = rng.integers(0, 19, B).astype(np.float32)
        t = [torch.as_tensor(a) for a in (u, i, m, c, x, y)]
        cb.keras_step(p, slots, it, *t)
        ott.train_step(po, so, u, i, m, c, x, y, it)
    for n, t in p.items():
        np.testing.assert_allclose(t.numpy(), po[names.get(n, n)], rtol=1e-4, atol=1e-6, err_msg=n)


def _numpy_fusion(als, tt, als_wins, promotion):
    """The reference's adaptive_fusion arithmetic (src/hybrid_system.py:62-72)
    written with numpy + sklearn directly on arrays in candidate order: als
    float64 (Python floats), tt float32 (np.float32 Keras scores), one
    MinMaxScaler.fit_transform per model, then w0 * als_norm[i] + w1 *
    tt_norm[i] per item. promotion "1.21": w1 * np.float32 -> float64 (numpy
    1.21.5, requirements.txt:5, value-based casting of the Python float);
    "2": NEP 50, the float32 product numpy >= 2 computes."""
    from sklearn.preprocessing import MinMaxScaler

    a = MinMaxScaler().fit_transform(np.asarray(als, np.float64).reshape(-1, 1)).flatten()
    t = MinMaxScaler().fit_transform(np.asarray(tt, np.float32).reshape(-1, 1)).flatten()
    w = (0.8, 0.2) if als_wins else (0.2, 0.8)
    if promotion == "1.21":
        return w[0] * a + w[1] * t.astype(np.float64)
    return w[0] * a + (np.float32(w[1]) * t).astype(np.float64)


@pytest.mark.parametrize("als_wins", [True, False])
def test_fusion_oracle_matches_numpy_sklearn(als_wins):
    """oracle.fusion.adaptive_fusion (the restatement the device fusion is
    checked against) == the numpy/sklearn arithmetic above: legacy=True is
    numpy 1.21's promotion bit for bit, legacy=False numpy 2's (the container
    runs numpy 2, so the latter is also exactly what the reference's own
    Python computes here)."""
    rng = np.random.default_rng(3 + als_wins)
    n = 3000
    ids = list(range(n))
    als = rng.normal(size=n) * 2
    tt = (rng.normal(size=n) * 3).astype(np.float32)
    tt[::50] = tt[0]   # ties
    for legacy, promo in ((True, "1.21"), (False, "2")):
        got = ofus.adaptive_fusion(list(zip(ids, als.tolist())), list(zip(ids, tt)), *((0.5, 0.1) if als_wins
                                   else (0.1, 0.5)), legacy=legacy)
        assert [i for i, _ in got] == ids   # dense ids: the set union iterates ascending
        np.testing.assert_array_equal(np.array([s for _, s in got], np.float64),
                                      _numpy_fusion(als, tt, als_wins, promo))


def test_parity_rule_decided_positions():
    """tests/parity_rules.py (the served-ranking rule of the trained-model GPU
    tests): a position is decided iff its item cannot trade places with any
    other under the tolerances; a swap at a decided position fails, one
    inside an undecided tie passes."""
    from parity_rules import check_served, decided_positions

    o = np.array([5.0, 9.0, 7.0, 7.00001, 1.0, 3.0])
    t = np.full(6, 1e-3)
    order, dec = decided_positions(o, t, 4)
    assert order.tolist() == [1, 3, 2, 0, 5, 4]
    assert dec.tolist() == [True, False, False, True]
    ids = list("abcdef")
    assert check_served(["b", "c", "d", "a"], ids, o, t, 4) is False   # the 7 / 7.00001 tie may swap
    with pytest.raises(AssertionError):
        check_served(["c", "b", "d", "a"], ids, o, t, 4)                # position 0 is decided
    assert check_served(["b", "d", "c", "a"], ids, o, np.full(6, 1e-9), 4) is True
