"""GPU: the drop-in API (src.als_model / src.two_tower_model / src.hybrid_system)
through the C-ABI, against the oracle and the reference's golden vectors.

Tolerances: ALS factors rtol 1e-4 after max_iter epochs (f64 Gramian, other
summation order); ALS scores and fusion bit-exact; two-tower forward rtol
1e-5 and gradients / parameters after Adam steps rtol 1e-4 against a float64
restatement of the Keras graph (GPU computes in f32, as Keras does).
"""
import numpy as np
from sklearn.preprocessing import MinMaxScaler
import pandas as pd
import pytest
import torch
from conftest import dec_pairs, load_golden

from oracle import als as oals
from oracle import build as obuild
from oracle import fusion as ofus
from oracle import two_tower as ott

pytestmark = pytest.mark.gpu


# --------------------------------------------------------------------- ALS
def _ratings_frame(rng, n_users=60, n_items=45, n=900):
    users = rng.integers(0, n_users, n) * 7 + 3      # sparse raw ids
    items = rng.integers(0, n_items, n) * 5 + 11
    return pd.DataFrame({
        "userId": users, "itemId": items,
        "average_review_rating": rng.integers(0, 19, n),
        "price": np.round(rng.uniform(1, 300, n), 2),
        "manufacturer_id": rng.integers(0, 9, n), "category_id": rng.integers(0, 5, n),
    })


def _frame_csr(df):
    u_ids, urow = np.unique(df["userId"].to_numpy(), return_inverse=True)
    i_ids, irow = np.unique(df["itemId"].to_numpy(), return_inverse=True)
    r = df["average_review_rating"].to_numpy().astype(np.float32)

    def csr(rows, cols, n):
        order = np.argsort(rows, kind="stable")
        ip = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=n))]).astype(np.int64)
        return ip, cols[order].astype(np.int32), r[order]

    return u_ids, i_ids, csr(urow, irow, len(u_ids)), csr(irow, urow, len(i_ids))


@pytest.mark.parametrize("k", [10, 100])
def test_als_train_matches_oracle(device, k):
    """rank 10 (the reference's grid, src/als_model.py:185-191) and rank 100
    (one workgroup per row, csrc/als_wide.hip) through the drop-in API."""
    from src.als_model import ALSModel

    rng = np.random.default_rng(0)
    df = _ratings_frame(rng)
    u_ids, i_ids, ucsr, icsc = _frame_csr(df)
    U0 = rng.normal(size=(len(u_ids), k)).astype(np.float32)
    U0 /= np.linalg.norm(U0, axis=1, keepdims=True)
    m = ALSModel(rank=k, max_iter=10, reg_param=0.1)
    assert m.train(df, initial_user_factors=U0) is True
    U, V = oals.fit(ucsr, icsc, U0, k, 0.1, 10, sweep=obuild.half_sweep)
    np.testing.assert_allclose(m.model.U[:, :k].cpu().numpy(), U, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(m.model.V[:, :k].cpu().numpy(), V, rtol=1e-4, atol=1e-5)
    assert m.global_mean == df["average_review_rating"].mean()

    # predict_for_user: known items bit-exact (JVM f32 dot), unknown -> fallback
    uid = int(u_ids[3])
    query = list(i_ids[:20]) + [999999, int(i_ids[5])]
    got = m.predict_for_user(uid, query)
    Ug = m.model.U[:, :k].cpu().numpy()
    Vg = m.model.V[:, :k].cpu().numpy()
    row = oals.score_matrix(Ug[3:4], Vg)[0]
    spark = {int(i): float(row[n]) for n, i in enumerate(i_ids)}
    exp = ofus.als_predict_with_fallback(spark, m.item_features, m.global_mean, query)
    assert [i for i, _ in got] == [i for i, _ in exp]
    for (_, a), (_, b) in zip(got, exp):
        assert float(a) == float(b)

    # unknown user -> every item through the fallback
    got = m.predict_for_user(-5, query[:6])
    exp = ofus.als_predict_with_fallback({}, m.item_features, m.global_mean, query[:6])
    assert [float(s) for _, s in got] == [float(s) for _, s in exp]


def test_als_train_error_sentinel(device, capsys):
    from src.als_model import ALSModel

    m = ALSModel(rank=8)
    assert m.train(pd.DataFrame({"userId": [0.5], "itemId": [1], "average_review_rating": [3]})) is False
    assert "Training error" in capsys.readouterr().out
    assert m.predict_for_user(1, [1, 2]) == []  # no model -> reference sentinel


def _rank1_model(device, item_scores, item_features, global_mean):
    """A fitted model whose JVM-order dot reproduces given predictions (k=1,
    U = [1.0]: 0 + 1*v is exact)."""
    from src.als_model import ALSModel, DeviceALSFactors

    ids = np.array(sorted(item_scores), dtype=np.int64)
    V = torch.zeros((len(ids), 16), dtype=torch.float32, device=device)
    V[:, 0] = torch.as_tensor(np.array([item_scores[i] for i in ids], np.float32))
    U = torch.zeros((1, 16), dtype=torch.float32, device=device)
    U[0, 0] = 1.0
    m = ALSModel(rank=1)
    m.initialize_spark()
    m.model = DeviceALSFactors(np.array([7]), ids, U, V, 1)
    m.item_features = item_features
    m.global_mean = global_mean
    return m


def test_als_fallback_golden(device):
    for case in load_golden("als_fallback.json")["cases"]:
        feats = {int(i): {"features": np.asarray(f, dtype=np.float64), "rating": r}
                 for i, f, r in case["item_features"]}
        known = {int(i): p for i, p in case["spark_predictions"] if p is not None}
        m = _rank1_model(device, known, feats, case["global_mean"])
        got = m.predict_for_user(7, case["query"])
        exp = dec_pairs(case["result"])
        assert [i for i, _ in got] == [i for i, _ in exp]
        for (_, a), (_, b) in zip(got, exp):
            assert float(a) == float(b) and type(a) is type(b)


def test_similar_items_golden(device):
    from src.als_model import ALSModel

    for case in load_golden("similar_items.json")["cases"]:
        m = ALSModel()
        m.initialize_spark()
        m.item_features = {int(i): {"features": np.asarray(f, dtype=np.float64), "rating": r}
                           for i, f, r in case["item_features"]}
        for q in case["queries"]:
            assert m._find_similar_items(q) == case["similar"][str(q)]


def test_als_save_load_roundtrip(device, tmp_path):
    from src.als_model import ALSModel

    rng = np.random.default_rng(1)
    df = _ratings_frame(rng, 30, 20, 300)
    m = ALSModel(rank=6, max_iter=3, seed=3)
    assert m.train(df)
    path = str(tmp_path / "models" / "als")
    m.save_model(path)
    m2 = ALSModel().load_model(path)
    assert m2 is not None and m2.rank == 6 and m2.global_mean == m.global_mean
    q = list(df["itemId"].unique()[:10])
    assert m.predict_for_user(int(df["userId"].iloc[0]), q) == m2.predict_for_user(int(df["userId"].iloc[0]), q)
    assert ALSModel().load_model(str(tmp_path / "missing")) is None


def test_als_model_dir_is_spark_layout(device, tmp_path):
    """save_model writes Spark 3.5's ALSModel directory (metadata JSON line +
    userFactors/itemFactors parquet of (id int, features array<float>)); a
    directory laid out like Spark's (several part files, rows in arbitrary
    order) loads back to the same model."""
    import json

    import pyarrow as pa
    import pyarrow.parquet as pq
    from src.als_model import ALSModel

    rng = np.random.default_rng(2)
    df = _ratings_frame(rng, 25, 15, 200)
    m = ALSModel(rank=5, max_iter=2, seed=4)
    assert m.train(df)
    path = tmp_path / "als"
    m.save_model(str(path))
    meta = json.loads((path / "metadata" / "part-00000").read_text().splitlines()[0])
    assert meta["class"] == "org.apache.spark.ml.recommendation.ALSModel" and meta["rank"] == 5
    assert meta["paramMap"]["userCol"] == "userId" and meta["paramMap"]["itemCol"] == "itemId"
    t = pq.read_table(str(path / "userFactors"))
    assert t.schema.field("id").type == pa.int32()
    assert t.schema.field("features").type.value_type == pa.float32()
    ids = t.column("id").to_numpy()
    feats = np.stack([np.asarray(x, np.float32) for x in t.column("features").to_pylist()])
    np.testing.assert_array_equal(feats, m.model.U[:, :5].cpu().numpy())
    # re-write userFactors as two shuffled part files, as Spark's partitions would be
    perm = rng.permutation(len(ids))
    for f in (path / "userFactors").glob("*.parquet"):
        f.unlink()
    for n, part in enumerate(np.array_split(perm, 2)):
        pq.write_table(pa.table({"id": pa.array(ids[part], pa.int32()),
                                 "features": pa.array([feats[i].tolist() for i in part], pa.list_(pa.float32()))}),
                       str(path / "userFactors" / f"part-0000{n}-x.snappy.parquet"))
    m2 = ALSModel().load_model(str(path))
    assert m2 is not None
    q = list(df["itemId"].unique()[:8])
    for u in df["userId"].unique()[:5]:
        assert m.predict_for_user(int(u), q) == m2.predict_for_user(int(u), q)


# --------------------------------------------------------------- two-tower
def _tt_params(rng, nu, ni, nm, nc, d):
    p = ott_init = {
        "user_emb": rng.uniform(-0.5, 0.5, (nu, d)), "item_emb": rng.uniform(-0.5, 0.5, (ni, d)),
        "man_emb": rng.uniform(-0.5, 0.5, (nm, 8)), "cat_emb": rng.uniform(-0.5, 0.5, (nc, 8)),
        "w1": rng.normal(size=(2, 16)), "b1": rng.normal(size=16) * 0.1,
        "w2": rng.normal(size=(d + 32, d)) * 0.2, "b2": rng.normal(size=d) * 0.1,
        "ln_user_gamma": 1 + 0.1 * rng.normal(size=d), "ln_user_beta": 0.1 * rng.normal(size=d),
        "ln_item_gamma": 1 + 0.1 * rng.normal(size=d), "ln_item_beta": 0.1 * rng.normal(size=d),
    }
    return {k: np.asarray(v, np.float32) for k, v in ott_init.items()}


def _tt_batch(rng, B, nu, ni, nm, nc):
    return (rng.integers(0, nu, B).astype(np.int32), rng.integers(0, ni, B).astype(np.int32),
            rng.integers(0, nm, B).astype(np.int32), rng.integers(0, nc, B).astype(np.int32),
            rng.uniform(0, 1, (B, 2)).astype(np.float32), rng.integers(0, 19, B).astype(np.float32))


@pytest.mark.parametrize("d", [16, 50, 64, 128, 256])
def test_tt_forward_backward_matches_oracle(device, d):
    from src import _hrec
    from src.tt_engine import DeviceTwoTower

    rng = np.random.default_rng(d)
    nu, ni, nm, nc, B = 40, 30, 7, 5, 77
    p = _tt_params(rng, nu, ni, nm, nc, d)
    eng = DeviceTwoTower(nu, ni, nm, nc, d, init=p)
    u, i, m, c, x, y = _tt_batch(rng, B, nu, ni, nm, nc)
    T = lambda a: torch.as_tensor(a, device=device)  # noqa: E731
    cache = ott.forward(p, u, i, m, c, x)
    np.testing.assert_allclose(eng.user_vectors(T(u)).cpu().numpy(), cache["uvec"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(eng.item_vectors(T(i), T(m), T(c), T(x)).cpu().numpy(), cache["ivec"],
                               rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(eng.predict_rows(T(u), T(i), T(m), T(c), T(x)).cpu().numpy(), cache["yhat"],
                               rtol=1e-5, atol=1e-4)
    gd, gu, gi, gm, gc = _hrec.tt_forward_backward(eng.params, T(u), T(i), T(m), T(c), T(x), T(y))
    grads, rows, sq, ab = ott.backward(p, cache, y)
    gd = gd.cpu().numpy()
    for name, (off, shape) in eng.layout.items():
        got = gd[off: off + int(np.prod(shape))].reshape(shape)
        scale = np.abs(grads[name]).max() + 1e-12
        np.testing.assert_allclose(got, grads[name], rtol=1e-4, atol=1e-4 * scale, err_msg=name)
    for name, g in (("user_emb", gu), ("item_emb", gi), ("man_emb", gm), ("cat_emb", gc)):
        scale = np.abs(rows[name]).max() + 1e-12
        np.testing.assert_allclose(g.cpu().numpy(), rows[name], rtol=1e-4, atol=1e-4 * scale, err_msg=name)
    np.testing.assert_allclose(gd[eng.n_dense:], [sq, ab], rtol=1e-5)


@pytest.mark.parametrize("d,n", [(16, 1), (50, 77), (64, 1000), (100, 333), (128, 4099), (256, 530)])
def test_tt_item_tower_mfma_matches_oracle(device, d, n):
    """K4m (csrc/tt_mfma.hip, f32 matrix cores, permuted-k Dense + fused LN)
    against the f64 Keras graph at rtol 1e-5, ragged tails and padded d
    included."""
    from src import _hrec
    from src.tt_engine import DeviceTwoTower

    rng = np.random.default_rng(d * 7 + n)
    nu, ni, nm, nc = 5, 3000, 11, 6
    p = _tt_params(rng, nu, ni, nm, nc, d)
    eng = DeviceTwoTower(nu, ni, nm, nc, d, init=p)
    u, i, m, c, x, _ = _tt_batch(rng, n, nu, ni, nm, nc)
    T = lambda a: torch.as_tensor(a, device=device)  # noqa: E731
    got = eng.item_vectors(T(i), T(m), T(c), T(x)).cpu().numpy()
    want = ott.forward(p, u, i, m, c, x)["ivec"]
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=2e-5)


def test_tt_item_tower_mfma_catalogue_sample(device):
    """A catalogue-sized call (1M items, d = 128, many persistent-loop trips
    per wave): sampled rows against the f64 graph, every row LayerNormed
    (mean = mean(beta) when gamma = 1)."""
    from src.tt_engine import DeviceTwoTower

    rng = np.random.default_rng(5)
    n, d, nm, nc = 1_000_000, 128, 2651, 255
    p = _tt_params(rng, 2, n, nm, nc, d)
    p["ln_item_gamma"][:] = 1.0
    eng = DeviceTwoTower(2, n, nm, nc, d, init=p)
    i = torch.arange(n, dtype=torch.int32, device=device)
    m = torch.as_tensor(rng.integers(0, nm, n).astype(np.int32), device=device)
    c = torch.as_tensor(rng.integers(0, nc, n).astype(np.int32), device=device)
    x = torch.as_tensor(rng.uniform(0, 1, (n, 2)).astype(np.float32), device=device)
    iv = eng.item_vectors(i, m, c, x)
    mu = iv.double().mean(1).cpu().numpy()
    np.testing.assert_allclose(mu, float(p["ln_item_beta"].astype(np.float64).mean()), atol=1e-5)
    rows = np.unique(np.concatenate([rng.integers(0, n, 500), [0, 15, 16, n - 17, n - 1]]))
    want = ott.forward(p, np.zeros(len(rows), np.int64), rows, m.cpu().numpy()[rows], c.cpu().numpy()[rows],
                       x.cpu().numpy()[rows])["ivec"]
    np.testing.assert_allclose(iv[torch.as_tensor(rows, device=device)].cpu().numpy(), want, rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("d,B", [(16, 1), (64, 256), (50, 77), (128, 300), (256, 40)])
def test_tt_backward_mfma_shapes_match_oracle(device, d, B):
    """K6m (dz and dW2 on the f32 matrix cores, column sums in one pass) at
    the batch shapes of its tilings (one sample, ragged, several sample
    stripes) against the f64 Keras graph's gradients (oracle/two_tower.py,
    checked against finite differences) at rtol 1e-4."""
    from src import _hrec
    from src.tt_engine import DeviceTwoTower

    rng = np.random.default_rng(d + B)
    nu, ni, nm, nc = 40, 30, 7, 5
    p = _tt_params(rng, nu, ni, nm, nc, d)
    eng = DeviceTwoTower(nu, ni, nm, nc, d, init=p)
    u, i, m, c, x, y = _tt_batch(rng, B, nu, ni, nm, nc)
    T = lambda a: torch.as_tensor(a, device=device)  # noqa: E731
    gd, gu, gi, gm, gc = _hrec.tt_forward_backward(eng.params, T(u), T(i), T(m), T(c), T(x), T(y))
    grads, rows, sq, ab = ott.backward(p, ott.forward(p, u, i, m, c, x), y)
    gd = gd.cpu().numpy()
    for name, (off, shape) in eng.layout.items():
        got = gd[off: off + int(np.prod(shape))].reshape(shape)
        scale = np.abs(grads[name]).max() + 1e-12
        np.testing.assert_allclose(got, grads[name], rtol=1e-4, atol=1e-4 * scale, err_msg=name)
    for name, g in (("user_emb", gu), ("item_emb", gi), ("man_emb", gm), ("cat_emb", gc)):
        scale = np.abs(rows[name]).max() + 1e-12
        np.testing.assert_allclose(g.cpu().numpy(), rows[name], rtol=1e-4, atol=1e-4 * scale, err_msg=name)


def test_tt_adam_steps_match_oracle(device):
    from src.tt_engine import TABLES, DeviceTwoTower

    rng = np.random.default_rng(9)
    nu, ni, nm, nc, d, B = 25, 20, 4, 3, 32, 64
    p = _tt_params(rng, nu, ni, nm, nc, d)
    eng = DeviceTwoTower(nu, ni, nm, nc, d, learning_rate=0.01, init=p)
    pref = {k: v.copy() for k, v in p.items()}
    slots = {k: (np.zeros_like(v), np.zeros_like(v)) for k, v in pref.items()}
    T = lambda a: torch.as_tensor(a, device=device)  # noqa: E731
    for it in range(6):
        u, i, m, c, x, y = _tt_batch(rng, B, nu, ni, nm, nc)  # many duplicate ids per batch
        eng.train_step(T(u), T(i), T(m), T(c), T(x), T(y))
        ott.train_step(pref, slots, u, i, m, c, x, y, it, lr=0.01)
    for name in list(ott.DENSE) + list(TABLES):
        np.testing.assert_allclose(eng.tensors[name].cpu().numpy(), pref[name], rtol=1e-4, atol=2e-6,
                                   err_msg=name)


@pytest.mark.parametrize("B,dim,n_rows", [(300, 80, 7), (257, 8, 2651), (64, 64, 1)])
def test_sparse_adam_dedup_order(device, B, dim, n_rows):
    """Duplicate ids of a batch are summed in batch order (TF's
    unsorted_segment_sum over the IndexedSlices) before the slot update: with
    beta_1 = 0, m of a touched row is exactly that ordered f32 sum. Covers
    batches past one 64-slot ballot, rows wider than a wave and all-equal ids."""
    from src import _hrec as h

    rng = np.random.default_rng(B + dim)
    idx = rng.integers(0, n_rows, B).astype(np.int32)
    g = rng.normal(size=(B, dim)).astype(np.float32)
    exp = {}
    for t in range(B):  # sequential f32 sums in batch order
        exp[idx[t]] = g[t].copy() if idx[t] not in exp else (exp[idx[t]] + g[t]).astype(np.float32)
    T = lambda a: torch.as_tensor(a, device=device)  # noqa: E731
    var = T(np.zeros((n_rows, dim), np.float32))
    m = T(np.full((n_rows, dim), 5.0, np.float32))
    v = T(np.ones((n_rows, dim), np.float32))
    mark = T(np.full(n_rows, -1, np.int32))
    gsum = torch.empty((B, dim), dtype=torch.float32, device=device)
    h.adam_sparse(var, m, v, T(idx), T(g), mark, gsum, 0.0, 0.0, 1.0, 0.0, 1.0, 1.0)
    mh = m.cpu().numpy()
    for r in range(n_rows):
        np.testing.assert_array_equal(mh[r], exp[r] if r in exp else np.zeros(dim, np.float32), err_msg=str(r))
    assert (mark.cpu().numpy() == -1).all()  # unmarked again for the next step


def test_sparse_adam_grouped_matches_per_table(device):
    """hrec_adam_sparse_tables (3 launches for all tables) == hrec_adam_sparse
    per table, bit for bit, incl. an empty batch and mixed row widths."""
    from src import _hrec as h

    rng = np.random.default_rng(21)
    shapes = [(1000, 64, 256), (300, 64, 256), (40, 8, 256), (7, 8, 0)]
    T = lambda a: torch.as_tensor(a, device=device)  # noqa: E731
    runs = []
    for _ in range(2):
        runs.append([])
    for n_rows, dim, B in shapes:
        var = rng.normal(size=(n_rows, dim)).astype(np.float32)
        m = rng.normal(size=(n_rows, dim)).astype(np.float32)
        v = rng.uniform(0, 1, size=(n_rows, dim)).astype(np.float32)
        idx = rng.integers(0, n_rows, B).astype(np.int32)
        g = rng.normal(size=(B, dim)).astype(np.float32)
        for run in runs:
            run.append((T(var), T(m), T(v), T(idx), T(g), T(np.full(n_rows, -1, np.int32)),
                        torch.empty((B, dim), dtype=torch.float32, device=device)))
    coef = (1e-3, 0.9, 0.1, 0.999, 1e-3, 1e-7)
    for tab in runs[0]:
        h.adam_sparse(*tab, *coef)
    h.adam_sparse_tables(runs[1], *coef)
    for a_, b_ in zip(runs[0], runs[1]):
        for j in (0, 1, 2, 5):  # var, m, v, mark
            assert torch.equal(a_[j], b_[j])


def test_sparse_adam_phased_matches_grouped(device):
    """hrec_adam_sparse_tables_phase 0..3 (the untouched-rows sweep on a side
    stream, overlapping the touched-rows phase) == hrec_adam_sparse_tables,
    bit for bit, incl. duplicate indices, an empty batch and a row-less table."""
    from src import _hrec as h

    rng = np.random.default_rng(22)
    shapes = [(1000, 64, 256), (300, 64, 256), (40, 8, 256), (7, 8, 0), (0, 8, 0)]
    T = lambda a: torch.as_tensor(a, device=device)  # noqa: E731
    runs = [[], []]
    for n_rows, dim, B in shapes:
        var = rng.normal(size=(n_rows, dim)).astype(np.float32)
        m = rng.normal(size=(n_rows, dim)).astype(np.float32)
        v = rng.uniform(0, 1, size=(n_rows, dim)).astype(np.float32)
        idx = rng.integers(0, max(n_rows, 1), B).astype(np.int32)
        g = rng.normal(size=(B, dim)).astype(np.float32)
        for run in runs:
            run.append((T(var), T(m), T(v), T(idx), T(g), T(np.full(n_rows, -1, np.int32)),
                        torch.empty((B, dim), dtype=torch.float32, device=device)))
    coef = (1e-3, 0.9, 0.1, 0.999, 1e-3, 1e-7)
    h.adam_sparse_tables(runs[0], *coef)
    arg = h.sparse_tables_arg([t[:4] + (None, t[5]) for t in runs[1]])
    h.adam_sparse_tables_phase(arg, h.SPARSE_MARK)
    side = torch.cuda.Stream(device=device)
    ev = torch.cuda.Event()
    ev.record()
    with torch.cuda.stream(side):
        side.wait_event(ev)
        h.adam_sparse_tables_phase(arg, h.SPARSE_SWEEP_UNTOUCHED, *coef)
        done = torch.cuda.Event()
        done.record(side)
    arg2 = h.sparse_tables_arg([t[:6] for t in runs[1]])
    h.adam_sparse_tables_phase(arg2, h.SPARSE_TOUCHED, *coef)
    torch.cuda.current_stream().wait_event(done)
    h.adam_sparse_tables_phase(arg, h.SPARSE_UNMARK)
    torch.cuda.synchronize()
    for a_, b_ in zip(runs[0], runs[1]):
        for j in (0, 1, 2, 5):  # var, m, v, mark
            assert torch.equal(a_[j], b_[j])


def test_sparse_adam_phase_argument_checks(device):
    from src import _hrec as h

    T = lambda a: torch.as_tensor(a, device=device)  # noqa: E731
    tab = (T(np.zeros((10, 6), np.float32)), T(np.zeros((10, 6), np.float32)), T(np.zeros((10, 6), np.float32)),
           T(np.zeros(4, np.int32)), None, T(np.full(10, -1, np.int32)))
    with pytest.raises(h.HrecError, match="dim % 4"):
        h.adam_sparse_tables_phase(h.sparse_tables_arg([tab]), h.SPARSE_MARK)
    with pytest.raises(h.HrecError, match="phase"):
        h.adam_sparse_tables_phase(h.sparse_tables_arg([]), 7)


def test_tt_engine_two_stream_step_matches_one_stream(device, monkeypatch):
    """TTEngine.train_step with the phased two-stream sparse Adam == the
    grouped one-stream call: every parameter and slot bit-identical after
    several steps with repeated ids in the batches."""
    from src import tt_engine

    rng = np.random.default_rng(23)
    engines = []
    for phased in ("1", "0"):
        monkeypatch.setenv("HREC_TT_PHASED", phased)
        e = tt_engine.DeviceTwoTower(500, 300, 20, 12, 64, 1e-3, seed=5, device=device)
        assert e._phased == (phased == "1")
        engines.append(e)
    B = 128
    for step in range(4):
        u = torch.as_tensor(rng.integers(0, 60, B).astype(np.int32), device=device)
        i = torch.as_tensor(rng.integers(0, 300, B).astype(np.int32), device=device)
        mn = torch.as_tensor(rng.integers(0, 20, B).astype(np.int32), device=device)
        ct = torch.as_tensor(rng.integers(0, 12, B).astype(np.int32), device=device)
        x = torch.as_tensor(rng.uniform(0, 1, (B, 2)).astype(np.float32), device=device)
        y = torch.as_tensor(rng.integers(0, 19, B).astype(np.float32), device=device)
        for e in engines:
            e.train_step(u, i, mn, ct, x, y)
    torch.cuda.synchronize()
    a, b = engines
    assert torch.equal(a.dense, b.dense) and torch.equal(a.m_dense, b.m_dense)
    for n in tt_engine.TABLES:
        assert torch.equal(a.tensors[n], b.tensors[n]), n
        assert torch.equal(a.m_tab[n], b.m_tab[n]) and torch.equal(a.v_tab[n], b.v_tab[n]), n
        assert (a.mark[n] == -1).all()


def _tt_frame(rng, n, nu, ni, nm, nc):
    return pd.DataFrame({
        "userId": rng.integers(0, nu, n), "itemId": rng.integers(0, ni, n),
        "manufacturer_id": rng.integers(0, nm, n), "category_id": rng.integers(0, nc, n),
        "price": np.round(rng.uniform(1, 300, n), 2), "average_review_rating": rng.integers(0, 19, n),
    })


def test_twotower_api_train_predict_save_load(device, tmp_path):
    from src.two_tower_model import TwoTowerModel

    rng = np.random.default_rng(4)
    train = _tt_frame(rng, 600, 50, 40, 6, 4)
    val = _tt_frame(rng, 120, 50, 40, 6, 4)
    tt = TwoTowerModel(50, 40, 6, 4, embedding_size=24)
    hist = tt.train(train, val, batch_size=64, epochs=4)
    assert tt.is_trained and len(hist.history["loss"]) >= 1 and "val_loss" in hist.history
    assert hist.history["loss"][-1] < hist.history["loss"][0]
    cand = train[["itemId", "manufacturer_id", "category_id", "price", "average_review_rating"]].head(17)
    preds = tt.predict_for_user(5, cand)
    assert [i for i, _ in preds] == list(cand["itemId"])
    assert all(isinstance(s, np.float32) for _, s in preds)
    p = {k: v for k, v in tt.model.state_dict().items() if not k.startswith("__")}
    num = tt.scaler.transform(cand[["price", "average_review_rating"]]).astype(np.float32)
    c = ott.forward(p, np.full(len(cand), 5), cand["itemId"].to_numpy(), cand["manufacturer_id"].to_numpy(),
                    cand["category_id"].to_numpy(), num)
    np.testing.assert_allclose([s for _, s in preds], c["yhat"], rtol=1e-5, atol=1e-4)
    # _build_item_tower (:38-66): (the four inputs, the tower as a function of them)
    names, item_vec = tt._build_item_tower()
    assert names == ["item_id_in", "manufacturer_in", "category_in", "numeric_in"]
    iv = item_vec(cand["itemId"].to_numpy(), cand["manufacturer_id"].to_numpy(), cand["category_id"].to_numpy(), num)
    np.testing.assert_allclose(iv.cpu().numpy(), c["ivec"], rtol=1e-5, atol=2e-5)
    path = str(tmp_path / "models" / "twotower.keras")
    tt.save_model(path)
    tt2 = TwoTowerModel.load_model(path)
    assert tt2.predict_for_user(5, cand) == preds


def test_twotower_golden_input_assembly(device):
    """predict_for_user feeds the tower exactly the inputs the reference
    builds (pinned by tests/golden/tt_inputs.json)."""
    from src.two_tower_model import TwoTowerModel

    for case in load_golden("tt_inputs.json")["cases"]:
        train = pd.DataFrame(case["train"])
        cand = pd.DataFrame(case["candidates"])
        tt = TwoTowerModel(50, 80, 9, 4, embedding_size=16)
        tt.build_model()
        feats = tt._prepare_features(train)
        assert feats["numeric_in"].tolist() == case["prepare_numeric_in"]
        seen = {}
        orig = tt._device_inputs

        def spy(f):
            seen.update(f)
            return orig(f)

        tt._device_inputs = spy
        out = tt.predict_for_user(31, cand)
        for k, v in case["inputs"].items():
            if k == "user_in":
                # the reference's column repeats one id n times; the device path
                # converts and sends that id once (one user vector serves every row)
                assert len(set(v)) == 1 and np.asarray(seen[k]).tolist() == v[:1], k
            else:
                assert np.asarray(seen[k]).tolist() == v, k
        assert [i for i, _ in out] == [i for i, _ in dec_pairs(case["result"])]


# ------------------------------------------------------------------ hybrid
class _Fixed:
    def __init__(self, preds):
        self.preds = preds

    def predict_for_user(self, user_id, all_items):
        return list(self.preds)


@pytest.mark.parametrize("case", load_golden("fusion.json")["cases"], ids=lambda c: c["name"])
def test_hybrid_api_golden(device, case):
    from src.hybrid_system import HybridRecommendationSystem

    als = dec_pairs(case["als"])
    tt = dec_pairs(case["tt"])
    h = HybridRecommendationSystem()
    h.als_f1_score, h.twotower_f1_score = case["als_f1"], case["tt_f1"]
    combined = h.adaptive_fusion(als, tt)
    exp_c = dec_pairs(case["combined"])
    legacy = ofus.adaptive_fusion(als, tt, case["als_f1"], case["tt_f1"], legacy=True)
    assert [i for i, _ in combined] == [i for i, _ in exp_c]
    # pinned-numpy semantics bit-exact; the golden (numpy 2 promotion when the
    # TT scores are float32) within 1e-6 relative
    assert [float(s) for _, s in combined] == [float(s) for _, s in legacy]
    np.testing.assert_allclose([float(s) for _, s in combined], [float(s) for _, s in exp_c], rtol=1e-6,
                               atol=1e-7)
    h.models_loaded = True
    h.als_model, h.twotower_model = _Fixed(als), _Fixed(tt)
    top = h.get_hybrid_recommendations(0, [], top_k=case["top_k"])
    assert top == [(i, s) for i, s in ofus.top_k(legacy, case["top_k"])]
    exp_top = dec_pairs(case["top"])
    # the served ranking equals the one the reference produced here, for every
    # case including the float32 two-tower ones: numpy 1.21's f64 promotion
    # (emulated) and numpy 2's f32 product (the goldens) give the same top-k
    # indices on all of them (checked case by case)
    assert [i for i, _ in top] == [i for i, _ in exp_top]
    np.testing.assert_allclose([float(s) for _, s in top], [float(s) for _, s in exp_top], rtol=1e-6, atol=1e-7)
    # both scalers are left fitted as the reference's fit_transform leaves them
    items = list(set(dict(als)).union(set(dict(tt))))
    for scaler, preds in ((h.als_scaler, dict(als)), (h.twotower_scaler, dict(tt))):
        col = np.array([preds.get(i, 0) for i in items])
        col = col if col.dtype == np.float32 else col.astype(np.float64)
        ref = MinMaxScaler().fit(col.reshape(-1, 1))
        for attr in ("data_min_", "data_max_", "data_range_", "scale_", "min_"):
            got, want = getattr(scaler, attr), getattr(ref, attr)
            assert got.dtype == want.dtype and np.array_equal(got, want), attr
        assert scaler.n_samples_seen_ == ref.n_samples_seen_
        assert np.array_equal(scaler.transform(col.reshape(-1, 1)), ref.transform(col.reshape(-1, 1)))


@pytest.mark.parametrize("k", [1024, 1025, 1500, 3000, 5000])
def test_topk_beyond_selection_bound(device, k):
    """top_k above the selection kernels' 1024 runs the device sort path
    (csrc/sort_topk.hip): still Python's stable sorted(reverse=True)[:k],
    incl. ties, -0.0 == 0.0 and NaN last (k > 2048 hung)."""
    from src import _hrec
    from src.evaluation import ranked_items

    rng = np.random.default_rng(k)
    n = 6000
    v = np.round(rng.normal(size=(3, n)), 1)
    v[0, :50] = 0.0
    v[0, 50:100] = -0.0
    v[1, ::97] = np.nan
    for dt in (np.float64, np.float32):
        x = torch.as_tensor(v.astype(dt), device=device)
        idx, val = _hrec.topk(x, k)
        for r in range(3):
            key = [(-np.inf if np.isnan(a) else a) for a in v[r].astype(dt)]
            order = sorted(range(n), key=lambda j: key[j], reverse=True)[:k]
            assert idx[r].cpu().tolist() == order
            np.testing.assert_array_equal(val[r].cpu().numpy(), v[r].astype(dt)[order])
    scores = {int(i): float(s) for i, s in enumerate(v[2])}
    exp = [i for i, _ in sorted(scores.items(), key=lambda x: x[1], reverse=True)[:k]]
    assert ranked_items(scores, k) == exp
    from src.hybrid_system import fuse_device

    a, t = v[2], v[0].astype(np.float32)
    fused, ti, ts = fuse_device(a, t, True, k)
    order = sorted(range(n), key=lambda j: fused[j], reverse=True)[:k]
    assert ti.tolist() == order


def test_hybrid_not_loaded_raises(device):
    from src.hybrid_system import HybridRecommendationSystem

    with pytest.raises(ValueError, match="Models not loaded"):
        HybridRecommendationSystem().get_hybrid_recommendations(1, [1, 2])


def test_hybrid_end_to_end(device, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)  # save_predictions writes results/predictions/ under the cwd
    from src.als_model import ALSModel
    from src.hybrid_system import HybridRecommendationSystem
    from src.two_tower_model import TwoTowerModel

    rng = np.random.default_rng(12)
    df = _tt_frame(rng, 800, 60, 35, 5, 4)
    als = ALSModel(rank=8, max_iter=4, seed=1)
    assert als.train(df)
    tt = TwoTowerModel(60, 35, 5, 4, embedding_size=16)
    tt.train(df, batch_size=128, epochs=2)
    als.save_model(str(tmp_path / "als"))
    tt.save_model(str(tmp_path / "tt.keras"))
    h = HybridRecommendationSystem()
    assert h.load_models(str(tmp_path / "als"), str(tmp_path / "tt.keras"))
    items = df[["itemId", "manufacturer_id", "category_id", "price", "average_review_rating"]].drop_duplicates(
        "itemId")
    uid = int(df["userId"].iloc[0])
    actual = {int(i): 1.0 for i in df[df["userId"] == uid]["itemId"]}
    # the reference hands the same all_items object to both models (D9)
    top = h.get_hybrid_recommendations(uid, items, actual_ratings=actual, top_k=5, save_predictions=True)
    assert len(top) == 5
    saved = h.load_predictions(uid)
    assert len(saved) == len(items)
    # iterating a DataFrame yields column names: the ALS side fails -> [] (as Spark's
    # IntegerType schema does) and the fusion sees ALS = 0 everywhere
    assert h.als_model.predict_for_user(uid, items) == []
    # same ranking as the oracle fusion over the two models' own outputs
    a = h.als_model.predict_for_user(uid, items)
    t = h.twotower_model.predict_for_user(uid, items)
    exp = ofus.top_k(ofus.adaptive_fusion(a, t, h.als_f1_score, h.twotower_f1_score, legacy=True), 5)
    assert top == exp
    # with an id list for ALS and the frame for the two-tower side
    item_ids = [int(i) for i in items["itemId"]]
    a = h.als_model.predict_for_user(uid, item_ids)
    assert len(a) == len(item_ids)
    fused = h.adaptive_fusion(a, t)
    assert [float(s) for _, s in fused] == [float(s) for _, s in
                                            ofus.adaptive_fusion(a, t, h.als_f1_score, h.twotower_f1_score)]


class _IdsFrame:
    """Candidates that iterate as item ids (the ALS side scores them) and
    index as a frame (the two-tower side), so one all_items object feeds
    both models with scores."""

    def __init__(self, df):
        self.df = df

    def __iter__(self):
        return iter(self.df["itemId"].tolist())

    def __len__(self):
        return len(self.df)

    def __getitem__(self, key):
        return self.df[key]


class _IdArray(np.ndarray):
    """An integer item id array (the ALS side iterates it) whose column
    lookups come from the item frame (the two-tower side): bench.py's
    api_call candidates."""

    def __getitem__(self, key):
        if isinstance(key, (str, list)):
            return self._df[key]
        return super().__getitem__(key)


def _id_array(df):
    a = df["itemId"].to_numpy().view(_IdArray)
    a._df = df
    return a


def test_hybrid_device_path_matches_list_path(device, monkeypatch, capsys):
    """get_hybrid_recommendations' array path (_top_on_device: fusion on the
    device scores, no Python lists) returns exactly what the list path
    (predict_for_user lists + _union + fuse_device) returns, and leaves the
    scalers fitted the same: frame wiring (ALS -> []), ids on both sides,
    cold-start rows (NaN -> fallback), duplicate ids, ties, top_k >= n and
    top_k = 0, both F1 orders. The array path builds the two-tower item
    inputs on the device (hrec_tt_item_inputs); the list runs build them on
    the host (_predict_device), so the cases with ids outside the table,
    infinite / NaN prices, an int rating column and a float32 price column
    pin the device inputs and their fallbacks to the host path's outcome."""
    from src.als_model import ALSModel
    from src.hybrid_system import HybridRecommendationSystem
    from src.two_tower_model import TwoTowerModel

    rng = np.random.default_rng(21)
    df = _tt_frame(rng, 900, 60, 40, 5, 4)
    als = ALSModel(rank=8, max_iter=3, seed=2)
    assert als.train(df)
    tt = TwoTowerModel(60, 40, 5, 4, embedding_size=16)
    tt.train(df, batch_size=128, epochs=1)
    items = df[["itemId", "manufacturer_id", "category_id", "price", "average_review_rating"]].drop_duplicates(
        "itemId").reset_index(drop=True)
    dup = pd.concat([items, items.head(7)], ignore_index=True)
    # tied two-tower scores: identical feature rows under a zero item table
    tie = items.copy()
    tie[["manufacturer_id", "category_id", "price", "average_review_rating"]] = tie.iloc[0][
        ["manufacturer_id", "category_id", "price", "average_review_rating"]].values
    # cold-start rows: ids inside the two-tower table that ALS never saw
    als_half = ALSModel(rank=8, max_iter=2, seed=3)
    assert als_half.train(df.head(60))
    assert len(set(items["itemId"]) - set(df["itemId"].head(60))) > 0
    bad_id, inf, nan, int_r, f32_p = (items.copy() for _ in range(5))
    bad_id.loc[3, "itemId"] = 10 ** 6        # outside the item table: IndexError -> []
    inf.loc[2, "price"] = np.inf              # sklearn's finiteness error -> []
    nan.loc[4, "price"] = np.nan              # NaN scores -> the list path
    int_r["average_review_rating"] = int_r["average_review_rating"].round().astype(np.int64)
    f32_p["price"] = f32_p["price"].astype(np.float32)  # outside the device input path
    cases = [("frame", items), ("ids", _IdsFrame(items)), ("dup", _IdsFrame(dup)), ("frame_dup", dup),
             ("id_array", _id_array(items)), ("id_array_dup", _id_array(dup)),
             ("bad_id", bad_id), ("inf", inf), ("nan", nan), ("int_rating", int_r), ("f32_price", f32_p)]
    calls = {"fast": 0, "tt_fast": set()}
    orig = HybridRecommendationSystem._top_on_device
    orig_tt = TwoTowerModel._predict_device_fast

    def counting_tt(self, uid, cand):
        r = orig_tt(self, uid, cand)
        if r is not None:
            calls["tt_fast"].add(type(cand).__name__)
        return r

    def counting(self, *a, **kw):
        r = orig(self, *a, **kw)
        calls["fast"] += r is not None
        return r

    def run(cand, uid, k, f1, list_path):
        h = HybridRecommendationSystem()
        h.als_model, h.twotower_model, h.models_loaded = als, tt, True
        h.als_f1_score, h.twotower_f1_score = f1
        with monkeypatch.context() as m:
            m.setattr(HybridRecommendationSystem, "_top_on_device",
                      (lambda self, *a, **kw: None) if list_path else counting)
            if list_path:  # the host-built two-tower inputs (_predict_device) as well
                m.setattr(TwoTowerModel, "_predict_device_fast", lambda self, *a: None)
            else:
                m.setattr(TwoTowerModel, "_predict_device_fast", counting_tt)
            top = h.get_hybrid_recommendations(uid, cand, top_k=k)
        return top, h

    saved = tt.model.tensors["item_emb"].clone()
    try:
        for name, cand in cases + [("cold", _IdsFrame(items)), ("tie", tie)]:
            if name == "cold":
                als_model = als
                als = als_half  # items holds ids this model never saw -> NaN -> fallback rows
            if name == "tie":
                als = als_model
                tt.model.tensors["item_emb"].zero_()
            for uid in (3, 17):
                for k in (0, 5, 50, 1000):
                    for f1 in ((0.5, 0.1), (0.1, 0.5)):
                        a, ha = run(cand, uid, k, f1, False)
                        b, hb = run(cand, uid, k, f1, True)
                        assert a == b, (name, uid, k, f1)
                        assert [type(i) for i, _ in a] == [type(i) for i, _ in b]
                        assert all(type(s) is np.float64 for _, s in a)
                        for x, y in ((ha.als_scaler, hb.als_scaler), (ha.twotower_scaler, hb.twotower_scaler)):
                            assert hasattr(x, "scale_") == hasattr(y, "scale_")
                            if name in ("bad_id", "inf"):  # both paths raised before fitting: []
                                assert a == [] and not hasattr(x, "scale_")
                                continue
                            assert hasattr(x, "scale_")
                            for attr in ("data_min_", "data_max_", "data_range_", "scale_", "min_"):
                                assert getattr(x, attr).dtype == getattr(y, attr).dtype
                                assert np.array_equal(getattr(x, attr), getattr(y, attr)), (name, attr)
                            assert x.n_samples_seen_ == y.n_samples_seen_
    finally:
        tt.model.tensors["item_emb"].copy_(saved)
    # the array path served the unique-id cases; the tie case fell back
    assert calls["fast"] > 0
    # the device-built item inputs served frames, ids frames and id arrays
    assert calls["tt_fast"] == {"DataFrame", "_IdsFrame", "_IdArray"}
    capsys.readouterr()


def test_batched_hybrid_matches_per_user_fusion(device):
    """ShardedRecommender (1 GPU) == the reference's per-user fusion + top-k
    over the same ALS (JVM-exact) and two-tower scores, bit for bit."""
    from src import _hrec
    from src.recommend import ShardedRecommender

    rng = np.random.default_rng(21)
    n_users, n_items, k, d, B = 300, 5000, 32, 24, 40
    U = np.zeros((n_users, 32), np.float32)
    U[:, :k] = rng.normal(size=(n_users, k))
    V = np.zeros((n_items, 32), np.float32)
    V[:, :k] = rng.normal(size=(n_items, k))
    uvec = torch.as_tensor(rng.normal(size=(B, d)).astype(np.float32), device=device)
    ivec = torch.as_tensor(rng.normal(size=(n_items, d)).astype(np.float32), device=device)
    dU = torch.as_tensor(U, device=device)
    Vt = _hrec.transpose(torch.as_tensor(V, device=device))
    rows = torch.as_tensor(rng.choice(n_users, B, replace=False), device=device)
    rec = ShardedRecommender(dU, Vt, ivec, 0, k)
    for als_wins in (True, False):
        idx, val = rec.recommend(rows, uvec, als_wins, 5)
        tt = _hrec.tt_score(uvec, ivec).cpu().numpy()
        als = oals.score_matrix(U[rows.cpu().numpy(), :k], V[:, :k])
        for b in range(B):
            a_pairs = [(j, float(als[b, j])) for j in range(n_items)]
            t_pairs = [(j, tt[b, j]) for j in range(n_items)]
            f1 = (0.5, 0.1) if als_wins else (0.1, 0.5)
            exp = ofus.top_k(ofus.adaptive_fusion(a_pairs, t_pairs, *f1, legacy=True), 5)
            assert idx[b].cpu().tolist() == [i for i, _ in exp]
            assert val[b].cpu().tolist() == [float(s) for _, s in exp]
    # the MFMA Dot agrees with a float64 reference
    ref = uvec.double().cpu().numpy() @ ivec.double().cpu().numpy().T
    np.testing.assert_allclose(_hrec.tt_score(uvec, ivec).cpu().numpy(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("d", [32, 50, 64])
def test_single_user_hybrid_equals_batched_recommender(device, monkeypatch, d):
    """get_hybrid_recommendations for ONE user (the array path:
    ALS transform, hrec_tt_score at B = 1, hrec_fuse_topk) and
    ShardedRecommender.recommend over a batch of 9 users holding that user
    (B >= 8: the exact hybrid K9x at d = 32 / 64, the materialised tiles
    otherwise; and the materialised path at every d) serve the same item ids
    and the same fused f64 scores, bit for bit — the two-tower score bits do
    not depend on the batch size."""
    from src import _hrec
    from src.als_model import ALSModel
    from src.hybrid_system import HybridRecommendationSystem
    from src.recommend import ShardedRecommender
    from src.two_tower_model import TwoTowerModel

    rng = np.random.default_rng(31 + d)
    df = _tt_frame(rng, 4000, 90, 700, 5, 4)
    als = ALSModel(rank=16, max_iter=3, seed=4)
    assert als.train(df)
    tt = TwoTowerModel(90, 700, 5, 4, embedding_size=d)
    tt.train(df, batch_size=256, epochs=1)
    m = als.model
    items = df[["itemId", "manufacturer_id", "category_id", "price", "average_review_rating"]].drop_duplicates(
        "itemId").reset_index(drop=True)
    items = items[np.isin(items["itemId"].to_numpy(), m.item_ids)].reset_index(drop=True)  # no cold rows
    cand = _id_array(items)
    h = HybridRecommendationSystem()
    h.als_model, h.twotower_model, h.models_loaded = als, tt, True
    seen = {}
    orig = _hrec.tt_score

    def capture(uvec, ivec):
        seen["u"], seen["i"] = uvec.clone(), ivec.clone()
        return orig(uvec, ivec)

    monkeypatch.setattr(_hrec, "tt_score", capture)
    users = [int(u) for u in np.random.default_rng(5).choice(m.user_ids, 9, replace=False)]
    for f1 in ((0.5, 0.1), (0.1, 0.5)):
        h.als_f1_score, h.twotower_f1_score = f1
        single, uvecs = [], []
        for uid in users:
            top = h.get_hybrid_recommendations(uid, cand, top_k=5)
            assert len(top) == 5
            single.append(top)
            uvecs.append(seen["u"])
        ivec = seen["i"]
        rows = torch.as_tensor(np.searchsorted(m.user_ids, users), device=device)
        irows = torch.as_tensor(np.searchsorted(m.item_ids, items["itemId"].to_numpy()), device=device)
        Vt = _hrec.transpose(m.V.index_select(0, irows).contiguous())
        U = torch.cat(uvecs).contiguous()
        for pruned in (True, False):
            rec = ShardedRecommender(m.U, Vt, ivec, 0, m.k, pruned=pruned)
            idx, val = rec.recommend(rows, U, f1[0] > f1[1], 5)
            ids = items["itemId"].to_numpy()[idx.cpu().numpy()]
            for b, top in enumerate(single):
                assert [int(i) for i, _ in top] == ids[b].tolist(), (pruned, b)
                assert np.array_equal(np.array([s for _, s in top], np.float64), val[b].cpu().numpy()), (pruned, b)


def test_twotower_resume_after_load_matches_continued_training(device, tmp_path):
    """save_model keeps the Adam slots (Keras include_optimizer=True), so
    training resumed from a loaded model equals uninterrupted training."""
    from src.two_tower_model import TwoTowerModel

    rng = np.random.default_rng(8)
    train = _tt_frame(rng, 500, 40, 30, 5, 4)
    tt = TwoTowerModel(40, 30, 5, 4, embedding_size=16)
    tt.train(train, batch_size=64, epochs=2, shuffle_seed=3)
    tt.save_model(str(tmp_path / "tt.keras"))
    back = TwoTowerModel.load_model(str(tmp_path / "tt.keras"))
    tt.train(train, batch_size=64, epochs=1, shuffle_seed=5)
    back.train(train, batch_size=64, epochs=1, shuffle_seed=5)
    a, b = tt.model.state_dict(), back.model.state_dict()
    assert a.keys() == b.keys()
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_als_hyperparameter_tuning(device):
    """src/als_model.py:142-169: a failing grid point (train -> False) is
    skipped; the best avg F1@10 over 50 sampled validation users wins."""
    from src import als_model

    rng = np.random.default_rng(30)
    train = _ratings_frame(rng, 50, 40, 900)
    val = _ratings_frame(rng, 50, 40, 200)
    grid = [{"rank": 4, "max_iter": 2}, {"rank": 0, "max_iter": 2}, {"rank": 8, "max_iter": 3, "reg_param": 0.05}]
    np.random.seed(11)
    best = als_model.hyperparameter_tuning(train, val, grid)
    # the same loop by hand, same global RNG stream for DataFrame.sample
    np.random.seed(11)
    best_f1, want = 0.0, None
    for params in grid:
        m = als_model.ALSModel(**params)
        if not m.train(train):
            continue
        f1s = []
        for uid in val["userId"].sample(50).unique():
            sel = val[val["userId"] == uid]
            preds = dict(m.predict_for_user(uid, val["itemId"].unique()))
            f1s.append(ofus.compute_f1_score(dict(zip(sel["itemId"], sel["average_review_rating"])), preds))
        if np.mean(f1s) > best_f1:
            best_f1, want = np.mean(f1s), params.copy()
    assert best == want and best is not None and best["rank"] != 0


def test_twotower_hyperparameter_tuning(device):
    """src/two_tower_model.py:169-236 with D4 (seeded Generator) and D4b
    (tables sized max(id) + 1): the grid point with the best avg
    F1@10 over the first 50 validation users wins; a failing grid point
    (here: batch_size 0) is printed and skipped."""
    from src import two_tower_model as ttm

    rng = np.random.default_rng(31)
    base = _tt_frame(rng, 600, 40, 30, 5, 4)
    grid = [{"batch_size": 64, "epochs": 1}, {"batch_size": 0, "epochs": 1}, {"batch_size": 128, "epochs": 2}]
    best = ttm.hyperparameter_tuning(base, grid, val_size=0.25, random_state=1)
    # the loop by hand: same split, same models (deterministic init / shuffle)
    users = base["userId"].unique()
    val_users = np.random.default_rng(1).choice(users, size=int(len(users) * 0.25), replace=False)
    tr, va = base[~base["userId"].isin(val_users)], base[base["userId"].isin(val_users)]
    items = va[["itemId", "manufacturer_id", "category_id", "price", "average_review_rating"]].drop_duplicates()
    best_f1, want = 0.0, None
    for params in grid:
        if params["batch_size"] == 0:
            continue
        m = ttm.TwoTowerModel(40, 30, 5, 4, embedding_size=50, learning_rate=0.001)
        m.train(tr, va, batch_size=params["batch_size"], epochs=params["epochs"])
        f1s = []
        for uid in va["userId"].unique()[:50]:
            sel = va[va["userId"] == uid]
            f1s.append(ofus.compute_f1_score(dict(zip(sel["itemId"], sel["average_review_rating"])),
                                             dict(m.predict_for_user(uid, items)), k=10))
        if np.mean(f1s) > best_f1:
            best_f1, want = np.mean(f1s), params.copy()
    assert best == want


def _fuse_rows_reference(als, tt, als_wins, kk):
    """numpy restatement of hrec_fuse_rows_topk's row fusion (MinMaxScaler per
    model and row: ALS in f64, two-tower in f32; f64 weighted sum with numpy
    1.21 promotion) + Python's stable sorted(reverse=True)[:kk]."""
    w0, w1 = (0.8, 0.2) if als_wins else (0.2, 0.8)
    idx, val = [], []
    for a, t in zip(als, tt):
        amin, amax = float(np.nanmin(a)), float(np.nanmax(a))
        ar = amax - amin
        ar = 1.0 if ar < 10 * np.finfo(np.float64).eps else ar
        asc = 1.0 / ar
        amn = 0.0 - amin * asc
        tmin, tmax = np.float32(np.nanmin(t)), np.float32(np.nanmax(t))
        tr = np.float32(tmax - tmin)
        tr = np.float32(1.0) if tr < 10 * np.finfo(np.float32).eps else tr
        tsc = np.float32(np.float32(1.0) / tr)
        tmn = np.float32(np.float32(0.0) - tmin * tsc)
        an = a.astype(np.float64) * asc + amn
        tn = (t * tsc + tmn).astype(np.float32)
        f = w0 * an + w1 * tn.astype(np.float64)
        order = sorted(range(len(f)), key=lambda j: f[j], reverse=True)[:kk]
        idx.append(order)
        val.append(f[order])
    return np.array(idx), np.array(val)


@pytest.mark.parametrize("n,kk,pattern", [(100_000, 5, "random"), (100_000, 1, "random"), (37_000, 8, "quantised"),
                                          (5000, 5, "constant"), (3000, 3, "two_levels"), (70, 5, "random"),
                                          (6_000_000, 5, "random"), (20_000, 10, "random")])
def test_fuse_rows_topk_filter_matches_reference(device, n, kk, pattern):
    """hrec_fuse_rows_topk's threshold-filter path (sample bound -> candidate
    lists -> keyed top-k; overflowing rows take the exact segment path on the
    device) returns the reference's fused top-k: indices bit-exact, values
    bit-exact (same f64 arithmetic). Covers ties (quantised scores, two
    levels), constant rows (every item a candidate -> overflow), short rows,
    a 6M-item shard and kk above the filter path's 8."""
    from src import _hrec

    rng = np.random.default_rng(n + kk)
    B = 3 if n > 1_000_000 else 7
    a = rng.normal(size=(B, n)).astype(np.float32)
    t = rng.normal(size=(B, n)).astype(np.float32)
    if pattern == "quantised":
        a, t = np.round(a, 1), np.round(t, 1)
    elif pattern == "constant":
        a[:] = 2.0
        t[1:] = 0.5
    elif pattern == "two_levels":
        a = (rng.random((B, n)) < 0.5).astype(np.float32)
        t = (rng.random((B, n)) < 0.5).astype(np.float32)
    A, T = torch.as_tensor(a, device=device), torch.as_tensor(t, device=device)
    amm, tmm = _hrec.rows_minmax(A), _hrec.rows_minmax(T)
    rows = range(B) if n <= 1_000_000 else range(1)
    for wins in (True, False):
        gi, gv = _hrec.fuse_rows_topk(A, T, amm, tmm, wins, kk, idx_offset=11)
        ei, ev = _fuse_rows_reference(a[list(rows)], t[list(rows)], wins, kk)
        np.testing.assert_array_equal(gi.cpu().numpy()[list(rows)], ei + 11)
        np.testing.assert_array_equal(gv.cpu().numpy()[list(rows)], ev)


def test_als_device_lookup_matches_host(device):
    """DeviceALSFactors.score's device id lookup (long candidate lists) ==
    the host binary search: same rows, -1 (-> NaN score) for unknown ids."""
    from src.als_model import DeviceALSFactors

    rng = np.random.default_rng(8)
    ids = np.unique(rng.integers(-50, 30000, 9000))
    U = torch.randn(4, 16, device=device)
    V = torch.randn(len(ids), 16, device=device)
    f = DeviceALSFactors(np.arange(4), ids, U, V, 10)
    keys = np.concatenate([rng.choice(ids, 6000), rng.integers(-100, 31000, 3000), [ids[0], ids[-1]]])
    host = DeviceALSFactors._lookup(f.item_ids, keys)
    assert (host == -1).any() and (host >= 0).any()
    assert np.array_equal(f._lookup_device(keys.astype(np.int64)).cpu().numpy(), host)
    a = f.score([1], keys.astype(np.int64)).cpu().numpy()
    b = f.score([1], keys.tolist()).cpu().numpy()
    assert np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)])


@pytest.mark.parametrize("als_wins", [True, False])
def test_top_on_device_matches_numpy_fusion(device, als_wins):
    """get_hybrid_recommendations' array path (_top_on_device) on
    f64 ALS + f32 two-tower device scores against the reference arithmetic
    written in numpy + sklearn (tests/test_oracle.py::_numpy_fusion). The
    device fusion follows numpy 1.21.5's promotion (requirements.txt:5: the
    Python-float weight times an np.float32 element widens to float64): top-k
    ids and scores bit-exact against it. Against numpy 2's float32 product
    (NEP 50, the container's numpy) the ids agree wherever the top-k is
    separated by more than the f32 product's rounding (2^-24 relative)."""
    from src.hybrid_system import HybridRecommendationSystem
    from test_oracle import _numpy_fusion

    rng = np.random.default_rng(31 + als_wins)
    n, k = 50_000, 10
    als = rng.normal(size=n) * 2
    tt = (rng.normal(size=n) * 3).astype(np.float32)
    frame = pd.DataFrame({"itemId": np.arange(n)})
    h = HybridRecommendationSystem()
    h.als_f1_score, h.twotower_f1_score = (0.5, 0.1) if als_wins else (0.1, 0.5)
    keys = np.arange(n, dtype=np.int64)
    top = h._top_on_device((keys.tolist(), keys, torch.as_tensor(als, device=device).float().double()),
                           (frame, torch.as_tensor(tt, device=device)), k)
    als_used = als.astype(np.float32).astype(np.float64)  # the ALS side hands over f32 transform scores
    ref = _numpy_fusion(als_used, tt, als_wins, "1.21")
    order = sorted(range(n), key=lambda j: ref[j], reverse=True)[:k]
    assert top is not None
    assert [i for i, _ in top] == order
    assert [float(s) for _, s in top] == [float(ref[j]) for j in order]
    np2 = _numpy_fusion(als_used, tt, als_wins, "2")
    o2 = sorted(range(n), key=lambda j: np2[j], reverse=True)
    gaps = np.abs(np.diff(np2[o2[: k + 1]]))
    for j in range(k):
        if gaps[j] > 1e-7 and (j == 0 or gaps[j - 1] > 1e-7):
            assert top[j][0] == o2[j]
