"""GPU: the ALS cold-start fallback precomputed once per model
(csrc/cold_start.hip, hrec_cold_fallback) —
ALSModel.predict_for_user's value for an item the transform left NaN
(/root/reference/src/als_model.py:78-86: the mean rating of the <= 3 most
similar other items with cosine > 0.5, :93-104, else the global mean).

Tolerance: BIT-EXACT. The vector must equal, item by item, what the per-item
search returns (_find_similar_items: hrec_cosine_sim + the stable top-k + the
sim > 0.5 filter, itself pinned by the reference-executed similar_items.json /
als_fallback.json fixtures in tests/test_gpu_api.py) and np.mean over those
items' ratings; predict_for_user and get_hybrid_recommendations must return
the same lists with and without the vector.
"""
import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu


def _features(rng, n, dim, quant):
    ids = rng.permutation(10 * n)[:n]  # dict order != id order
    x = rng.normal(size=(n, dim))
    if quant:  # coarse grid: exact similarity ties, zero vectors, sims of exactly 0.5 / 1
        x = np.round(x * 2) / 2
    if n > 3:
        x[1] = 0.0
        x[2] = x[3]
    r = rng.integers(0, 19, n).astype(float)
    return {int(i): {"features": x[p].copy(), "rating": float(r[p])} for p, i in enumerate(ids)}


def _model(feats, gm=3.25):
    from src.als_model import ALSModel

    m = ALSModel()
    m.initialize_spark()
    m.item_features = feats
    m.global_mean = gm
    return m


@pytest.mark.parametrize("n,dim,quant", [(1, 3, False), (2, 3, True), (3, 2, False), (300, 1, False),
                                         (2000, 3, True), (5000, 3, False), (1500, 8, True), (777, 16, False),
                                         (20_000, 3, True)])
def test_cold_fallback_equals_per_item_search(device, n, dim, quant):
    from src import _hrec

    rng = np.random.default_rng(n + dim)
    feats = _features(rng, n, dim, quant)
    m = _model(feats)
    fb = m._fallback()
    assert fb is not None
    ids, pos, mat = m._feature_matrix()
    ratings = torch.as_tensor(np.array([feats[i]["rating"] for i in ids]), device=device)
    _, _, idx = _hrec.cold_fallback(mat, ratings, want_idx=True)
    idx = idx.cpu().numpy()
    sample = ids if n <= 2000 else [ids[p] for p in np.random.default_rng(1).choice(n, 1500, replace=False)]
    sims = m._similar_batch(list(sample))
    for it, sim in zip(sample, sims):
        p = pos[it]
        assert [ids[j] for j in idx[p] if j >= 0] == sim, it
        assert int(fb["cnt_h"][p]) == len(sim)
        if sim:
            exp = np.mean([feats[s]["rating"] for s in sim])
            assert fb["mean_h"][p] == exp and type(fb["mean_h"][p]) is type(exp)


def test_cold_fallback_invalidated_with_features(device):
    """Assigning item_features drops the vector; a new one is computed."""
    rng = np.random.default_rng(4)
    m = _model(_features(rng, 500, 3, True))
    a = m._fallback()
    assert m._fallback() is a  # cached
    m.item_features = _features(rng, 400, 3, False)
    b = m._fallback()
    assert b is not a and len(b["cnt_h"]) == 400


def _cold_user_model(device, n_items, dim=3, seed=0):
    """A fitted rank-8 model over n_items, every item with features; user 7
    is known, user 10**6 is not (every row NaN: the reference protocol's
    cold test users)."""
    from src.als_model import DeviceALSFactors

    rng = np.random.default_rng(seed)
    feats = _features(rng, n_items, dim, True)
    item_ids = np.array(sorted(feats), np.int64)
    V = torch.zeros((n_items, 16), dtype=torch.float32, device=device)
    V[:, :8] = torch.as_tensor(rng.normal(size=(n_items, 8)).astype(np.float32))
    U = torch.zeros((1, 16), dtype=torch.float32, device=device)
    U[0, :8] = torch.as_tensor(rng.normal(size=8).astype(np.float32))
    m = _model(feats, gm=np.float64(7.125))
    m.model = DeviceALSFactors(np.array([7]), item_ids, U, V, 8)
    return m, item_ids


def test_predict_for_user_cold_matches_per_item_path(device, monkeypatch):
    """predict_for_user for a cold user (every row NaN) and for a known user
    over unknown items: the vector path returns the per-item path's list —
    values and types (np.float64 means, the global mean object)."""
    from src.als_model import ALSModel

    m, item_ids = _cold_user_model(device, 3000)
    query = [int(i) for i in item_ids[::3]] + [10 ** 7, 10 ** 7 + 1]  # + items without features
    for uid in (10 ** 6, 7):
        fast = m.predict_for_user(uid, query)
        with monkeypatch.context() as mp:
            mp.setattr(ALSModel, "_fallback", lambda self: None)
            slow = m.predict_for_user(uid, query)
        assert [i for i, _ in fast] == [i for i, _ in slow]
        for (_, a), (_, b) in zip(fast, slow):
            assert a == b and type(a) is type(b)


def test_predict_for_user_nonfinite_features_error(device, capsys):
    """A NaN feature vector: sklearn's cosine_similarity raises inside the
    reference's fallback loop -> 'Prediction error' and [] (an item without
    features alone still takes the global mean)."""
    rng = np.random.default_rng(3)
    feats = _features(rng, 50, 3, False)
    first = next(iter(feats))
    feats[first]["features"][1] = np.nan
    from src.als_model import DeviceALSFactors

    m = _model(feats)
    V = torch.zeros((1, 16), dtype=torch.float32, device=device)
    m.model = DeviceALSFactors(np.array([7]), np.array([10 ** 8]), V[:1].clone(), V, 1)
    assert m.predict_for_user(7, [first]) == []
    assert "Input contains NaN" in capsys.readouterr().out
    assert m.predict_for_user(7, [10 ** 9]) == [(10 ** 9, m.global_mean)]


def test_hybrid_cold_user_array_path_matches_list_path(device, monkeypatch):
    """get_hybrid_recommendations for a cold user: the array path (ALS rows
    filled from the vector on the device) returns the list path's top-k and
    leaves the scalers fitted the same."""
    from src.hybrid_system import HybridRecommendationSystem
    from src.two_tower_model import TwoTowerModel
    from sklearn.preprocessing import MinMaxScaler

    n = 4000
    m, item_ids = _cold_user_model(device, n, seed=2)
    tt = TwoTowerModel(20, n, 30, 10, embedding_size=32, seed=3)
    tt.build_model()
    rng = np.random.default_rng(5)
    items = pd.DataFrame({"itemId": np.arange(n), "manufacturer_id": rng.integers(0, 30, n),
                          "category_id": rng.integers(0, 10, n), "price": rng.random(n) * 100,
                          "average_review_rating": rng.integers(0, 19, n).astype(np.float64)})
    tt.scaler = MinMaxScaler().fit(items[["price", "average_review_rating"]])
    # ALS ids = the frame's ids (the feature dict is keyed by them too)
    from src.als_model import DeviceALSFactors

    feats = {int(i): v for i, v in zip(range(n), m.item_features.values())}
    m.item_features = feats
    m.model = DeviceALSFactors(np.array([7]), np.arange(n), m.model.U, m.model.V, 8)

    class IdArray(np.ndarray):
        def __getitem__(self, key):
            if isinstance(key, (str, list)):
                return items[key]
            return super().__getitem__(key)

    cand = items["itemId"].to_numpy().view(IdArray)
    calls = {"fast": 0}
    orig = HybridRecommendationSystem._top_on_device

    def counting(self, *a, **kw):
        r = orig(self, *a, **kw)
        calls["fast"] += r is not None
        return r

    for f1 in ((0.5, 0.1), (0.1, 0.5)):
        for uid in (3, 7, 11):  # the ALS model knows user 7 only; all three are two-tower users
            res = []
            for list_path in (False, True):
                h = HybridRecommendationSystem()
                h.als_model, h.twotower_model, h.models_loaded = m, tt, True
                h.als_f1_score, h.twotower_f1_score = f1
                with monkeypatch.context() as mp:
                    mp.setattr(HybridRecommendationSystem, "_top_on_device",
                               (lambda self, *a, **kw: None) if list_path else counting)
                    res.append((h.get_hybrid_recommendations(uid, cand, top_k=5), h))
            (a, ha), (b, hb) = res
            assert a == b and len(a) == 5, (uid, f1)
            for x, y in ((ha.als_scaler, hb.als_scaler), (ha.twotower_scaler, hb.twotower_scaler)):
                for attr in ("data_min_", "data_max_", "scale_", "min_"):
                    assert np.array_equal(getattr(x, attr), getattr(y, attr)), attr
    assert calls["fast"] >= 4  # the cold users stayed on the array path
