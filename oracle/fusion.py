"""Oracle restatement of the hybrid fusion, top-k and F1 (pure Python/numpy).

Test infrastructure only (see oracle/__init__.py). Follows:
  * HybridRecommendationSystem.adaptive_fusion  src/hybrid_system.py:57-75
  * top-k = sorted(combined, key=score, reverse=True)[:top_k]  :108
  * compute_f1_score  src/als_model.py:171-177 (== two_tower_model.py:238-245
    apart from the k > 0 guard)
  * sklearn MinMaxScaler.fit_transform arithmetic (container sklearn
    preprocessing/_data.py:518-522 and :261-262): scale = 1/range with
    range < 10*eps(dtype) -> 1, min_ = 0 - data_min*scale, X*scale + min_.

numpy promotion of `weights[1] * tt_norm[i]` for an np.float32 element:
numpy 1.21.5 (pinned, requirements.txt:5) widens to float64 before the
multiply; numpy >= 2 (NEP 50) multiplies in float32. `legacy=True`
reproduces the pinned behaviour (what libhrec implements).
"""
import numpy as np


def minmax(x):
    """MinMaxScaler().fit_transform(x.reshape(-1, 1)).flatten(), restated."""
    x = np.asarray(x)
    if x.dtype.kind in "iub":
        x = x.astype(np.float64)
    dt = x.dtype.type
    dmin = np.nanmin(x)
    dmax = np.nanmax(x)
    rng = dt(dmax - dmin)
    if rng < dt(10) * np.finfo(x.dtype).eps:
        rng = dt(1.0)
    scale = dt(dt(1) / rng)
    min_ = dt(dt(0) - dmin * scale)
    return (x * scale + min_).astype(x.dtype)


def union_order(als_keys, tt_keys):
    """Iteration order of set(als).union(set(tt)) (src/hybrid_system.py:61)."""
    return list(set(als_keys).union(set(tt_keys)))


def adaptive_fusion(als_predictions, tt_predictions, als_f1, tt_f1, legacy=True):
    als_dict = dict(als_predictions)
    tt_dict = dict(tt_predictions)
    items = union_order(als_dict.keys(), tt_dict.keys())
    als_arr = np.array([als_dict.get(it, 0) for it in items])
    tt_arr = np.array([tt_dict.get(it, 0) for it in items])
    als_norm = minmax(als_arr)
    tt_norm = minmax(tt_arr)
    w = (0.8, 0.2) if als_f1 > tt_f1 else (0.2, 0.8)
    out = []
    for n, it in enumerate(items):
        a = w[0] * als_norm[n]
        t = tt_norm[n]
        if legacy:
            t = w[1] * float(t)
        else:
            t = w[1] * t
        out.append((it, a + t))
    return out


def top_k(combined, k):
    return sorted(combined, key=lambda x: x[1], reverse=True)[:k]


def compute_f1_score(actual, pred, k=10):
    actual_items = set(actual.keys())
    ranked = sorted(pred.items(), key=lambda x: x[1], reverse=True)[:k]
    pred_items = set(item for item, _ in ranked)
    tp = len(actual_items & pred_items)
    precision = tp / k if k > 0 else 0
    recall = tp / len(actual_items) if actual_items else 0
    if precision + recall > 0:
        return 2 * (precision * recall) / (precision + recall)
    return 0


def cosine(a, b):
    """sklearn cosine_similarity([a], [b])[0][0]: normalise rows, then dot."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    na = np.sqrt(np.dot(a, a))
    nb = np.sqrt(np.dot(b, b))
    na = 1.0 if na == 0 else na
    nb = 1.0 if nb == 0 else nb
    return float(np.dot(a / na, b / nb))


def find_similar_items(item_features, item_id, k=3):
    """ALSModel._find_similar_items (src/als_model.py:93-104)."""
    if item_id not in item_features:
        return []
    target = item_features[item_id]["features"]
    sims = []
    for other_id, feats in item_features.items():
        if other_id == item_id:
            continue
        sims.append((other_id, cosine(target, feats["features"])))
    ranked = sorted(sims, key=lambda x: x[1], reverse=True)[:k]
    return [it for it, s in ranked if s > 0.5]


def als_predict_with_fallback(spark_predictions, item_features, global_mean, query):
    """The per-item loop of ALSModel.predict_for_user (src/als_model.py:78-87):
    a non-NaN Spark prediction becomes float(pred); otherwise the mean rating
    of up to 3 similar items, else global_mean."""
    out = []
    for item in query:
        pred = spark_predictions.get(item)
        if pred is not None and not np.isnan(pred):
            out.append((item, float(pred)))
        else:
            sims = find_similar_items(item_features, item)
            val = np.mean([item_features[s]["rating"] for s in sims]) if sims else global_mean
            out.append((item, val))
    return out
