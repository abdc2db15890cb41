"""Offline quality metrics: the drop-in for src/evaluation.py.

`RecommenderEvaluator` keeps the reference's per-user dict API
(src/evaluation.py:19-149): Precision@k / Recall@k against the "manuscript"
relevance band (ratings within ±0.1 of the user's mean rating), NDCG@k on
3-level grades, MAE/RMSE after a 1–5 rescale, and `comprehensive_evaluation`.
The ranking step of P@k/R@k — `sorted(scores, reverse=True)[:k]`, stable, so
ties keep dict order — is the device's stable top-k (`hrec_topk_f64`); the
per-user set arithmetic that follows is O(k) host work. NDCG and MAE/RMSE
call the same sklearn functions the reference calls (its dependency,
requirements.txt), on the same inputs in the same set-iteration order.

`compute_f1_score` is also exported here: src/hybrid_system.py:15 imports it
from this module, where the reference never defines it.

Reference behaviour kept on purpose (pinned by tests/golden/evaluation.json,
produced by executing the reference):
  * `comprehensive_evaluation` raises ValueError — it hands dicts to
    sklearn's f1_score;
  * NDCG on a single common item and MAE/RMSE on constant ratings raise
    ValueError (sklearn rejects one document / NaN).
Plotting needs matplotlib/seaborn, which this build does not ship.
"""
import os

import numpy as np
import torch

from . import _hrec
from .als_model import compute_f1_score  # noqa: F401  (D2)

_BAND = 0.1  # the manuscript's relevance tolerance around the mean rating


def _relevance_band(actual_ratings, tolerance=_BAND):
    """(threshold, relevant item set): items rated within ±tolerance of the
    mean rating (src/evaluation.py:29-31, 142-146)."""
    threshold = np.mean(list(actual_ratings.values()))
    lo, hi = threshold - tolerance, threshold + tolerance
    return threshold, {item for item, r in actual_ratings.items() if lo <= r <= hi}


def ranked_items(predicted_scores, k):
    """The first k items of sorted(predicted_scores.items(), key=score,
    reverse=True): a stable descending top-k on the device."""
    items = list(predicted_scores.keys())
    k = int(k) if k >= 0 else max(len(items) + int(k), 0)  # Python slice [:k] semantics
    if k == 0 or not items:
        return []
    _hrec.require_device()
    vals = torch.tensor([float(v) for v in predicted_scores.values()], dtype=torch.float64, device="cuda")
    idx, _ = _hrec.topk(vals, min(int(k), len(items)))
    return [items[i] for i in idx[0].tolist()]


def _common(actual_ratings, predicted_scores):
    # the reference's set intersection, iterated in the same (hash) order
    common = set(actual_ratings.keys()) & set(predicted_scores.keys())
    return ([actual_ratings[i] for i in common], [predicted_scores[i] for i in common]) if common else None


class RecommenderEvaluator:
    """src/evaluation.py:19 — same methods and return values."""

    def __init__(self):
        from sklearn.preprocessing import MinMaxScaler

        self.scaler = MinMaxScaler()
        self.rating_scaler = MinMaxScaler()

    def precision_at_k(self, actual_ratings, predicted_scores, k=10):
        _, relevant = _relevance_band(actual_ratings)
        hits = sum(1 for item in ranked_items(predicted_scores, k) if item in relevant)
        return hits / k if k > 0 else 0.0

    def recall_at_k(self, actual_ratings, predicted_scores, k=10):
        _, relevant = _relevance_band(actual_ratings)
        if not relevant:
            return 0.0
        return len(set(ranked_items(predicted_scores, k)) & relevant) / len(relevant)

    def ndcg_at_k(self, actual_ratings, predicted_scores, k=10):
        from sklearn.metrics import ndcg_score

        pair = _common(actual_ratings, predicted_scores)
        if pair is None:
            return 0.0
        y_true, y_pred = (np.array(v).reshape(-1, 1) for v in pair)
        # both columns on the TRUE ratings' min-max fit, then 3 grades
        t = self.rating_scaler.fit_transform(y_true).ravel()
        p = self.rating_scaler.transform(y_pred).ravel()
        edges = [0.33, 0.66]
        return ndcg_score([np.digitize(t, edges)], [np.digitize(p, edges)], k=k)

    def mae_rmse(self, actual_ratings, predicted_scores):
        from sklearn.metrics import mean_absolute_error, mean_squared_error

        pair = _common(actual_ratings, predicted_scores)
        if pair is None:
            return 0.0, 0.0

        def to_1_5(v):
            lo, hi = min(v), max(v)
            return 1 + 4 * (np.array(v) - lo) / (hi - lo)

        with np.errstate(divide="ignore", invalid="ignore"):  # constant input -> NaN -> sklearn raises
            t, p = to_1_5(pair[0]), to_1_5(pair[1])
        return mean_absolute_error(t, p), np.sqrt(mean_squared_error(t, p))

    def _binarize(self, ratings_dict, tolerance=0.1):
        threshold = np.mean(list(ratings_dict.values()))
        return {item: int(threshold - tolerance <= r <= threshold + tolerance) for item, r in ratings_dict.items()}

    def comprehensive_evaluation(self, actual_ratings, predicted_scores, k_values=(5, 10, 15, 20)):
        from sklearn.metrics import f1_score

        results = {}
        for k in k_values:
            results[f"Precision@{k}"] = self.precision_at_k(actual_ratings, predicted_scores, k)
            results[f"Recall@{k}"] = self.recall_at_k(actual_ratings, predicted_scores, k)
        # the reference passes the binarised DICTS to sklearn, which
        # rejects them (ValueError) — kept as the reference behaves.
        results["F1_Score"] = f1_score(self._binarize(actual_ratings), self._binarize(predicted_scores))
        results["NDCG"] = self.ndcg_at_k(actual_ratings, predicted_scores)
        results["MAE"], results["RMSE"] = self.mae_rmse(actual_ratings, predicted_scores)
        return results

    def plot_precision_recall_at_k(self, results_dict, k_values, model_name, save_path=None):
        try:
            import matplotlib.pyplot as plt  # noqa: F401
        except ImportError as e:
            raise ImportError("plot_precision_recall_at_k needs matplotlib, which this build does not ship") from e
        raise NotImplementedError("plotting is outside the MI355X hot path")

    def load_predictions(self, user_id, pred_dir="results/predictions"):
        import pandas as pd

        df = pd.read_csv(os.path.join(pred_dir, f"user_{user_id}_predictions.csv"))
        return list(zip(df["itemId"], df["hybrid_score"]))
