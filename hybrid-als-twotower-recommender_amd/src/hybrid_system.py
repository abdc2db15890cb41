"""Hybrid ALS + two-tower fusion — drop-in for the reference's src/hybrid_system.py.

Same class and methods as src/hybrid_system.py:20-120. adaptive_fusion and
the top-k of get_hybrid_recommendations run on the device through
hrec_fuse_topk (K9): sklearn MinMaxScaler arithmetic per model in its numpy
dtype, the (0.8, 0.2) / (0.2, 0.8) weights chosen by the strict
als_f1 > tt_f1 test, f64 fusion with numpy 1.21's scalar promotion (the
pinned numpy, requirements.txt:5), and a stable descending top-k that keeps
Python's sorted(..., reverse=True) tie order. The item order of the fused
list is the iteration order of set(als).union(set(tt)) (:61), built on the
host exactly as the reference builds it.
"""
import itertools
import os
import warnings

import numpy as np
import pandas as pd
import torch
from sklearn.preprocessing import MinMaxScaler

from . import _hrec
from .als_model import ALSModel
from .evaluation import compute_f1_score
from .two_tower_model import TwoTowerModel

warnings.filterwarnings("ignore")

def _as_scores(values):
    """np.array(list) as the reference builds it, then the dtype
    MinMaxScaler computes in (ints/bools -> float64, float32 stays)."""
    arr = np.array(values)
    if arr.dtype == np.float32:
        out = arr
    else:
        out = arr.astype(np.float64)
    if out.size == 0:
        raise ValueError("Found array with 0 sample(s) (shape=(0, 1)) while a minimum of 1 is required by "
                         "MinMaxScaler.")
    if np.isinf(out).any():
        raise ValueError("Input X contains infinity or a value too large for dtype('float64').")
    return out


def _set_fitted(scaler, lo, hi, n, dtype):
    """Leave `scaler` in the state MinMaxScaler.fit_transform of an [n, 1]
    column of `dtype` with min lo / max hi leaves it (the reference refits both
    scalers per fusion, src/hybrid_system.py:66-67); the O(1) attribute
    arithmetic is sklearn's (_data.py partial_fit, feature_range (0, 1))."""
    dmin = np.array([lo], dtype=dtype)
    dmax = np.array([hi], dtype=dtype)
    drange = dmax - dmin
    safe = drange.copy()
    safe[safe < 10 * np.finfo(safe.dtype).eps] = 1.0
    scaler.n_features_in_ = 1
    scaler.n_samples_seen_ = int(n)
    scaler.data_min_, scaler.data_max_, scaler.data_range_ = dmin, dmax, drange
    scaler.scale_ = (1 - 0) / safe
    scaler.min_ = 0 - dmin * scaler.scale_


def fuse_device(als_scores, tt_scores, als_wins, top_k, device=None, want_fused=True, scalers=None):
    """Fusion + stable top-k on the device. Returns (fused f64 [n] or None,
    top indices, top scores) as numpy arrays. `scalers` = (als_scaler,
    tt_scaler) are left fitted as the reference's fit_transform leaves them."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    a = torch.as_tensor(als_scores, device=device)
    t = torch.as_tensor(tt_scores, device=device)
    n = a.numel()
    kk = n if top_k is None else (max(n + top_k, 0) if top_k < 0 else min(top_k, n))
    mm = torch.empty(4, dtype=torch.float64, device=device) if scalers is not None else None
    idx, sc, fused = _hrec.fuse_topk(a, t, als_wins, kk, want_fused=want_fused, minmax=mm)
    fused_np = fused.cpu().numpy() if fused is not None else None
    if scalers is not None:
        m = mm.cpu().numpy()
        _set_fitted(scalers[0], m[0], m[1], n, np.float64)
        _set_fitted(scalers[1], m[2], m[3], n, np.dtype(tt_scores.dtype))
    return fused_np, idx.cpu().numpy(), sc.cpu().numpy()


def _unique(vals, col):
    """No repeated id: a bincount when the ids are small non-negative ints
    (catalogue ids), else pandas' hash check."""
    if vals.size == 0:
        return True
    lo, hi = int(vals.min()), int(vals.max())
    if lo >= 0 and hi < 4 * vals.size + 4096:
        return int(np.bincount(vals.astype(np.int64, copy=False)).max()) <= 1
    return bool(col.is_unique)


def _scored(model, cls, user_id, all_items):
    if type(model).predict_for_user is cls.predict_for_user:
        return model._predict_device(user_id, all_items)
    return model.predict_for_user(user_id, all_items)


class HybridRecommendationSystem:
    def __init__(self):
        self.als_model = None
        self.twotower_model = None
        self.als_scaler = MinMaxScaler()
        self.twotower_scaler = MinMaxScaler()
        self.als_f1_score = 0.0
        self.twotower_f1_score = 0.0
        self.models_loaded = False
        self._flags_bad = False

    def load_models(self, als_model_path, twotower_model_path):
        try:
            print("=== Loading Pre-trained Models ===")
            self.als_model = ALSModel().load_model(als_model_path)
            self.twotower_model = TwoTowerModel.load_model(twotower_model_path)
            self.models_loaded = True
            print("\n=== Models loaded successfully ===")
            return True
        except Exception as e:
            print(f"Error loading models: {str(e)}")
            return False

    def evaluate_individual_models(self, test_user_id, actual_ratings, all_items, k=10):
        try:
            als_preds = self.als_model.predict_for_user(test_user_id, all_items)
            tt_preds = self.twotower_model.predict_for_user(test_user_id, all_items)
            self.als_f1_score = compute_f1_score(actual_ratings, dict(als_preds))
            self.twotower_f1_score = compute_f1_score(actual_ratings, dict(tt_preds))
            print(f"Model F1 Scores - ALS: {self.als_f1_score:.4f}, "
                  f"Two-Tower: {self.twotower_f1_score:.4f}")
            return self.als_f1_score, self.twotower_f1_score
        except Exception as e:
            print(f"Error evaluating models: {str(e)}")
            return 0.0, 0.0

    def _union(self, als_predictions, twotower_predictions):
        als_dict = dict(als_predictions)
        tt_dict = dict(twotower_predictions)
        items = list(set(als_dict.keys()).union(set(tt_dict.keys())))
        # [d.get(item, 0) for item in items] (:62-63), via map (same values)
        als_scores = _as_scores(list(map(als_dict.get, items, itertools.repeat(0))))
        tt_scores = _as_scores(list(map(tt_dict.get, items, itertools.repeat(0))))
        return items, als_scores, tt_scores

    def adaptive_fusion(self, als_predictions, twotower_predictions):
        try:
            items, als_scores, tt_scores = self._union(als_predictions, twotower_predictions)
            fused, _, _ = fuse_device(als_scores, tt_scores, self.als_f1_score > self.twotower_f1_score, 0,
                                      scalers=(self.als_scaler, self.twotower_scaler))
            return [(item, fused[i]) for i, item in enumerate(items)]
        except Exception as e:
            print(f"Error in adaptive fusion: {str(e)}")
            return []

    def save_predictions(self, user_id, predictions, save_dir="results/predictions"):
        os.makedirs(save_dir, exist_ok=True)
        file_path = os.path.join(save_dir, f"user_{user_id}_predictions.csv")
        df = pd.DataFrame(predictions, columns=["itemId", "hybrid_score"])
        df["userId"] = user_id
        df["prediction_rank"] = range(1, len(df) + 1)
        df["timestamp"] = pd.Timestamp.now()
        df.to_csv(file_path, index=False)
        print(f"Predictions saved to {file_path}")
        return file_path

    def load_predictions(self, user_id, save_dir="results/predictions"):
        file_path = os.path.join(save_dir, f"user_{user_id}_predictions.csv")
        if not os.path.exists(file_path):
            raise FileNotFoundError(f"No predictions found for user {user_id}")
        df = pd.read_csv(file_path)
        return list(zip(df["itemId"], df["hybrid_score"]))

    def get_hybrid_recommendations(self, user_id, all_items, actual_ratings=None, top_k=5,
                                   save_predictions=False):
        if not self.models_loaded:
            raise ValueError("Models not loaded. Call load_models() first.")
        try:
            # the drop-in models hand over device scores (the lists are built
            # below only if the list path runs); other model objects are used
            # through their predict_for_user as the reference does
            als_preds = _scored(self.als_model, ALSModel, user_id, all_items)
            tt_fast = None
            if (not save_predictions and not actual_ratings
                    and type(self.twotower_model).predict_for_user is TwoTowerModel.predict_for_user):
                # the candidate frame's item inputs built on the device (ids,
                # scaler, uniqueness checked there; read back with the top-k)
                tt_fast = self.twotower_model._predict_device_fast(user_id, all_items)
            if tt_fast is not None:
                self._flags_bad = False
                try:
                    top = self._top_on_device(als_preds, tt_fast[:2], top_k, flags=tt_fast[2])
                except Exception:
                    top, self._flags_bad = None, True
                if top is not None:
                    return top
                # ties or NaN scores: the list path on the same scores; bad
                # inputs: the host path (raises where the reference raises)
                tt_preds = tt_fast[:2] if not self._flags_bad else _scored(self.twotower_model, TwoTowerModel,
                                                                           user_id, all_items)
            else:
                tt_preds = _scored(self.twotower_model, TwoTowerModel, user_id, all_items)
            if actual_ratings:
                self.evaluate_individual_models(user_id, actual_ratings, all_items)
            if not save_predictions and tt_fast is None:
                try:
                    top = self._top_on_device(als_preds, tt_preds, top_k)
                except Exception:  # the list path below meets the same error and reports it as the reference does
                    top = None
                if top is not None:
                    return top
            if isinstance(als_preds, tuple):  # the lists predict_for_user returns (:101-102)
                als_preds = self.als_model._predictions_guarded(als_preds[0], als_preds[2])
            if isinstance(tt_preds, tuple):
                tt_preds = self.twotower_model._predictions(*tt_preds)
            try:
                items, als_scores, tt_scores = self._union(als_preds, tt_preds)
                fused, idx, sc = fuse_device(als_scores, tt_scores, self.als_f1_score > self.twotower_f1_score,
                                             top_k, want_fused=save_predictions,
                                             scalers=(self.als_scaler, self.twotower_scaler))
            except Exception as e:  # adaptive_fusion's own guard (:73-75) -> []
                print(f"Error in adaptive fusion: {str(e)}")
                items, fused, idx, sc = [], None, [], []
            top_recommendations = [(items[i], np.float64(s)) for i, s in zip(idx, sc)]
            if save_predictions:
                combined = [(item, fused[i]) for i, item in enumerate(items)] if fused is not None else []
                self.save_predictions(user_id, combined)
            return top_recommendations
        except Exception as e:
            print(f"Error generating recommendations: {str(e)}")
            return []

    def _top_on_device(self, als_side, tt_side, top_k, flags=None):
        """get_hybrid_recommendations without the Python lists: when both
        sides cover the same unique candidate ids (or the ALS side is empty,
        the reference's DataFrame wiring) the union is those ids;
        the fusion runs on the device scores (a cold ALS user's rows already
        hold the model's fallback vector, ALSModel._predict_device) and the
        top_k + 1 fused scores come back. If they are finite and strictly decreasing, the stable
        top_k is the same whatever order the reference's set(...) union put
        the items in, so it is returned; otherwise (ties, NaN/inf scores,
        duplicate or mismatched ids) None sends the call down the list path,
        which reproduces the set order exactly. The scalers are fitted as
        fit_transform leaves them either way (min/max are order-free).
        flags: the device input flags of TwoTowerModel._predict_device_fast
        (its device check replaces the host uniqueness pass); read back with
        the top-k; non-zero sets self._flags_bad and returns None."""
        if not isinstance(tt_side, tuple) or not isinstance(top_k, (int, np.integer)) or top_k < 0:
            return None
        frame, t = tt_side
        col = frame["itemId"]
        vals = col.values
        if not isinstance(vals, np.ndarray) or vals.dtype.kind not in "iu":
            return None
        if flags is None and not _unique(vals, col):
            return None
        n = t.numel()
        if isinstance(als_side, tuple):
            items, keys, a = als_side
            if keys.shape != vals.shape or not np.array_equal(keys, vals):
                return None
            a = a.double()
            def item(i): return items[i]      # the union keeps the ALS side's key objects
        elif not als_side:
            a = torch.zeros(n, dtype=torch.float64, device=t.device)  # finite: only t is checked below
            def item(i): return vals.item(i)  # iterating the Series yields .item() scalars
        else:
            return None
        k = min(int(top_k), n)
        k1 = min(k + 1, n)
        mm = torch.empty(4, dtype=torch.float64, device=t.device)
        idx, sc, _ = _hrec.fuse_topk(a, t, self.als_f1_score > self.twotower_f1_score, k1, want_fused=False,
                                     minmax=mm)
        fin = torch.isfinite(t).all()
        if isinstance(als_side, tuple):
            fin = fin & torch.isfinite(a).all()
        bad = fin.logical_not().double().view(1)
        parts = [sc, idx.double(), mm, bad] + ([flags.double()] if flags is not None else [])
        host = torch.cat(parts).cpu().numpy()
        sc_h, idx_h, m = host[:k1], host[k1:2 * k1].astype(np.int64), host[2 * k1: 2 * k1 + 4]
        if flags is not None and host[2 * k1 + 5] != 0:
            self._flags_bad = True
            return None
        if host[2 * k1 + 4] != 0 or not np.all(sc_h[:-1] > sc_h[1:]):
            return None
        _set_fitted(self.als_scaler, m[0], m[1], n, np.float64)
        _set_fitted(self.twotower_scaler, m[2], m[3], n, np.float32)
        return [(item(int(i)), np.float64(s)) for i, s in zip(idx_h[:k], sc_h[:k])]

    def cleanup(self):
        if self.als_model:
            self.als_model.stop_spark()
