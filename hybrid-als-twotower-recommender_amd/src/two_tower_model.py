"""Two-tower content model — drop-in for the reference's src/two_tower_model.py.

Same class, methods, arguments and return values as src/two_tower_model.py:17-245.
The Keras graph (:38-89), `model.fit` (:111) and `model.predict` (:145) are
replaced by the device engine in tt_engine.py (hrec_tt_* / hrec_adam_* HIP
kernels). Host-side feature assembly (_prepare_features, the MinMaxScaler on
[price, average_review_rating]) is kept exactly, including the scaler refit
on every _prepare_features call.

Deviations from the committed reference (documented in DESIGN.md):
  * `if val_data:` on a DataFrame raises in the reference (D5); here
    val_data is tested with `is not None`, so EarlyStopping(patience=3,
    restore_best_weights=True) on val_loss works as the code intends. The
    ModelCheckpoint('tmp_best.keras') file is not written.
  * load_model's missing Keras import (D3) is not reproduced.
  * ids go through float32 like Keras Input(shape=(1,)) (D11) and must then
    index inside the tables (Keras raises there too).
"""
import os
import pickle

import numpy as np
import pandas as pd
import torch
from sklearn.model_selection import train_test_split  # noqa: F401  (reference import surface)
from sklearn.preprocessing import MinMaxScaler

from . import _hrec
from .tt_engine import TABLES, DeviceTwoTower


class History:
    """The subset of keras.callbacks.History the reference touches."""

    def __init__(self):
        self.history = {}
        self.epoch = []


def _ids(values, n, name):
    """Keras Input(shape=(1,)) is float32; Embedding casts to int32 (D11)."""
    a = np.asarray(values).astype(np.float32).astype(np.int64)
    if a.size and (a.min() < 0 or a.max() >= n):
        raise IndexError(f"{name}: id out of range [0, {n})")
    return a.astype(np.int32)


def _minmax_transform(scaler, frame, cols):
    """scaler.transform(frame[cols]) (:143). For a fitted MinMaxScaler over
    plain int / float64 columns this is sklearn's own arithmetic on a float64
    copy (X *= scale_; X += min_, sklearn/preprocessing/_data.py) without its
    per-call validation overhead (~2 ms per 100k rows); anything else — other
    scalers, clip, float32 or object columns, non-finite values, name or width
    mismatches — goes through scaler.transform itself."""
    sub = frame[cols]
    names = getattr(scaler, "feature_names_in_", None)
    if (type(scaler) is not MinMaxScaler or scaler.clip or not hasattr(scaler, "scale_") or len(sub) == 0
            or getattr(scaler, "n_features_in_", None) != len(cols)
            or (names is not None and list(names) != list(cols))
            or not all(dt == np.float64 or (dt.kind in "iu" and dt != np.bool_) for dt in sub.dtypes)):
        return scaler.transform(sub)
    X = sub.to_numpy(dtype=np.float64, copy=True)
    if np.isinf(X).any():
        return scaler.transform(sub)  # sklearn's own error
    X *= scaler.scale_
    X += scaler.min_
    return X


class TwoTowerModel:
    """Two-Tower Model Architecture (src/two_tower_model.py:17-36)."""

    def __init__(self, num_users, num_items, num_manufacturers, num_categories,
                 embedding_size=50, learning_rate=0.001, seed=0):
        self.num_users = num_users
        self.num_items = num_items
        self.num_manufacturers = num_manufacturers
        self.num_categories = num_categories
        self.embedding_size = embedding_size
        self.learning_rate = learning_rate
        self.model = None
        self.scaler = MinMaxScaler()
        self.is_trained = False
        self.seed = seed
        self._inputs_ws = None  # hrec_tt_item_inputs' presence bitmap, reused across calls

    def _build_item_tower(self):
        """(:38-66) -> (inputs, item_vec) as the reference returns them: the
        four inputs by their Input-layer names, and the tower itself —
        item_vec = LN(Dense(d)(concat[E_item, E_man(8), E_cat(8),
        relu(Dense(16)(numeric))])) — as a function of those inputs on the
        device (K4, csrc/tt_mfma.hip; the parameters build_model allocates)."""
        inputs = ["item_id_in", "manufacturer_in", "category_in", "numeric_in"]

        def item_vec(item_id_in, manufacturer_in, category_in, numeric_in):
            if self.model is None:
                raise RuntimeError("item tower: call build_model() first (it owns the tower's weights)")
            dev, sz = self.model.device, self.model.sizes
            ids = [torch.as_tensor(_ids(x, sz[t], name), device=dev)
                   for x, t, name in ((item_id_in, "item_emb", "item_id_in"), (manufacturer_in, "man_emb", "manufacturer_in"),
                                      (category_in, "cat_emb", "category_in"))]
            num = np.ascontiguousarray(np.asarray(numeric_in, dtype=np.float32).reshape(-1, 2))
            return self.model.item_vectors(*ids, torch.as_tensor(num, device=dev))

        return inputs, item_vec

    def build_model(self, init=None):
        """Allocate the parameters (Keras initialisers) on the device (:68-89)."""
        self.model = DeviceTwoTower(self.num_users, self.num_items, self.num_manufacturers, self.num_categories,
                                    self.embedding_size, self.learning_rate, seed=self.seed, init=init)
        return self.model

    # ------------------------------------------------------------ features
    def _prepare_features(self, data):
        if data is None:
            return None
        return {
            "user_in": data["userId"].values,
            "item_id_in": data["itemId"].values,
            "manufacturer_in": data["manufacturer_id"].values,
            "category_in": data["category_id"].values,
            "numeric_in": self.scaler.fit_transform(data[["price", "average_review_rating"]]),
        }

    def _device_inputs(self, feats):
        dev = self.model.device
        sz = self.model.sizes
        return (torch.as_tensor(_ids(feats["user_in"], sz["user_emb"], "user_in"), device=dev),
                torch.as_tensor(_ids(feats["item_id_in"], sz["item_emb"], "item_id_in"), device=dev),
                torch.as_tensor(_ids(feats["manufacturer_in"], sz["man_emb"], "manufacturer_in"), device=dev),
                torch.as_tensor(_ids(feats["category_in"], sz["cat_emb"], "category_in"), device=dev),
                torch.as_tensor(np.ascontiguousarray(np.asarray(feats["numeric_in"], dtype=np.float32).reshape(-1, 2)), device=dev))

    # --------------------------------------------------------------- train
    def _evaluate_loss(self, dev_inputs, y):
        pred = self.model.predict_rows(*dev_inputs).cpu().numpy()
        e = pred - y.cpu().numpy()
        return float(np.mean(e * e))

    def fit_batches(self, dev_inputs, y, batches):
        """Run train steps over explicit index batches (one Keras epoch with a
        given shuffle order); returns (sum_sq_err, sum_abs_err) over the epoch."""
        stats = []
        for idx in batches:
            idx_t = torch.as_tensor(np.asarray(idx, dtype=np.int64), device=self.model.device)
            parts = [t.index_select(0, idx_t).contiguous() for t in dev_inputs]  # batch assembly
            stats.append(self.model.train_step(*parts, y.index_select(0, idx_t).contiguous()))
        if not stats:
            return 0.0, 0.0
        st = torch.stack(stats).cpu().numpy().astype(np.float64)
        return float(st[:, 0].sum()), float(st[:, 1].sum())

    def train(self, train_data, val_data=None, batch_size=256, epochs=10, shuffle_seed=None):
        """Training process with early stopping (:91-121)."""
        if self.model is None:
            self.build_model()
        train_features = self._prepare_features(train_data)
        val_features = self._prepare_features(val_data) if val_data is not None else None
        dev_in = self._device_inputs(train_features)
        y = torch.as_tensor(np.asarray(train_data["average_review_rating"], dtype=np.float32),
                            device=self.model.device)
        if val_features is not None:
            val_in = self._device_inputs(val_features)
            val_y = torch.as_tensor(np.asarray(val_data["average_review_rating"], dtype=np.float32),
                                    device=self.model.device)
        n = len(y)
        rng = np.random.default_rng(self.seed if shuffle_seed is None else shuffle_seed)
        history = History()
        best, best_snap, wait = np.inf, None, 0
        for epoch in range(int(epochs)):
            order = rng.permutation(n)  # Keras fit(shuffle=True)
            batches = [order[s: s + batch_size] for s in range(0, n, batch_size)]
            sq, ab = self.fit_batches(dev_in, y, batches)
            history.epoch.append(epoch)
            history.history.setdefault("loss", []).append(sq / n)
            history.history.setdefault("mae", []).append(ab / n)
            if val_features is not None:
                vl = self._evaluate_loss(val_in, val_y)
                history.history.setdefault("val_loss", []).append(vl)
                # EarlyStopping(monitor='val_loss', patience=3, restore_best_weights=True)
                if vl < best:
                    best, best_snap, wait = vl, self.model.snapshot(), 0
                else:
                    wait += 1
                    if wait >= 3:
                        if best_snap is not None:
                            self.model.restore(best_snap)
                        break
        self.is_trained = True
        return history

    # ------------------------------------------------------------- predict
    def predict_for_user(self, user_id, item_features):
        """Generate predictions for one user over candidate rows (:136-146)."""
        scored = self._predict_device(user_id, item_features)
        return self._predictions(*scored) if scored else []

    def _score_device(self, inputs):
        """model.predict on the assembled inputs: f32 device scores [n]."""
        dev_in = self._device_inputs(inputs)
        u = dev_in[0][:1]
        uvec = self.model.user_vectors(u)
        ivec = self.model.item_vectors(*dev_in[1:])
        return _hrec.tt_score(uvec, ivec).reshape(-1)

    @staticmethod
    def _predictions(item_features, scores):
        predictions = scores.cpu().numpy().reshape(-1, 1)
        col = item_features["itemId"]
        # iterating a numpy-backed Series yields values.item(i), which is
        # what ndarray.tolist() builds in one call (same objects and types)
        keys = col.to_numpy().tolist() if isinstance(col.array, pd.arrays.NumpyExtensionArray) else col
        return list(zip(keys, predictions.flatten()))

    def _predict_device(self, user_id, item_features):
        """For HybridRecommendationSystem's array path: predict_for_user up to
        the device scores, (item_features, f32 device scores [n]); [] for an
        empty frame. Raises where predict_for_user raises."""
        inputs = {
            # the reference's np.full(len(item_features), user_id) column holds
            # one id n times, and one user vector serves every row
            # (_score_device): that id alone is converted and range-checked
            # (the same cast, the same error) and sent to the device
            "user_in": np.full(1, user_id),
            "item_id_in": item_features["itemId"].values,
            "manufacturer_in": item_features["manufacturer_id"].values,
            "category_in": item_features["category_id"].values,
            "numeric_in": _minmax_transform(self.scaler, item_features, ["price", "average_review_rating"]),
        }
        if len(item_features) == 0:
            return []
        return item_features, self._score_device(inputs)

    _FAST_ID_COLS = ("itemId", "manufacturer_id", "category_id")
    _FAST_NUM_COLS = ("price", "average_review_rating")

    def _predict_device_fast(self, user_id, item_features):
        """_predict_device for a plain candidate frame with the item-side
        input work on the device (hrec_tt_item_inputs: id casts and range
        checks, the MinMaxScaler transform, the candidates' uniqueness):
        (item_features, f32 device scores [n], device flags int32 [1]), or
        None when the frame or scaler is outside that path. Non-zero flags
        mean the inputs are NOT the model's (an id out of range, an infinite
        value, a repeated item id): the caller redoes the call through
        _predict_device, which raises where predict_for_user raises. The user
        id is checked here, on the host, first — as _device_inputs does."""
        sc = self.scaler
        if (self.model is None or type(sc) is not MinMaxScaler
                or sc.clip or not hasattr(sc, "scale_") or getattr(sc, "n_features_in_", None) != 2):
            return None
        names = getattr(sc, "feature_names_in_", None)
        if names is not None and list(names) != list(self._FAST_NUM_COLS):
            return None
        series = self._fast_columns(item_features)
        if series is None:
            return None
        n = len(item_features)
        cols = []
        for c, s in zip(self._FAST_ID_COLS + self._FAST_NUM_COLS, series):
            a = s.to_numpy()
            if not isinstance(a, np.ndarray) or a.ndim != 1 or len(a) != n:
                return None
            if c in self._FAST_ID_COLS:
                if a.dtype.kind not in "iu" or a.dtype == np.uint64:
                    return None
                a = a.astype(np.int64, copy=False)
            else:  # to_numpy(dtype=float64) of _minmax_transform: floats as they are, ints converted
                if not (a.dtype == np.float64 or (a.dtype.kind in "iu" and a.dtype != np.bool_)):
                    return None
                a = a.astype(np.float64, copy=False)
            cols.append(np.ascontiguousarray(a))
        dev, sz = self.model.device, self.model.sizes
        u = torch.as_tensor(_ids(np.full(1, user_id), sz["user_emb"], "user_in"), device=dev)
        t = [torch.from_numpy(a).to(dev) for a in cols]
        item, man, cat, num, flags, self._inputs_ws = _hrec.tt_item_inputs(
            *t, (sz["item_emb"], sz["man_emb"], sz["cat_emb"]), sc.scale_, sc.min_, self._inputs_ws)
        uvec = self.model.user_vectors(u)
        ivec = self.model.item_vectors(item, man, cat, num)
        return item_features, _hrec.tt_score(uvec, ivec).reshape(-1), flags

    def _fast_columns(self, item_features):
        """The five Series _predict_device reads, through the same lookups
        (frame["col"] for the ids, frame[[price, rating]] for the scaler), or
        None: an empty candidate set, a missing or repeated column, or a
        lookup that is not a plain Series. Besides a DataFrame this takes any
        candidates object answering those lookups from a frame (e.g. an item
        id array whose ["col"] comes from the item frame, bench.py)."""
        try:
            if len(item_features) == 0:
                return None
            if isinstance(item_features, pd.DataFrame):
                if not item_features.columns.is_unique or not all(
                        c in item_features.columns for c in self._FAST_ID_COLS + self._FAST_NUM_COLS):
                    return None
                return [item_features[c] for c in self._FAST_ID_COLS + self._FAST_NUM_COLS]
            ids = [item_features[c] for c in self._FAST_ID_COLS]
            sub = item_features[list(self._FAST_NUM_COLS)]
        except Exception:  # the host path makes the same lookups and reports the error
            return None
        if (not isinstance(sub, pd.DataFrame) or list(sub.columns) != list(self._FAST_NUM_COLS)
                or not all(type(s) is pd.Series for s in ids)):
            return None
        return ids + [sub[c] for c in self._FAST_NUM_COLS]

    # --------------------------------------------------------- persistence
    def save_model(self, model_path="models/twotower.keras"):
        os.makedirs(os.path.dirname(model_path) or ".", exist_ok=True)
        state = self.model.state_dict()
        state.update(self.model.optimizer_state())  # Keras saves the optimizer too (include_optimizer=True)
        meta = np.array([self.num_users, self.num_items, self.num_manufacturers, self.num_categories,
                         self.embedding_size], dtype=np.int64)
        with open(model_path, "wb") as f:
            np.savez(f, __meta__=meta, __lr__=np.float64(self.learning_rate), **state)
        with open(f"{model_path}_scaler.pkl", "wb") as f:
            pickle.dump(self.scaler, f)

    @classmethod
    def load_model(cls, model_path="models/twotower.keras"):
        with np.load(model_path, allow_pickle=False) as z:
            state = {k: z[k] for k in z.files}
        with open(f"{model_path}_scaler.pkl", "rb") as f:
            scaler = pickle.load(f)  # written by save_model above (own file)
        nu, ni, nm, nc, d = (int(x) for x in state["__meta__"])
        loaded_model = cls(nu, ni, nm, nc, d, float(state["__lr__"]))
        loaded_model.build_model(init={k: v for k, v in state.items() if not k.startswith("__")})
        loaded_model.model.iterations = int(state["__iterations__"])
        loaded_model.model.load_optimizer_state(state)
        loaded_model.scaler = scaler
        loaded_model.is_trained = True
        return loaded_model


def hyperparameter_tuning(train_data, param_grid, val_size=0.2, random_state=42):
    """F1-based grid search (:169-236) over the device model. np.random.choice
    with random_state= raises TypeError in the reference (D4); a seeded
    Generator is used instead."""
    best_params = None
    best_f1 = 0.0
    train_users = train_data["userId"].unique()
    rng = np.random.default_rng(random_state)
    val_users = rng.choice(train_users, size=int(len(train_users) * val_size), replace=False)
    train_sub = train_data[~train_data["userId"].isin(val_users)]
    val_sub = train_data[train_data["userId"].isin(val_users)]
    # D4b: the reference sizes the tables by train_sub's distinct counts
    # (:186-189), but ids index the tables: once the validation users are
    # removed the largest user id is (almost surely) >= that count, Keras'
    # lookup raises, every grid point is skipped (:232-234) and the function
    # can only return None. Tables sized max(id) + 1 over train_data let the
    # loop do what it is written for.
    num_users = int(train_data["userId"].max()) + 1
    num_items = int(train_data["itemId"].max()) + 1
    num_man = int(train_data["manufacturer_id"].max()) + 1
    num_cat = int(train_data["category_id"].max()) + 1
    for params in param_grid:
        print(f"\nTesting parameters: {params}")
        try:
            model = TwoTowerModel(num_users=num_users, num_items=num_items, num_manufacturers=num_man,
                                  num_categories=num_cat, embedding_size=50, learning_rate=0.001)
            model.train(train_sub, val_sub, batch_size=params["batch_size"], epochs=params["epochs"])
            f1_scores = []
            items = val_sub[["itemId", "manufacturer_id", "category_id", "price",
                             "average_review_rating"]].drop_duplicates()
            for user_id in val_sub["userId"].unique()[:50]:
                sel = val_sub[val_sub["userId"] == user_id]
                actual = dict(zip(sel["itemId"], sel["average_review_rating"]))
                preds = model.predict_for_user(user_id, items)
                f1_scores.append(compute_f1_score(actual, dict(preds), k=10))
            avg_f1 = np.mean(f1_scores)
            print(f"  Avg F1@10: {avg_f1:.4f}")
            if avg_f1 > best_f1:
                best_f1 = avg_f1
                best_params = params.copy()
        except Exception as e:
            print(f"  Error with params {params}: {str(e)}")
            continue
    return best_params


def compute_f1_score(actual, pred, k=10):
    """src/two_tower_model.py:238-245 (k > 0 guarded)."""
    actual_items = set(actual.keys())
    pred_items = set(item for item, _ in sorted(pred.items(), key=lambda x: x[1], reverse=True)[:k])
    tp = len(actual_items & pred_items)
    precision = tp / k if k > 0 else 0
    recall = tp / len(actual_items) if len(actual_items) > 0 else 0
    return 2 * (precision * recall) / (precision + recall) if (precision + recall) > 0 else 0
