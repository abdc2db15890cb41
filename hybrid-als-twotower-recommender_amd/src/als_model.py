"""ALS collaborative filtering — drop-in for the reference's src/als_model.py.

Same class, method names, arguments, return values and error sentinels as
src/als_model.py:21-177; the Spark engine underneath (ALS.fit at :62,
ALSModel.transform at :75) is replaced by libhrec's HIP kernels:

  train            -> device CSR/CSC ingest + hrec_als_init_factors +
                      max_iter x (item half-sweep, user half-sweep)  [K1]
                      (under an initialised torch.distributed world of W
                      > 1 ranks — torchrun, one GPU per rank — every rank
                      calls train with the same frame; the users and items
                      are split into nnz-balanced row shards, the factors
                      replicated by RCCL all-gathers after each half-sweep,
                      and every rank ends with the full model: the factors
                      are bit-identical to the one-rank fit)
  predict_for_user -> hrec_als_score (JVM-exact f32 dot, NaN for unknown
                      ids = coldStartStrategy "drop")                [K2]
                      + cold-start fallback via hrec_cosine_sim +
                      hrec_topk_f64 (_find_similar_items)            [K3]

`initialize_spark` / `stop_spark` keep their names: they bind / release the
HIP device session that plays the SparkSession's role.
"""
import json
import os
import pickle
import time
import warnings

import numpy as np
import torch

from . import _hrec
from .als_engine import DeviceALS, padded_k, process_group
from .als_ingest import check_same_frame, frame_fingerprint, sharded_ingest
from .data_preprocessing import get_item_features
from .synthetic import DeviceCSR

warnings.filterwarnings("ignore")


class DeviceSession:
    """What SparkSession is to the reference: the engine handle (one HIP
    device, its default stream)."""

    def __init__(self, device=None):
        _hrec.require_device()
        _hrec.lib()
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)

    def stop(self):
        torch.cuda.synchronize(self.device)


class DeviceALSFactors:
    """The fitted model (Spark's ALSModel): ids + factor matrices on the device."""

    def __init__(self, user_ids, item_ids, U, V, k):
        self.user_ids = np.asarray(user_ids)   # sorted unique raw ids
        self.item_ids = np.asarray(item_ids)
        self.U = U                               # [n_users, kp] f32 device
        self.V = V                               # [n_items, kp] f32 device
        self.k = int(k)
        self.Vt = _hrec.transpose(V) if V.shape[0] else V.t().contiguous()
        self._item_ids_dev = None

    @staticmethod
    def _lookup(ids, keys):
        keys = np.fromiter(keys, np.int64, len(keys)) if isinstance(keys, list) else np.asarray(keys)
        if len(ids) == 0:
            return np.full(keys.shape, -1, dtype=np.int64)
        pos = np.searchsorted(ids, keys)
        pos = np.clip(pos, 0, len(ids) - 1)
        ok = ids[pos] == keys
        return np.where(ok, pos, -1).astype(np.int64)

    def _lookup_device(self, keys):
        """_lookup for long candidate lists: the same binary search on the
        device over a cached copy of the sorted item ids."""
        dev = self.U.device
        if self._item_ids_dev is None:
            self._item_ids_dev = torch.as_tensor(np.asarray(self.item_ids, np.int64), device=dev)
        ids = self._item_ids_dev
        k = torch.as_tensor(keys, device=dev)
        if ids.numel() == 0:
            return torch.full_like(k, -1)
        pos = torch.searchsorted(ids, k).clamp_(max=ids.numel() - 1)
        return torch.where(ids[pos] == k, pos, torch.full_like(pos, -1))

    def score(self, user_ids, item_list):
        """f32 [len(user_ids), len(item_list)]; NaN where either id is unknown."""
        dev = self.U.device
        urows_h = self._lookup(self.user_ids, user_ids)
        if urows_h.size and (urows_h < 0).all():  # unknown users only: NaN everywhere, no transform to run
            return torch.full((urows_h.size, len(item_list)), float("nan"), dtype=torch.float32, device=dev)
        urows = torch.as_tensor(urows_h, device=dev)
        if isinstance(item_list, np.ndarray) and item_list.dtype == np.int64 and item_list.size > 4096:
            irows = self._lookup_device(item_list)
        else:
            irows = torch.as_tensor(self._lookup(self.item_ids, item_list), device=dev)
        return _hrec.als_score(self.U, urows, self.Vt, irows, irows.numel(), self.k)

    # Spark 3.5 ALSModel directory layout (MLWriter): metadata/part-00000 is
    # one JSON line with the model params and "rank"; userFactors/ and
    # itemFactors/ are parquet datasets of (id: int, features: array<float>).
    # A model saved here loads in Spark and vice versa.
    def save(self, path, params=None):
        import uuid

        import pyarrow as pa
        import pyarrow.parquet as pq

        meta = {"class": "org.apache.spark.ml.recommendation.ALSModel", "timestamp": int(time.time() * 1000),
                "sparkVersion": "3.5.1", "uid": f"ALS_{uuid.uuid4().hex[:12]}",
                "paramMap": dict(params or {}),
                "defaultParamMap": {"blockSize": 4096, "predictionCol": "prediction", "itemCol": "item",
                                    "userCol": "user", "coldStartStrategy": "nan"},
                "rank": self.k}
        os.makedirs(os.path.join(path, "metadata"), exist_ok=True)
        with open(os.path.join(path, "metadata", "part-00000"), "w") as f:
            f.write(json.dumps(meta, separators=(",", ":")) + "\n")
        open(os.path.join(path, "metadata", "_SUCCESS"), "w").close()
        feat_t = pa.list_(pa.field("element", pa.float32(), nullable=False))
        for name, ids, fac in (("userFactors", self.user_ids, self.U), ("itemFactors", self.item_ids, self.V)):
            d = os.path.join(path, name)
            os.makedirs(d, exist_ok=True)
            mat = fac[:, : self.k].cpu().numpy()
            feats = pa.FixedSizeListArray.from_arrays(pa.array(mat.reshape(-1), pa.float32()), self.k)
            table = pa.table({"id": pa.array(np.asarray(ids, np.int32), pa.int32()),
                              "features": feats.cast(feat_t)})
            pq.write_table(table, os.path.join(d, f"part-00000-{uuid.uuid4()}-c000.snappy.parquet"),
                           compression="snappy")
            open(os.path.join(d, "_SUCCESS"), "w").close()

    @classmethod
    def load(cls, path, device):
        import pyarrow.parquet as pq

        with open(os.path.join(path, "metadata", "part-00000")) as f:
            k = int(json.loads(f.readline())["rank"])
        kp = padded_k(k)

        def fac(name):
            t = pq.read_table(os.path.join(path, name))
            ids = np.asarray(t.column("id").to_numpy(), np.int64)
            flat = t.column("features").combine_chunks().flatten().to_numpy(zero_copy_only=False)
            mat = np.asarray(flat, np.float32).reshape(len(ids), k)
            order = np.argsort(ids, kind="stable")  # Spark writes partitions in any order
            out = torch.zeros((len(ids), kp), dtype=torch.float32, device=device)
            out[:, :k] = torch.as_tensor(mat[order], device=device)
            return ids[order], out

        user_ids, U = fac("userFactors")
        item_ids, V = fac("itemFactors")
        return cls(user_ids, item_ids, U, V, k)


class _PyInts:
    """Candidate ids from a pandas Index / Series: element i is the Python int
    the Series iteration yields (vals.item(i)); the list is built only if
    someone iterates (the per-item list path)."""

    def __init__(self, vals):
        self.vals = vals

    def __len__(self):
        return len(self.vals)

    def __getitem__(self, i):
        return self.vals.item(i)

    def __iter__(self):
        return iter(self.vals.tolist())


def _int_ids(col, name):
    a = np.asarray(col)
    if a.dtype.kind == "f":
        if not np.all(np.isfinite(a)) or not np.all(a == np.floor(a)):
            raise ValueError(f"{name} must hold integer ids (Spark casts them to Int)")
        a = a.astype(np.int64)
    if a.dtype.kind not in "iu":
        raise ValueError(f"{name} must hold integer ids, got dtype {a.dtype}")
    a = a.astype(np.int64)
    if a.size and (a.min() < -(2 ** 31) or a.max() >= 2 ** 31):
        raise ValueError(f"{name} ids must fit a 32-bit Int (Spark ALS)")
    return a


def build_csr(rows, cols, vals, n_rows, n_cols, alias=False, rows_in_order=None, indptr=None):
    """Device CSR of COO ratings (hrec_coo_to_csr): rows ascending, a row's
    entries in input order; duplicate (u, i) ratings stay separate terms, as
    in Spark. rows/cols int32, vals f32, all device tensors. alias: rows
    already in order hand back cols / vals themselves (no copy);
    rows_in_order / indptr: the rows' order and row pointer when known (from
    encode_ids(..., order=True); else checked / built on the device)."""
    indptr, indices, values = _hrec.coo_to_csr(rows, cols, vals, int(n_rows), alias=alias,
                                               rows_in_order=rows_in_order, indptr=indptr)
    return DeviceCSR(indptr, indices, values, 0, int(n_rows), int(n_cols))


def java_string_hash(s):
    """java.lang.String.hashCode (s[0] 31^(n-1) + ... + s[n-1], int32)."""
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


def default_seed():
    """Spark ALS's default seed, HasSeed's this.getClass.getName.hashCode:
    the same in every process (Python's str hash is salted per process, so a
    torchrun world would start each rank from other factors)."""
    return java_string_hash("org.apache.spark.ml.recommendation.ALS") & ((1 << 63) - 1)


class ALSModel:
    """src/als_model.py:21 — same constructor signature (+ optional seed)."""

    CHUNKS = 4  # W > 1: user-side row chunks per rank (overlapped all-gathers)

    def __init__(self, rank=10, max_iter=10, reg_param=0.1, cold_start_strategy="drop", seed=None):
        self.rank = rank
        self.max_iter = max_iter
        self.reg_param = reg_param
        self.cold_start_strategy = cold_start_strategy
        self.model = None
        self.spark = None
        self.global_mean = 3.0
        self.item_features = None
        self.seed = seed
        self.ingest_peak_bytes = None  # device bytes the last train's ingest peaked at (cuda only)

    @property
    def item_features(self):
        return self._item_features

    @item_features.setter
    def item_features(self, value):
        """Assigning the features (train, load_model, a caller) drops what was
        derived from them: the feature matrix and the cold-start fallback."""
        self._item_features = value
        self._feat_cache = None
        self._fb_cache = None
        self._fb_keys = None

    # -------------------------------------------------------- engine handle
    def initialize_spark(self):
        try:
            if self.spark is None:
                self.spark = DeviceSession()
            return True
        except Exception as e:
            print(f"Spark init error: {str(e)}")
            return False

    def stop_spark(self):
        if self.spark:
            self.spark.stop()

    # ---------------------------------------------------------------- train
    def _fit(self, data, U0=None):
        if self.cold_start_strategy not in ("drop", "nan"):
            raise ValueError(f"coldStartStrategy {self.cold_start_strategy!r} is not supported")
        dev = self.spark.device
        users_h = _int_ids(data["userId"], "userId")
        items_h = _int_ids(data["itemId"], "itemId")
        ratings_h = np.asarray(data["average_review_rating"], dtype=np.float32)
        k = int(self.rank)
        world, rank, group = process_group()
        track = dev.type == "cuda"
        if track:  # the ingest's peak device memory (tests: W = 2 holds about half of W = 1)
            torch.cuda.synchronize(dev)
            base = torch.cuda.memory_allocated(dev)
            torch.cuda.reset_peak_memory_stats(dev)
        if world > 1:
            # this rank's slice of the frame only; ids encoded
            # over the whole frame, this rank's nnz-balanced row parts built
            # from the ratings exchanged to it (src/als_ingest.py)
            check_same_frame(frame_fingerprint(users_h, items_h, ratings_h), dev, group)
            user_ids, item_ids, csr, csc, ulay, ilay = sharded_ingest(users_h, items_h, ratings_h, world, rank, group,
                                                                      self.CHUNKS, dev)
            n_u, n_i = len(user_ids), len(item_ids)
        else:
            users, items = torch.as_tensor(users_h).to(dev), torch.as_tensor(items_h).to(dev)
            ratings = torch.as_tensor(ratings_h).to(dev)
            # ingest on the device (§8(f) row 1): dense codes + CSR (users) / CSC (items)
            rng = (lambda a: (int(a.min()), int(a.max())) if a.size else None)
            user_ids_t, urow, u_ord, u_ptr = _hrec.encode_ids(users, rng(users_h), order=True)
            item_ids_t, irow, i_ord, _ = _hrec.encode_ids(items, rng(items_h), order=True)
            user_ids, item_ids = user_ids_t.cpu().numpy(), item_ids_t.cpu().numpy()
            n_u, n_i = len(user_ids), len(item_ids)
            # ratings grouped by user: the row pointer came with the codes, the CSR is the input (no pass)
            csr = build_csr(urow, irow, ratings, n_u, n_i, alias=True, rows_in_order=u_ord, indptr=u_ptr)
            csc = build_csr(irow, urow, ratings, n_i, n_u, rows_in_order=i_ord)
            del urow, irow, ratings, users, items, user_ids_t, item_ids_t
        if track:
            torch.cuda.synchronize(dev)
            self.ingest_peak_bytes = int(torch.cuda.max_memory_allocated(dev) - base)
        if world > 1:
            eng = DeviceALS(n_u, n_i, k, float(self.reg_param), csr, csc, world=world, rank=rank, group=group,
                            chunks=self.CHUNKS, item_chunks=1, user_layout=ulay, item_layout=ilay)
        else:
            eng = DeviceALS(n_u, n_i, k, float(self.reg_param), csr, csc)
        if U0 is not None:
            eng.set_user_factors(U0)
        else:
            seed = default_seed() if self.seed is None else int(self.seed) & ((1 << 63) - 1)
            if world > 1:  # every rank starts from rank 0's factors
                t = torch.tensor([seed], dtype=torch.int64, device=dev)
                torch.distributed.broadcast(t, 0, group=group)
                seed = int(t.item())
            eng.init_user_factors(seed)
        eng.fit(int(self.max_iter))
        if world == 1:
            U, V = eng.U[:n_u].contiguous(), eng.V[:n_i].contiguous()
        else:  # every rank holds the replicated factors; back to global row order
            U = torch.zeros((n_u, eng.kp), dtype=torch.float32, device=dev)
            V = torch.zeros((n_i, eng.kp), dtype=torch.float32, device=dev)
            U[:, :k] = eng.user_factors
            V[:, :k] = eng.item_factors
        return DeviceALSFactors(user_ids, item_ids, U, V, k)

    def train(self, data, initial_user_factors=None):
        """src/als_model.py:43-66. `initial_user_factors` (optional, [n_users, rank]
        in sorted-userId order) injects Spark's random init for parity runs."""
        try:
            if not self.initialize_spark():
                return False
            self.item_features = get_item_features(data)
            self.global_mean = data["average_review_rating"].mean()
            self.model = self._fit(data, initial_user_factors)
            return True
        except Exception as e:
            print(f"Training error: {str(e)}")
            return False

    # --------------------------------------------------------------- predict
    @staticmethod
    def _check_int_ids(values):
        """Spark's createDataFrame(pairs, IntegerType schema) at :71-75
        rejects non-integer ids (e.g. the column names of a DataFrame, SURVEY
        D9). One pass over the distinct element types; the slow per-item scan
        only runs to name the offending value."""
        def ok(t):
            return issubclass(t, (int, np.integer)) and not issubclass(t, (bool, np.bool_))

        if all(ok(t) for t in set(map(type, values))):
            return
        for x in values:
            if not ok(type(x)):
                raise TypeError(f"field itemId: IntegerType() can not accept object {x!r} in type {type(x)}")

    @staticmethod
    def _id_array(all_items):
        """(items, int64 keys) for an integer numpy array / pandas Index /
        Series of candidate ids without a per-element Python pass, else None.
        `items` is indexable and iterates like `all_items` does in the
        reference's loop (:70): a numpy array yields numpy scalars, an Index or
        Series Python ints."""
        if isinstance(all_items, np.ndarray):
            if all_items.ndim == 1 and all_items.dtype.kind in "iu":
                return all_items, np.asarray(all_items).astype(np.int64, copy=False)
            return None
        import pandas as pd

        if isinstance(all_items, (pd.Index, pd.Series)) and all_items.dtype.kind in "iu":
            vals = all_items.to_numpy()
            return _PyInts(vals), vals.astype(np.int64, copy=False)
        return None

    def _score_device(self, user_id, all_items):
        """predict_for_user up to the transform: (items, int64 keys, f32 device
        scores [n] or None). Raises where the reference's createDataFrame /
        transform would."""
        self._check_int_ids([user_id])
        fast = self._id_array(all_items)
        if fast is not None:
            items, keys = fast
        else:
            items = list(all_items)
            self._check_int_ids(items)
            keys = np.fromiter(items, np.int64, len(items)) if items else None
        if len(items) == 0:
            return items, None, None
        return items, keys, self.model.score([user_id], keys)[0]

    def _predict_device(self, user_id, all_items):
        """For HybridRecommendationSystem's array path: (items, keys, f32
        device scores), else the predict_for_user list itself (same prints,
        same []). A user the model does not know (every row NaN: the
        reference protocol's test users) gets the fallback vector
        gathered for the candidates (f64, _cold_scores) when it applies; other
        NaN rows (unknown items) stay NaN, and the array path sends them to
        the list path, which applies the fallback through _predictions."""
        try:
            items, keys, scores = self._score_device(user_id, all_items)
            if scores is not None:
                if self.model._lookup(self.model.user_ids, [user_id])[0] < 0:
                    cold = self._cold_scores(keys)
                    if cold is not None:
                        scores = cold
                return items, keys, scores
            return self._predictions(items, scores)
        except Exception as e:
            print(f"Prediction error: {str(e)}")
            return []

    def predict_for_user(self, user_id, all_items):
        try:
            items, _, scores = self._score_device(user_id, all_items)
            return self._predictions(items, scores)
        except Exception as e:
            print(f"Prediction error: {str(e)}")
            return []

    def _predictions_guarded(self, items, scores):
        """_predictions under predict_for_user's own error contract (:68-91):
        a failing cold-start fallback prints 'Prediction error: ...' and gives
        [] for the ALS side only — for callers that took the scores through
        _predict_device and finish the list later (the hybrid's list path)."""
        try:
            return self._predictions(items, scores)
        except Exception as e:
            print(f"Prediction error: {str(e)}")
            return []

    def _predictions(self, items, scores):
        """The (item, prediction) list of :84 with the cold-start fallback
        (:78-86) for rows the transform left NaN: the per-item values of the
        precomputed fallback vector (_fallback), or — for features the kernel
        does not take — the per-call similarity search."""
        scores = scores.cpu().numpy() if scores is not None else np.zeros(0, np.float32)
        out = list(zip(items, scores.tolist()))  # (item, float(prediction)) as :84
        missing = np.flatnonzero(np.isnan(scores)).tolist()
        if not missing:
            return out
        # cold-start fallback (:78-86): mean rating of <= 3 similar items, else the global mean
        if self.item_features is not None:
            self._check_finite_features([items[n] for n in missing])
        fb = self._fallback() if self.item_features is not None else None
        if fb is not None:
            pos, mean, cnt = fb["pos"], fb["mean_h"], fb["cnt_h"]
            for n in missing:
                p = pos.get(items[n])  # the reference's item_features[item] (KeyError -> [] -> global mean)
                out[n] = (items[n], mean[p] if p is not None and cnt[p] > 0 else self.global_mean)
            return out
        sims = self._similar_batch([items[n] for n in missing])
        for n, sim in zip(missing, sims):
            out[n] = (items[n], np.mean([self.item_features[s]["rating"] for s in sim]) if sim
                      else self.global_mean)
        return out

    def _check_finite_features(self, query_items):
        """sklearn's cosine_similarity (:100) validates both arrays: a NaN or
        infinite feature vector anywhere in item_features raises ValueError
        from the reference's loop as soon as an item with features needs the
        fallback (and has another item to compare with)."""
        ids, pos, mat = self._feature_matrix()
        bad = self._feat_cache[4]
        if bad is None or len(ids) < 2 or not any(it in pos for it in query_items):
            return
        raise ValueError(bad)

    def _features_key(self):
        f = self.item_features
        return id(f), (len(f) if f is not None else -1)

    def _feature_matrix(self):
        key = self._features_key()
        if self._feat_cache is None or self._feat_cache[0] != key:
            feats = self.item_features or {}
            ids = list(feats.keys())
            bad = None
            if ids:
                mat = np.stack([np.asarray(feats[i]["features"], dtype=np.float64).ravel() for i in ids])
                dev_mat = torch.as_tensor(mat, device=self.spark.device if self.spark else "cuda")
                if not np.isfinite(mat).all():  # sklearn check_array's messages
                    bad = ("Input contains NaN." if np.isnan(mat).any() else
                           "Input contains infinity or a value too large for dtype('float64').")
            else:
                dev_mat = None
            self._feat_cache = (key, ids, {i: n for n, i in enumerate(ids)}, dev_mat, bad)
        return self._feat_cache[1:4]

    def _fallback(self):
        """The cold-start fallback of every item with features, computed once
        per item_features on the device (hrec_cold_fallback: the <= 3 most
        similar other items with cosine > 0.5 of :93-104 and np.mean of their
        ratings — the value of :84-85 for any user). A dict with "pos" (item
        -> row), "mean_h" (np.float64 per row), "cnt_h" (similar items kept)
        and their device copies; None when the features are outside the
        kernel (wider than 16, or ratings that are not Python / numpy f64
        floats, whose np.mean would run in another dtype), or absent."""
        key = self._features_key()
        if self._fb_cache is not None and self._fb_cache[0] == key:
            return self._fb_cache[1]
        ids, pos, mat = self._feature_matrix()
        fb = None
        feats = self.item_features
        if mat is not None and mat.shape[1] <= _hrec.COLD_MAX_DIM:
            r = [feats[i]["rating"] for i in ids]
            # np.mean converts ints (not bools) to f64 the same way; float32 etc. would sum in their dtype
            if all(type(x) in (float, int, np.float64, np.int64) for x in r):
                ratings = torch.as_tensor(np.asarray(r, np.float64), device=mat.device)
                mean, cnt, _ = _hrec.cold_fallback(mat, ratings)
                fb = {"ids": ids, "pos": pos, "mean": mean, "cnt": cnt, "mean_h": mean.cpu().numpy(),
                      "cnt_h": cnt.cpu().numpy()}
        self._fb_cache = (key, fb)
        self._fb_keys = None
        return fb

    def _cold_scores(self, keys):
        """For a cold user on the hybrid's array path: f64 device [n], the
        fallback value of each candidate key (global mean where the item has
        no features or no similar item), or None when _fallback is None, the
        features are not finite or the feature ids are not integers. Cached
        for the last candidate set."""
        if self.item_features is None:
            return None
        fb = self._fallback()
        if fb is None or self._feat_cache[4] is not None:  # non-finite features: the list path raises
            return None
        c = self._fb_keys
        if c is not None and c[0] is fb and c[1].shape == keys.shape and np.array_equal(c[1], keys):
            return c[2]
        if "sorted" not in fb:
            arr = np.asarray(fb["ids"])
            fb["sorted"] = None
            if arr.dtype.kind in "iu" and arr.dtype != np.uint64:
                order = np.argsort(arr, kind="stable")
                dev = fb["mean"].device
                fb["sorted"] = (torch.as_tensor(arr[order].astype(np.int64), device=dev),
                                torch.as_tensor(order.astype(np.int64), device=dev))
        if fb["sorted"] is None:
            return None
        sid, order = fb["sorted"]
        k = torch.as_tensor(np.asarray(keys, np.int64), device=sid.device)
        p = torch.searchsorted(sid, k).clamp_(max=sid.numel() - 1)
        row = order[p]
        hit = (sid[p] == k) & (fb["cnt"][row] > 0)
        gm = torch.full_like(fb["mean"][:1], float(self.global_mean))
        vals = torch.where(hit, fb["mean"][row], gm)
        self._fb_keys = (fb, np.array(keys, np.int64, copy=True), vals)
        return vals

    def _similar_batch(self, query_items, k=3):
        """_find_similar_items for many items at once on the device: cosine
        similarities (hrec_cosine_sim) + stable top-k (dict order breaks
        ties, like the reference's sorted()) + the sim > 0.5 filter."""
        if self.item_features is None:
            raise TypeError("'NoneType' object is not subscriptable")  # reference: None[item_id]
        ids, pos, mat = self._feature_matrix()
        res = [[] for _ in query_items]
        q = [(n, pos[it]) for n, it in enumerate(query_items) if it in pos]
        if not q or mat is None:
            return res
        dev = mat.device
        for s in range(0, len(q), 4096):
            chunk = q[s: s + 4096]
            qrows = torch.as_tensor([r for _, r in chunk], dtype=torch.int64, device=dev)
            sims = _hrec.cosine_sim(mat, qrows)
            idx, val = _hrec.topk(sims, k)
            idx, val = idx.cpu().numpy(), val.cpu().numpy()
            for (n, _), ii, vv in zip(chunk, idx, val):
                res[n] = [ids[j] for j, v in zip(ii, vv) if j >= 0 and v > 0.5]
        return res

    def _find_similar_items(self, item_id, k=3):
        try:
            self.item_features[item_id]
            return self._similar_batch([item_id], k)[0]
        except KeyError:
            return []

    # ----------------------------------------------------------- persistence
    def save_model(self, model_path="models/als"):
        try:
            os.makedirs(os.path.dirname(model_path) or ".", exist_ok=True)
            self.model.save(model_path, {"userCol": "userId", "itemCol": "itemId", "predictionCol": "prediction",
                                         "coldStartStrategy": self.cold_start_strategy, "blockSize": 4096})
            metadata = {
                "rank": self.rank,
                "max_iter": self.max_iter,
                "reg_param": self.reg_param,
                "global_mean": self.global_mean,
                "item_features": self.item_features,
            }
            with open(f"{model_path}_metadata.pkl", "wb") as f:
                pickle.dump(metadata, f)
            print(f"Model saved to {model_path}")
        except Exception as e:
            print(f"Saving error: {str(e)}")

    def load_model(self, model_path="models/als"):
        try:
            if not self.initialize_spark():
                raise RuntimeError("no device session")
            self.model = DeviceALSFactors.load(model_path, self.spark.device)
            with open(f"{model_path}_metadata.pkl", "rb") as f:
                metadata = pickle.load(f)  # written by save_model above (own format)
                self.rank = metadata["rank"]
                self.max_iter = metadata["max_iter"]
                self.reg_param = metadata["reg_param"]
                self.global_mean = metadata["global_mean"]
                self.item_features = metadata["item_features"]
            return self
        except Exception as e:
            print(f"Loading error: {str(e)}")
            return None


def hyperparameter_tuning(train_data, val_data, param_grid):
    """src/als_model.py:142-169 (driver loop over the device ALS)."""
    best_params = None
    best_f1 = 0.0
    for params in param_grid:
        model = ALSModel(**params)
        if not model.train(train_data):
            continue
        f1_scores = []
        for user_id in val_data["userId"].sample(50).unique():
            sel = val_data[val_data["userId"] == user_id]
            actual = dict(zip(sel["itemId"], sel["average_review_rating"]))
            preds = model.predict_for_user(user_id, val_data["itemId"].unique())
            f1_scores.append(compute_f1_score(actual, {item: score for item, score in preds}))
        avg_f1 = np.mean(f1_scores)
        if avg_f1 > best_f1:
            best_f1 = avg_f1
            best_params = params.copy()
        model.stop_spark()
    return best_params


def compute_f1_score(actual, pred, k=10):
    """src/als_model.py:171-177 (k = 0 raises ZeroDivisionError, as there)."""
    actual_items = set(actual.keys())
    pred_items = set(item for item, _ in sorted(pred.items(), key=lambda x: x[1], reverse=True)[:k])
    tp = len(actual_items & pred_items)
    precision = tp / k
    recall = tp / len(actual_items) if actual_items else 0
    return 2 * (precision * recall) / (precision + recall) if (precision + recall) > 0 else 0
