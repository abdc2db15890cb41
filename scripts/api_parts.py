"""Host/device split of one get_hybrid_recommendations call on the array path
(c2: 100k candidate items, rank 64, d 64): times each part over many reps."""
import contextlib
import io
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hybrid-als-twotower-recommender_amd"))
from sklearn.preprocessing import MinMaxScaler  # noqa: E402

from src.als_model import ALSModel, DeviceALSFactors, DeviceSession  # noqa: E402
from src.hybrid_system import HybridRecommendationSystem  # noqa: E402
from src.two_tower_model import TwoTowerModel, _minmax_transform  # noqa: E402

n_users, n_items, k, reps = 100_000, 100_000, 64, 50
out = sys.stdout
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)
U = torch.randn(n_users, k, device=dev, generator=g) * 0.1
V = torch.randn(n_items, k, device=dev, generator=g) * 0.1
als = ALSModel(rank=k)
als.spark = DeviceSession()
als.model = DeviceALSFactors(np.arange(n_users), np.arange(n_items), U, V, k)
als.item_features = {}
tt = TwoTowerModel(n_users, n_items, 2651, 255, embedding_size=64, seed=4)
tt.build_model()
rng = np.random.default_rng(9)
items = pd.DataFrame({"itemId": np.arange(n_items), "manufacturer_id": rng.integers(0, 2651, n_items),
                      "category_id": rng.integers(0, 255, n_items), "price": rng.random(n_items) * 100,
                      "average_review_rating": rng.integers(0, 19, n_items).astype(np.float64)})
tt.scaler = MinMaxScaler().fit(items[["price", "average_review_rating"]])
h = HybridRecommendationSystem()
h.als_model, h.twotower_model, h.models_loaded = als, tt, True
ids = [int(i) for i in items["itemId"]]


class Candidates:
    def __iter__(self):
        return iter(ids)

    def __len__(self):
        return len(items)

    def __getitem__(self, key):
        return items[key]


both = Candidates()


class IdArray(np.ndarray):
    def __getitem__(self, key):
        if isinstance(key, (str, list)):
            return items[key]
        return super().__getitem__(key)


arr = items["itemId"].to_numpy().view(IdArray)
keys = np.asarray(arr)


def timed(name, fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print(f"{name:44s} {(time.perf_counter() - t0) / reps * 1e3:8.3f} ms", file=out, flush=True)


a_side = als._predict_device(3, both)
t_side = tt._predict_device(3, items)
with contextlib.redirect_stdout(io.StringIO()):
    timed("api call (both sides)", lambda: h.get_hybrid_recommendations(3, both, top_k=5))
    timed("api call (reference wiring)", lambda: h.get_hybrid_recommendations(3, items, top_k=5))
    timed("api call (id array)", lambda: h.get_hybrid_recommendations(3, arr, top_k=5))
timed("ALS _predict_device (id array)", lambda: als._predict_device(3, arr))
timed("ALS keys H2D", lambda: torch.as_tensor(keys, device=dev))
timed("ALS _lookup_device", lambda: als.model._lookup_device(keys))
irows = als.model._lookup_device(keys)
urow = torch.as_tensor(als.model._lookup(als.model.user_ids, [3]), device=dev)
from src import _hrec  # noqa: E402
timed("ALS als_score", lambda: _hrec.als_score(als.model.U, urow, als.model.Vt, irows, n_items, k))
timed("ALS model.score", lambda: als.model.score([3], keys))
timed("array_equal(keys, vals)", lambda: np.array_equal(keys, items["itemId"].values))
timed("frame[[price, rating]]", lambda: items[["price", "average_review_rating"]])
timed("TT _fast_columns (frame)", lambda: tt._fast_columns(items))
timed("TT _fast_columns (id array)", lambda: tt._fast_columns(arr))
timed("TT _predict_device_fast (id array)", lambda: tt._predict_device_fast(3, arr))
a_arr = als._predict_device(3, arr)
t_arr = tt._predict_device_fast(3, arr)
timed("_top_on_device (id array, flags)", lambda: h._top_on_device(a_arr, t_arr[:2], 5, flags=t_arr[2]))
timed("ALS list(all_items)", lambda: list(both))
timed("ALS _check_int_ids", lambda: ALSModel._check_int_ids(ids))
timed("ALS fromiter", lambda: np.fromiter(ids, np.int64, len(ids)))
timed("ALS _predict_device", lambda: als._predict_device(3, both))
timed("TT _minmax_transform", lambda: _minmax_transform(tt.scaler, items, ["price", "average_review_rating"]))
timed("TT _predict_device", lambda: tt._predict_device(3, items))
timed("TT _predict_device_fast", lambda: tt._predict_device_fast(3, items))
cols = [torch.from_numpy(items[c].to_numpy()) for c in ("itemId", "manufacturer_id", "category_id", "price",
                                                         "average_review_rating")]
timed("TT H2D of the 5 columns", lambda: [c.to(dev) for c in cols])
timed("_top_on_device", lambda: h._top_on_device(a_side, t_side, 5))

if os.environ.get("API_PROFILE"):
    import cProfile
    import pstats

    with contextlib.redirect_stdout(io.StringIO()):
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(reps):
            h.get_hybrid_recommendations(3, arr, top_k=5)
        pr.disable()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(30)
