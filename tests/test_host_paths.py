"""CPU: host-side shortcuts of the drop-in API, each against the library
call it stands in for (exact equality).

* `_minmax_transform` == `MinMaxScaler.transform` (src/two_tower_model.py:143)
  on the candidate frames predict_for_user sees, and it defers to sklearn for
  everything it does not cover (same result or same exception);
* `_unique` == pandas' `Series.is_unique` on the item-id columns
  `get_hybrid_recommendations`' array path checks.
"""
import numpy as np
import pandas as pd
import pytest
from sklearn.preprocessing import MinMaxScaler

from src.hybrid_system import _unique
from src.two_tower_model import _minmax_transform

COLS = ["price", "average_review_rating"]


def _frame(rng, n, rating_dtype=np.int64, price_dtype=np.float64):
    return pd.DataFrame({"price": (rng.random(n) * 300).astype(price_dtype),
                         "average_review_rating": rng.integers(0, 19, n).astype(rating_dtype)})


@pytest.mark.parametrize("fit_on", ["frame", "array"])
@pytest.mark.parametrize("rating_dtype,price_dtype", [(np.int64, np.float64), (np.float64, np.float64),
                                                      (np.int32, np.float64), (np.float32, np.float32),
                                                      (np.int64, np.float32), (np.int64, np.int64)])
def test_minmax_transform_matches_sklearn(fit_on, rating_dtype, price_dtype):
    rng = np.random.default_rng(3)
    train = _frame(rng, 500)
    sc = MinMaxScaler().fit(train[COLS] if fit_on == "frame" else train[COLS].to_numpy())
    cand = _frame(rng, 2000, rating_dtype, price_dtype)
    cand.loc[5, "price"] = np.nan if price_dtype != np.int64 else cand.loc[5, "price"]
    cand.loc[7, "price"] = cand["price"].max() * 3  # outside the fitted range (no clip)
    got, want = _minmax_transform(sc, cand, COLS), sc.transform(cand[COLS])
    assert got.dtype == want.dtype and got.shape == want.shape
    np.testing.assert_array_equal(got, want)


def test_minmax_transform_defers_to_sklearn():
    rng = np.random.default_rng(4)
    train = _frame(rng, 300)
    cand = _frame(rng, 50)
    clip = MinMaxScaler(clip=True).fit(train[COLS])
    np.testing.assert_array_equal(_minmax_transform(clip, cand, COLS), clip.transform(cand[COLS]))
    sc = MinMaxScaler().fit(train[COLS])
    bad = cand.copy()
    bad.loc[3, "price"] = np.inf
    for frame in (bad, cand.iloc[:0]):  # infinity / zero samples: sklearn's own ValueError
        with pytest.raises(ValueError) as a:
            sc.transform(frame[COLS])
        with pytest.raises(ValueError) as b:
            _minmax_transform(sc, frame, COLS)
        assert str(a.value) == str(b.value)
    with pytest.raises(Exception):  # unfitted
        _minmax_transform(MinMaxScaler(), cand, COLS)


@pytest.mark.parametrize("vals", [np.arange(1000), np.arange(1000)[::-1].copy(), np.array([3, 1, 3]),
                                  np.array([0, 10 ** 12, 5]), np.array([-1, 2, -1]), np.array([], np.int64),
                                  np.arange(50, dtype=np.uint64), np.r_[np.arange(100), 99]])
def test_unique_matches_pandas(vals):
    col = pd.Series(vals)
    assert _unique(vals, col) == col.is_unique
