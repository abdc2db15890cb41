"""Data helpers the hot path needs from the reference's preprocessing module.

Only `get_item_features` lives here: the reference imports it at
src/als_model.py:17 and calls it at :48, but src/data_preprocessing.py never
defines it. Its contract is inferred from its uses
(src/als_model.py:84, 95, 100): dict[itemId] -> {'features': 1-D float vector,
'rating': float}. The feature definition below is this build's choice and is
"parity unpinned" (no reference output exists for it). The ETL pipeline of the
reference (download, imputation, label encoding, split) is out of scope.
"""
import numpy as np
import pandas as pd

CONTENT_COLUMNS = ("price", "manufacturer_id", "category_id")


def get_item_features(data):
    """Per item, in order of first appearance: min-max scaled content columns
    (those of CONTENT_COLUMNS present in `data`; a constant column scales to 0)
    as float64 features, and the item's mean `average_review_rating`."""
    if data is None or len(data) == 0:
        return {}
    df = pd.DataFrame(data)
    cols = [c for c in CONTENT_COLUMNS if c in df.columns]
    g = df.groupby("itemId", sort=False)
    ratings = g["average_review_rating"].mean() if "average_review_rating" in df.columns else None
    if cols:
        first = g[cols].first().astype(np.float64)
        mat = first.to_numpy()
        lo = np.nanmin(mat, axis=0)
        rng = np.nanmax(mat, axis=0) - lo
        rng = np.where(rng < 10 * np.finfo(np.float64).eps, 1.0, rng)
        mat = (mat - lo) / rng
        ids = first.index
    else:
        ids = g.size().index
        mat = np.zeros((len(ids), 1))
    out = {}
    for n, item in enumerate(ids):
        rating = float(ratings.loc[item]) if ratings is not None else 0.0
        out[item.item() if hasattr(item, "item") else item] = {"features": mat[n].copy(), "rating": rating}
    return out
