"""Oracle restatement of the Keras two-tower model (numpy) — test
infrastructure only (see oracle/__init__.py).

Reference: src/two_tower_model.py:38-89 (graph), :91-121 (fit), :123-146
(feature assembly), Keras/TF 2.8 semantics [ext, requirements.txt:2]:
Embedding lookup; Dense = x @ W + b; LayerNormalization(axis=-1,
epsilon=1e-3, biased variance, gamma=1/beta=0 init); Dot(axes=1);
loss MSE; Adam(lr, beta1=0.9, beta2=0.999, epsilon=1e-7) with TF's
lr_t = lr*sqrt(1-b2^t)/(1-b1^t) and dense decay of the embedding slots.
"""
import numpy as np

LN_EPS = 1e-3


def scaler_fit(X):
    """MinMaxScaler.fit on float64 columns: (scale_, min_, data_min, data_max)."""
    X = np.asarray(X, dtype=np.float64)
    dmin = np.nanmin(X, axis=0)
    dmax = np.nanmax(X, axis=0)
    rng = dmax - dmin
    rng = np.where(rng < 10 * np.finfo(np.float64).eps, 1.0, rng)
    scale = 1.0 / rng
    min_ = 0.0 - dmin * scale
    return scale, min_, dmin, dmax


def scaler_transform(X, scale, min_):
    X = np.asarray(X, dtype=np.float64).copy()
    X *= scale
    X += min_
    return X
