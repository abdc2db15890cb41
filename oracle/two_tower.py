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


# ----------------------------------------------------------- model math
def _ln(x, gamma, beta):
    mean = x.mean(axis=-1, keepdims=True)
    xc = x - mean
    var = (xc * xc).mean(axis=-1, keepdims=True)
    rstd = 1.0 / np.sqrt(var + LN_EPS)
    xhat = xc * rstd
    return xhat * gamma + beta, xhat, rstd


def forward(p, user, item, man, cat, numeric):
    """float64 forward of the Keras graph; p holds float32 arrays."""
    f = {k: np.asarray(v, dtype=np.float64) for k, v in p.items()}
    x = np.asarray(numeric, dtype=np.float32).astype(np.float64)
    h = np.maximum(x @ f["w1"] + f["b1"], 0.0)
    z = np.concatenate([f["item_emb"][item], f["man_emb"][man], f["cat_emb"][cat], h], axis=1)
    pre = z @ f["w2"] + f["b2"]
    ivec, ixhat, irstd = _ln(pre, f["ln_item_gamma"], f["ln_item_beta"])
    uvec, uxhat, urstd = _ln(f["user_emb"][user], f["ln_user_gamma"], f["ln_user_beta"])
    yhat = (uvec * ivec).sum(axis=1)
    return dict(x=x, h=h, z=z, ivec=ivec, ixhat=ixhat, irstd=irstd, uvec=uvec, uxhat=uxhat, urstd=urstd,
                yhat=yhat)


def backward(p, c, y):
    """MSE (mean over the batch) gradients: dense grads + per-sample
    embedding-row grads (IndexedSlices values)."""
    f = {k: np.asarray(v, dtype=np.float64) for k, v in p.items()}
    B = len(y)
    d = f["b2"].shape[0]
    e = c["yhat"] - np.asarray(y, dtype=np.float64)
    dy = 2.0 * e / B
    dvi = dy[:, None] * c["uvec"]
    dvu = dy[:, None] * c["ivec"]

    def ln_back(dout, xhat, rstd, gamma):
        dxh = dout * gamma
        return rstd * (dxh - dxh.mean(axis=1, keepdims=True) - xhat * (dxh * xhat).mean(axis=1, keepdims=True))

    dp = ln_back(dvi, c["ixhat"], c["irstd"], f["ln_item_gamma"])
    g_user = ln_back(dvu, c["uxhat"], c["urstd"], f["ln_user_gamma"])
    dz = dp @ f["w2"].T
    dpre = dz[:, d + 16:] * (c["h"] > 0)
    grads = {
        "w2": c["z"].T @ dp, "b2": dp.sum(0),
        "ln_item_gamma": (dvi * c["ixhat"]).sum(0), "ln_item_beta": dvi.sum(0),
        "ln_user_gamma": (dvu * c["uxhat"]).sum(0), "ln_user_beta": dvu.sum(0),
        "w1": c["x"].T @ dpre, "b1": dpre.sum(0),
    }
    rows = {"user_emb": g_user, "item_emb": dz[:, :d], "man_emb": dz[:, d:d + 8], "cat_emb": dz[:, d + 8:d + 16]}
    return grads, rows, float((e * e).sum()), float(np.abs(e).sum())


DENSE = ("w2", "b2", "ln_item_gamma", "ln_item_beta", "ln_user_gamma", "ln_user_beta", "w1", "b1")
TABLES = ("user_emb", "item_emb", "man_emb", "cat_emb")


def adam_coefficients(lr, it, b1=0.9, b2=0.999):
    f = np.float32
    t = f(it + 1)
    b1, b2, lr, one = f(b1), f(b2), f(lr), f(1.0)
    b1p = f(np.power(b1, t, dtype=np.float32))
    b2p = f(np.power(b2, t, dtype=np.float32))
    sparse_lr = f(lr * f(np.sqrt(f(one - b2p)) / f(one - b1p)))
    dense_alpha = f(f(lr * np.sqrt(f(one - b2p))) / f(one - b1p))
    return dict(b1=b1, b2=b2, omb1=f(one - b1), omb2=f(one - b2), sparse_lr=sparse_lr, dense_alpha=dense_alpha)


def train_step(p, slots, user, item, man, cat, numeric, y, it, lr=0.001, eps=1e-7):
    """One Keras train_step with TF 2.8 Adam: dense ResourceApplyAdam for the
    Dense/LN variables, Adam._resource_apply_sparse (whole-table slot decay,
    deduplicated slices) for the embedding tables. Updates p/slots in place
    (float32). Returns (sum_sq_err, sum_abs_err)."""
    c = forward(p, user, item, man, cat, numeric)
    grads, rows, sq, ab = backward(p, c, y)
    k = adam_coefficients(lr, it)
    f = np.float32
    eps = f(eps)
    for name in DENSE:
        g = grads[name].astype(np.float32)
        m, v = slots[name]
        m += (g - m) * f(f(1) - k["b1"])
        v += (g * g - v) * f(f(1) - k["b2"])
        p[name] -= (m * k["dense_alpha"]) / (np.sqrt(v) + eps)
    for name, idx in (("user_emb", user), ("item_emb", item), ("man_emb", man), ("cat_emb", cat)):
        g_rows = rows[name].astype(np.float32)
        uniq, first = [], {}
        for s, key in enumerate(idx):
            if key not in first:
                first[key] = len(uniq)
                uniq.append([key, g_rows[s].copy()])
            else:
                uniq[first[key]][1] = uniq[first[key]][1] + g_rows[s]
        m, v = slots[name]
        m *= k["b1"]
        v *= k["b2"]
        for key, g in uniq:
            m[key] = m[key] + g * k["omb1"]
            v[key] = v[key] + (g * g) * k["omb2"]
        p[name] -= (k["sparse_lr"] * m) / (np.sqrt(v) + eps)
    return sq, ab
