"""CPU baselines for bench.py's secondary lines — TEST INFRASTRUCTURE ONLY
(bench.py's cpu_baseline leg; see oracle/__init__.py). Never imported by the
shipped package.

PySpark and TensorFlow are not installed here or on the GPU box (SURVEY
§8c), so — per BASELINE.md §2 — the CPU baseline of each path is this repo's
own CPU restatement of the same algorithm, run on the GPU box's host cores
in the same process as the GPU measurement, on a BOUNDED sample of the same
workload, scaled to the line's unit:

  * scoring (Spark ALSModel.transform, src/als_model.py:75, + the stable
    sorted()[:k], src/hybrid_system.py:108): oracle_score_topk, the C
    restatement of Spark's JVM f32 dot (no FMA), OpenMP over users;
  * two-tower scoring / hybrid fusion: torch-CPU f32 GEMM (Keras Dot,
    src/two_tower_model.py:80,145) + the fusion of src/hybrid_system.py:57-75
    in f64 + torch.topk;
  * two-tower training: the Keras graph of src/two_tower_model.py:38-89 +
    MSE + TF 2.8 Adam (dense form for Dense/LN, IndexedSlices form with
    whole-table slot decay for the embeddings) in torch-CPU f32, the same
    arithmetic as oracle/two_tower.py (which runs in f64 as the checker);
  * item-vector precompute (c4): the Keras item tower (:38-66) in
    torch-CPU f32 over a slice of the catalogue.
"""
import os
import time

import numpy as np
import torch

from . import build as obuild


def cpu_model():
    """The host CPU's model string (lscpu's "Model name")."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def threads():
    """Threads used: OMP_NUM_THREADS (16 on the GPU box), else the affinity set."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def _setup():
    n = threads()
    torch.set_num_threads(n)
    return n


def _line(value, unit, kind, sample, cores):
    return {"value": value, "unit": unit, "cores": cores, "kind": kind, "sample": sample,
            "cpu_model": cpu_model()}


# --------------------------------------------------------------- scoring
def als_scoring(U_rows, V, k, top_k, n_users_total_batch):
    """JVM-exact ALS scores of the sampled users against every item + stable
    top-k, C oracle (OpenMP). U_rows: [s, >=k] f32 host, V: [n_items, >=k]."""
    cores = obuild.load().oracle_max_threads()
    rows = np.arange(U_rows.shape[0], dtype=np.int64)
    obuild.score_topk(U_rows[:2], rows[:2], V, k, top_k)  # warm
    t0 = time.perf_counter()
    obuild.score_topk(U_rows, rows, V, k, top_k)
    dt = time.perf_counter() - t0
    pairs = U_rows.shape[0] * V.shape[0]
    return _line(pairs / dt, "pairs/s", "port", (
        f"C restatement of Spark's JVM f32 predict (no FMA) + stable top-{top_k} (oracle_score_topk, OpenMP) "
        f"for {U_rows.shape[0]} of the batch's {n_users_total_batch} users x {V.shape[0]} items, "
        f"{dt:.2f} s"), int(cores))


def tt_scoring(n_items_slice, n_items_total, n_users, d, top_k, reps=2, seed=0):
    """Keras Dot over a slice of the catalogue (torch-CPU f32 GEMM) + top-k,
    timed per batch of n_users and scaled to pairs/s."""
    cores = _setup()
    g = torch.Generator().manual_seed(seed)
    V = torch.randn((n_items_slice, d), generator=g) * d ** -0.5
    U = torch.randn((n_users, d), generator=g)
    torch.topk(U[:4] @ V[:4096].T, top_k, dim=1)
    t0 = time.perf_counter()
    for _ in range(reps):
        torch.topk(U @ V.T, top_k, dim=1)
    dt = (time.perf_counter() - t0) / reps
    return _line(n_users * n_items_slice / dt, "pairs/s", "port", (
        f"torch-CPU f32 GEMM (Keras Dot) + torch.topk({top_k}): {n_users} users x {n_items_slice} of the "
        f"{n_items_total} candidates (d = {d}), {reps} batches, {dt:.2f} s each"), cores)


def hybrid(n_users, n_items, k, d, top_k, reps=2, seed=0):
    """get_hybrid_recommendations for a batch of users on the CPU: ALS and
    two-tower scores (torch f32 GEMMs), per-row MinMaxScaler of each model,
    0.2/0.8 weighted fusion in f64, top-k (src/hybrid_system.py:57-75,108)."""
    cores = _setup()
    g = torch.Generator().manual_seed(seed)
    Ua, Va = torch.randn((n_users, k), generator=g), torch.randn((n_items, k), generator=g)
    Ut, Vt = torch.randn((n_users, d), generator=g), torch.randn((n_items, d), generator=g)

    def run():
        a = (Ua @ Va.T).double()
        t = (Ut @ Vt.T).double()

        def mm(x):
            lo, hi = x.min(1, keepdim=True).values, x.max(1, keepdim=True).values
            rng = hi - lo
            rng = torch.where(rng < 10 * np.finfo(np.float64).eps, torch.ones_like(rng), rng)
            return (x - lo) / rng

        f = 0.2 * mm(a) + 0.8 * mm(t)
        return torch.topk(f, top_k, dim=1)

    run()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    return _line(n_users * n_items / dt, "pairs/s", "port", (
        f"torch-CPU: ALS (rank {k}) + two-tower (d = {d}) f32 score GEMMs, per-row min-max in f64, weighted "
        f"fusion, torch.topk({top_k}); {n_users} users x {n_items} items, {reps} batches, {dt * 1e3:.1f} ms each"),
        cores)


# ------------------------------------------------------------ two-tower
def _ln(x, gamma, beta, eps=1e-3):
    mean = x.mean(1, keepdim=True)
    xc = x - mean
    var = (xc * xc).mean(1, keepdim=True)
    rstd = torch.rsqrt(var + eps)
    xh = xc * rstd
    return xh * gamma + beta, xh, rstd


def _ln_back(dout, xh, rstd, gamma):
    dxh = dout * gamma
    return rstd * (dxh - dxh.mean(1, keepdim=True) - xh * (dxh * xh).mean(1, keepdim=True))


def _init(sizes, d, g):
    def uni(*shape, lim=0.05):
        return (torch.rand(shape, generator=g) * 2 - 1) * lim

    p = {"user_emb": uni(sizes[0], d), "item_emb": uni(sizes[1], d), "man_emb": uni(sizes[2], 8),
         "cat_emb": uni(sizes[3], 8), "w1": uni(2, 16, lim=(6 / 18) ** 0.5), "b1": torch.zeros(16),
         "w2": uni(d + 32, d, lim=(6 / (2 * d + 32)) ** 0.5), "b2": torch.zeros(d),
         "gi": torch.ones(d), "bi": torch.zeros(d), "gu": torch.ones(d), "bu": torch.zeros(d)}
    return p


def item_tower(p, item, man, cat, num):
    h = torch.relu(num @ p["w1"] + p["b1"])
    z = torch.cat([p["item_emb"][item], p["man_emb"][man], p["cat_emb"][cat], h], 1)
    pre = z @ p["w2"] + p["b2"]
    iv, xh, rstd = _ln(pre, p["gi"], p["bi"])
    return iv, z, h, xh, rstd


def keras_step(p, slots, it, u, i, m, c, x, y, lr=0.001, b1=0.9, b2=0.999, eps=1e-7):
    """One Keras train_step in torch-CPU f32 (p, slots updated in place)."""
    d = p["b2"].shape[0]
    iv, z, h, ixh, irstd = item_tower(p, i, m, c, x)
    uv, uxh, urstd = _ln(p["user_emb"][u], p["gu"], p["bu"])
    e = (uv * iv).sum(1) - y
    dy = 2.0 * e / len(y)
    dvi, dvu = dy[:, None] * uv, dy[:, None] * iv
    dp = _ln_back(dvi, ixh, irstd, p["gi"])
    gu = _ln_back(dvu, uxh, urstd, p["gu"])
    dz = dp @ p["w2"].T
    dpre = dz[:, d + 16:] * (h > 0)
    dense = {"w2": z.T @ dp, "b2": dp.sum(0), "gi": (dvi * ixh).sum(0), "bi": dvi.sum(0),
             "gu": (dvu * uxh).sum(0), "bu": dvu.sum(0), "w1": x.T @ dpre, "b1": dpre.sum(0)}
    t = it + 1
    lr_t = lr * (1 - b2 ** t) ** 0.5 / (1 - b1 ** t)
    for n, gr in dense.items():
        mm, vv = slots[n]
        mm.add_((gr - mm) * (1 - b1))
        vv.add_((gr * gr - vv) * (1 - b2))
        p[n].sub_(lr_t * mm / (vv.sqrt() + eps))
    for n, idx, gr in (("user_emb", u, gu), ("item_emb", i, dz[:, :d]), ("man_emb", m, dz[:, d:d + 8]),
                       ("cat_emb", c, dz[:, d + 8:d + 16])):
        uq, inv = torch.unique(idx, return_inverse=True)
        gs = torch.zeros((len(uq), gr.shape[1])).index_add_(0, inv, gr)
        mm, vv = slots[n]
        mm.mul_(b1).index_add_(0, uq, gs * (1 - b1))       # whole-table decay (Keras sparse Adam)
        vv.mul_(b2).index_add_(0, uq, gs * gs * (1 - b2))
        p[n].addcdiv_(mm, vv.sqrt().add_(eps), value=-lr_t)
    return float((e * e).sum())


def tt_train(n_users, n_items, n_man, n_cat, d, batch, steps, lr=0.001, seed=0):
    """Keras fit steps (forward + MSE + backward + TF 2.8 Adam) in torch-CPU f32
    on tables of the bench's sizes."""
    cores = _setup()
    g = torch.Generator().manual_seed(seed)
    p = _init((n_users, n_items, n_man, n_cat), d, g)
    slots = {n: (torch.zeros_like(t), torch.zeros_like(t)) for n, t in p.items()}

    def step(it, *b):
        keras_step(p, slots, it, *b, lr=lr)

    def batch_of(j):
        gj = torch.Generator().manual_seed(100 + j)
        return (torch.randint(0, n_users, (batch,), generator=gj), torch.randint(0, n_items, (batch,), generator=gj),
                torch.randint(0, n_man, (batch,), generator=gj), torch.randint(0, n_cat, (batch,), generator=gj),
                torch.rand((batch, 2), generator=gj), torch.randint(0, 19, (batch,), generator=gj).float())

    batches = [batch_of(j) for j in range(steps + 1)]
    step(0, *batches[0])
    t0 = time.perf_counter()
    for j in range(steps):
        step(j + 1, *batches[j + 1])
    dt = (time.perf_counter() - t0) / steps
    return _line(batch / dt, "samples/s", "port", (
        f"torch-CPU f32 restatement of the Keras fit step (graph + MSE + TF 2.8 Adam, whole-table sparse slot "
        f"decay) on the bench's tables ({n_users} users, {n_items} items, {n_man} manufacturers, {n_cat} "
        f"categories, d = {d}), batch {batch}, {steps} steps, {dt * 1e3:.0f} ms each"), cores)


def item_vectors(n_slice, n_total, d, n_man=2651, n_cat=255, chunk=1 << 18, seed=0):
    """The Keras item tower (Dense(16, relu) + concat + Dense(d) + LN) over a
    slice of the catalogue, torch-CPU f32, scaled to items/s."""
    cores = _setup()
    g = torch.Generator().manual_seed(seed)
    p = _init((1, n_slice, n_man, n_cat), d, g)
    item = torch.arange(n_slice)
    man = torch.randint(0, n_man, (n_slice,), generator=g)
    cat = torch.randint(0, n_cat, (n_slice,), generator=g)
    num = torch.rand((n_slice, 2), generator=g)
    item_tower(p, item[:1024], man[:1024], cat[:1024], num[:1024])
    t0 = time.perf_counter()
    for s in range(0, n_slice, chunk):
        e = min(n_slice, s + chunk)
        item_tower(p, item[s:e], man[s:e], cat[s:e], num[s:e])
    dt = time.perf_counter() - t0
    return _line(n_slice / dt, "items/s", "port", (
        f"torch-CPU f32 Keras item tower (Dense(16, relu) + concat + Dense({d}) + LayerNorm) over {n_slice} of the "
        f"{n_total} catalogue items, {dt:.2f} s"), cores)


# ------------------------------------------------------------- API call
def api_call(n_items, k, d, top_k, users=8, seed=0):
    """One get_hybrid_recommendations call per user on the CPU, restated:
    Spark's JVM-exact f32 transform over every candidate (the per-rank
    sequential mul/add of oracle/als.py, vectorised over items), the Keras
    item tower + user tower + Dot (torch-CPU f32) over the same candidates,
    the per-model MinMaxScaler fusion in f64 (src/hybrid_system.py:57-75) and
    the stable sorted()[:top_k] (:108)."""
    from . import als as oals

    cores = _setup()
    g = torch.Generator().manual_seed(seed)
    rng = np.random.default_rng(seed)
    U = rng.normal(size=(users + 1, k)).astype(np.float32)
    V = rng.normal(size=(n_items, k)).astype(np.float32)
    p = _init((users + 1, n_items, 2651, 255), d, g)
    item = torch.arange(n_items)
    man = torch.randint(0, 2651, (n_items,), generator=g)
    cat = torch.randint(0, 255, (n_items,), generator=g)
    num = torch.rand((n_items, 2), generator=g)

    def call(u):
        a = oals.score_matrix(U[u: u + 1], V)[0].astype(np.float64)
        iv = item_tower(p, item, man, cat, num)[0]
        uv = _ln(p["user_emb"][u: u + 1], p["gu"], p["bu"])[0]
        t = (iv @ uv[0]).numpy()

        def mm(x):
            lo, hi = x.min(), x.max()
            r = hi - lo
            r = 1.0 if r < 10 * np.finfo(x.dtype).eps else r
            return (x - lo) / r

        fused = 0.2 * mm(a) + 0.8 * mm(t).astype(np.float64)
        return np.argsort(-fused, kind="stable")[:top_k]

    call(users)
    t0 = time.perf_counter()
    for u in range(users):
        call(u)
    dt = (time.perf_counter() - t0) / users
    return _line(1.0 / dt, "users/s", "port", (
        f"one user per call over {n_items} candidates: JVM-exact f32 ALS transform (rank {k}, numpy, "
        f"oracle/als.py score_matrix) + Keras item/user towers and Dot (d = {d}, torch-CPU f32) + f64 min-max "
        f"fusion + stable top-{top_k}; {users} users, {dt * 1e3:.1f} ms each"), cores)


def cold_call(n_items, dim=3, sample=64, seed=0):
    """The reference's cold-start fallback on the CPU (src/als_model.py:78-86,
    93-104) for a user the model does not know: EVERY candidate
    runs _find_similar_items — a cosine against every other item, the stable
    sorted()[:3], sim > 0.5 — and np.mean of the kept ratings. Restated with
    numpy vectorised over the other items (one normalised-row dot per pair,
    the per-pair arithmetic of oracle/fusion.py cosine); `sample` candidates
    are timed and scaled to the n_items of one call (the reference recomputes
    this per candidate per call)."""
    cores = _setup()
    rng = np.random.default_rng(seed)
    feats = rng.random((n_items, dim))
    ratings = rng.integers(0, 19, n_items).astype(np.float64)
    nrm = np.sqrt((feats * feats).sum(1))
    nrm[nrm == 0] = 1.0
    xn = feats / nrm[:, None]
    gm = float(ratings.mean())

    def one(q):
        sims = xn @ xn[q]
        sims[q] = -np.inf
        top = np.argsort(-sims, kind="stable")[:3]
        keep = [j for j in top if sims[j] > 0.5]
        return np.mean(ratings[keep]) if keep else gm

    one(0)
    qs = rng.choice(n_items, sample, replace=False)
    t0 = time.perf_counter()
    for q in qs:
        one(int(q))
    per_item = (time.perf_counter() - t0) / sample
    per_call = per_item * n_items
    return _line(1.0 / per_call, "users/s", "port", (
        f"cold user over {n_items} candidates: every candidate's fallback (cosine vs every other item, "
        f"stable top-3, sim > 0.5, mean rating; numpy, dim {dim}); {sample} candidates timed "
        f"({per_item * 1e3:.2f} ms each), scaled to one call = {per_call:.1f} s"), cores)
