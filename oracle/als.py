"""Oracle restatement of Spark 3.5.1 explicit ALS (numpy + scipy LAPACK).

Test infrastructure only (see oracle/__init__.py).

The reference fits ALS through pyspark (src/als_model.py:52-62, `als.fit`).
Spark's arithmetic lives in org.apache.spark.ml.recommendation.ALS
(pyspark==3.5.1, requirements.txt:1 — not vendored, not installed here).
Restated from its published source [ext]:

  * NormalEquation.add(a, b): copy the f32 factor to f64 `da`;
    blas.dspr("U", k, 1.0, da, 1, ata)  (packed upper, column-major);
    if (b != 0) blas.daxpy(k, b, da, 1, atb, 1)
  * computeFactors: per dst row, add() every rating, numExplicits += 1,
    then solver.solve(ne, numExplicits * regParam)
  * CholeskySolver.solve: ata[diag] += lambda walking i = 0, j = 2,
    i += j, j += 1; lapack.dppsv("U", k, 1, ata, atb) ; x = atb.toFloat
  * ALS.train (explicit): for iter: itemFactors = computeFactors(userFactors)
    then userFactors = computeFactors(itemFactors)

`half_sweep_spark` is the literal restatement (sequential dspr, the same
LAPACK dppsv through scipy). `half_sweep_blas` forms the same Gramian with one
BLAS product per row (summation order differs at the 1e-16 level) for larger
CPU cases.
"""
import numpy as np
from scipy.linalg import lapack


def _packed_upper(A):
    """Column-major packed upper triangle of a symmetric k x k matrix."""
    k = A.shape[0]
    return np.concatenate([A[: j + 1, j] for j in range(k)])


def _add_lambda_diag(ap, k, lam):
    i, j = 0, 2
    tri = k * (k + 1) // 2
    while i < tri:
        ap[i] += lam
        i += j
        j += 1


def solve_row_packed(ap, atb, k, n, reg):
    """CholeskySolver.solve on a packed-upper Gramian (modifies copies)."""
    ap = ap.astype(np.float64).copy()
    _add_lambda_diag(ap, k, n * reg)
    x, info = lapack.dppsv(k, ap, atb.astype(np.float64).reshape(k, 1).copy())
    if info != 0:
        return np.full(k, np.nan, dtype=np.float32)
    return x[:, 0].astype(np.float32)


def half_sweep_spark(indptr, indices, values, src, k, reg):
    """One computeFactors pass, literal form. src: [n_src, >=k] f32."""
    n_rows = len(indptr) - 1
    out = np.zeros((n_rows, k), dtype=np.float32)
    tri = k * (k + 1) // 2
    iu = np.triu_indices(k)
    # column-major packed-upper position of (row i, col j), i <= j
    pos = (iu[1] * (iu[1] + 1)) // 2 + iu[0]
    for r in range(n_rows):
        b, e = int(indptr[r]), int(indptr[r + 1])
        if b == e:
            continue
        ata = np.zeros(tri, dtype=np.float64)
        atb = np.zeros(k, dtype=np.float64)
        for p in range(b, e):
            da = src[indices[p], :k].astype(np.float64)
            outer = np.outer(da, da)
            ata[pos] += outer[iu]
            rating = float(values[p])
            if rating != 0.0:
                atb += rating * da
        out[r] = solve_row_packed(ata, atb, k, e - b, reg)
    return out


def half_sweep_blas(indptr, indices, values, src, k, reg):
    n_rows = len(indptr) - 1
    out = np.zeros((n_rows, k), dtype=np.float32)
    for r in range(n_rows):
        b, e = int(indptr[r]), int(indptr[r + 1])
        if b == e:
            continue
        V = src[indices[b:e], :k].astype(np.float64)
        R = values[b:e].astype(np.float64)
        A = V.T @ V
        atb = V.T @ R
        out[r] = solve_row_packed(_packed_upper(A), atb, k, e - b, reg)
    return out


def fit(user_csr, item_csc, U0, k, reg, max_iter, sweep=half_sweep_blas):
    """Spark ALS.train explicit loop. user_csr / item_csc: (indptr, indices,
    values) over all users / items. Returns (U, V) f32."""
    U = np.asarray(U0, dtype=np.float32)[:, :k].copy()
    V = None
    for _ in range(max_iter):
        V = sweep(*item_csc, U, k, reg)
        U = sweep(*user_csr, V, k, reg)
    return U, V


def predict(U, V, users, items):
    """ALSModel.transform's predict UDF [ext]: f32 sequential dot, no FMA."""
    out = np.zeros(len(users), dtype=np.float32)
    for n, (u, i) in enumerate(zip(users, items)):
        acc = np.float32(0.0)
        for c in range(U.shape[1]):
            acc = np.float32(acc + np.float32(U[u, c] * V[i, c]))
        out[n] = acc
    return out


def score_matrix(U_rows, V):
    """Vectorised predict for a user block x all items, same rounding as
    `predict` (numpy f32 ops round each product and each sum)."""
    U_rows = np.asarray(U_rows, dtype=np.float32)
    V = np.asarray(V, dtype=np.float32)
    acc = np.zeros((U_rows.shape[0], V.shape[0]), dtype=np.float32)
    for c in range(U_rows.shape[1]):
        prod = np.multiply.outer(U_rows[:, c], V[:, c]).astype(np.float32)
        acc = (acc + prod).astype(np.float32)
    return acc
