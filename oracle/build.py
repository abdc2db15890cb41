"""Build + load the C restatement (oracle/als_oracle.c) — test infrastructure.

Output goes to oracle/_build/ (git-ignored; travels to the GPU box with the
snapshot like libhrec.so). -march=x86-64-v3 keeps the object portable between
this container's Xeon and the GPU box's host CPU.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "als_oracle.c")
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "libals_oracle.so")


def build(force=False):
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    cmd = ["gcc", "-O3", "-march=x86-64-v3", "-fno-fast-math", "-ffp-contract=off", "-fopenmp",
           "-shared", "-fPIC", SRC, "-o", LIB + ".tmp", "-lm"]
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        vp, i64, u64, i32, dbl = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int, ctypes.c_double
        lib.oracle_synth_row.restype = i64
        lib.oracle_synth_row.argtypes = [u64, u64, u64, u64, i64, i32, i32, vp, vp]
        lib.oracle_half_sweep.restype = None
        lib.oracle_half_sweep.argtypes = [vp, vp, vp, i64, vp, i64, i32, dbl, vp, i64]
        lib.oracle_max_threads.restype = i32
        lib.oracle_score_topk.restype = None
        lib.oracle_score_topk.argtypes = [vp, i64, vp, i64, vp, i64, i64, i32, i32, vp, vp]
        _lib = lib
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def synth_csr(n_users, n_items, density, transposed, row_begin, n_rows, seed, seed2, n_levels=19):
    import numpy as np

    from .synth import threshold

    lib = load()
    total = n_items if transposed else n_users
    n_cols = n_users if transposed else n_items
    thr = threshold(density)
    indptr = np.zeros(n_rows + 1, dtype=np.int64)
    cap = max(16, int(n_rows * n_cols * density * 1.5) + 64 * n_rows)
    idx = np.empty(cap, dtype=np.int32)
    val = np.empty(cap, dtype=np.float32)
    pos = 0
    for r in range(n_rows):
        g = row_begin + r
        if g < total:
            if pos + n_cols > cap:
                cap = max(cap * 2, pos + n_cols)
                idx = np.resize(idx, cap)
                val = np.resize(val, cap)
            c = lib.oracle_synth_row(seed, seed2, thr, g, n_cols, int(transposed), n_levels,
                                     ctypes.c_void_p(idx.ctypes.data + 4 * pos),
                                     ctypes.c_void_p(val.ctypes.data + 4 * pos))
            pos += c
        indptr[r + 1] = pos
    return indptr, idx[:pos].copy(), val[:pos].copy()


def half_sweep(indptr, indices, values, src, k, reg):
    import numpy as np

    lib = load()
    src = np.ascontiguousarray(src, dtype=np.float32)
    n_rows = len(indptr) - 1
    out = np.zeros((n_rows, k), dtype=np.float32)
    ip = np.ascontiguousarray(indptr, np.int64)
    ix = np.ascontiguousarray(indices, np.int32)
    vv = np.ascontiguousarray(values, np.float32)
    lib.oracle_half_sweep(_p(ip), _p(ix), _p(vv), n_rows, _p(src), src.shape[1], k, float(reg), _p(out), k)
    return out


def score_topk(U, rows, V, k, top_k):
    """JVM-exact ALS scores of U[rows] against every row of V + stable top-k
    (oracle_score_topk). Returns (idx int64 [n, top_k], val f32 [n, top_k])."""
    import numpy as np

    lib = load()
    U = np.ascontiguousarray(U, dtype=np.float32)
    V = np.ascontiguousarray(V, dtype=np.float32)
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    idx = np.empty((len(rows), top_k), dtype=np.int64)
    val = np.empty((len(rows), top_k), dtype=np.float32)
    lib.oracle_score_topk(_p(U), U.shape[1], _p(rows), len(rows), _p(V), V.shape[1], V.shape[0], int(k),
                          int(top_k), _p(idx), _p(val))
    return idx, val
