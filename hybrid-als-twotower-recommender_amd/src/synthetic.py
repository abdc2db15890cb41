"""Synthetic interaction matrices generated on the device (K10).

Replaces the Amazon CSV the reference downloads (src/data_preprocessing.py:22-35)
for the perf configurations of BASELINE.json. The matrix is defined by a
counter-based hash predicate:

    (u, i) in R  <=>  h64(seed, u, i) < threshold(density)
    rating(u, i)  =   h64(seed2, u, i) mod 19      (label-encoded 0..18,
                                                     src/data_preprocessing.py:79-80)

so CSR rows (users) and CSC columns (items) are generated independently and
every shard of every world size sees the same matrix.
"""
from dataclasses import dataclass

import torch

from . import _hrec

SEED = 20250620
SEED2 = 20250621
SEED_INIT = 7
N_LEVELS = 19


def threshold(density):
    """uint64 acceptance threshold: int(density * 2**64) (double product)."""
    if not 0.0 <= density < 1.0:
        raise ValueError("density must be in [0, 1)")
    return int(float(density) * 18446744073709551616.0)


@dataclass
class DeviceCSR:
    """One shard of a compressed-row matrix on the device.

    Rows are global rows row_begin .. row_begin + n_rows - 1; indptr is local
    (starts at 0). For the item side (CSC of R) rows are items and column
    indices are user ids."""
    indptr: torch.Tensor   # int64 [n_rows + 1]
    indices: torch.Tensor  # int32 [nnz]
    values: torch.Tensor   # f32   [nnz]
    row_begin: int
    n_rows: int
    n_cols: int
    col_layout: object = None  # RowLayout the column ids were remapped to (None: global ids)

    @property
    def nnz(self):
        return int(self.indices.numel())


def generate_parts(n_users, n_items, density, transposed, parts, seed=SEED, seed2=SEED2, n_levels=N_LEVELS,
                   device=None):
    """One CSR over several row ranges of R (transposed=False: user rows over
    items) or R^T (item rows over users), concatenated in order: parts =
    [(row_begin, n_rows, n_real)], each range's rows past its first n_real
    (or past the matrix) empty. The index / value arrays are allocated once
    and every range is filled in place (no concatenation: a c3 shard is
    ~100 GB per side, so a copy would not fit beside it)."""
    _hrec.require_device()
    device = device or torch.device("cuda", torch.cuda.current_device())
    total_rows = n_items if transposed else n_users
    n_cols = n_users if transposed else n_items
    thr = threshold(density)
    spans, off = [], 0
    for b, n, real in parts:
        real = max(0, min(int(n), total_rows - int(b), int(real)))
        spans.append((int(b), off, real))
        off += int(n)
    counts = torch.zeros(off, dtype=torch.int64, device=device)
    for b, o, real in spans:
        if real > 0:
            _hrec.synth_row_counts(seed, thr, b, real, n_cols, transposed, counts[o: o + real])
    indptr = _hrec.exclusive_scan(counts)
    del counts
    nnz = int(indptr[-1].item())
    indices = torch.empty(max(nnz, 1), dtype=torch.int32, device=device)[:nnz]
    values = torch.empty(max(nnz, 1), dtype=torch.float32, device=device)[:nnz]
    if nnz > 0:
        for b, o, real in spans:
            if real > 0:  # indptr entries are absolute positions in indices / values
                _hrec.synth_fill(seed, seed2, thr, b, real, n_cols, transposed, n_levels, indptr[o:],
                                 indices, values)
    return DeviceCSR(indptr, indices, values, parts[0][0] if parts else 0, off, n_cols)


def generate(n_users, n_items, density, transposed, row_begin=0, n_rows=None, seed=SEED,
             seed2=SEED2, n_levels=N_LEVELS, device=None, n_real=None):
    """Generate rows [row_begin, row_begin+n_rows) of R (transposed=False:
    user rows over items) or of R^T (transposed=True: item rows over users).
    Rows past the end of the matrix, or past the first n_real rows, are empty
    (shard padding)."""
    total_rows = n_items if transposed else n_users
    if n_rows is None:
        n_rows = total_rows - row_begin
    real = n_rows if n_real is None else min(n_rows, int(n_real))
    return generate_parts(n_users, n_items, density, transposed, [(row_begin, n_rows, real)], seed=seed,
                          seed2=seed2, n_levels=n_levels, device=device)


def generate_ranges(n_users, n_items, density, transposed, ranges, **kw):
    """One CSR over several row ranges [(row_begin, n_rows), ...] of R or R^T,
    concatenated in order (a chunk-interleaved shard, als_engine.shard_chunks)."""
    return generate_parts(n_users, n_items, density, transposed, [(b, n, n) for b, n in ranges], **kw)


def generate_layout(n_users, n_items, density, transposed, layout, rank, **kw):
    """This rank's shard under an als_engine.RowLayout: its parts (chunk
    order), each part's rows followed by empty rows up to the layout's cs,
    with GLOBAL column ids (DeviceALS remaps them)."""
    return generate_parts(n_users, n_items, density, transposed,
                          [(b, layout.cs, cnt) for b, cnt in layout.part_rows(rank)], **kw)


def row_counts(n_users, n_items, density, transposed, seed=SEED, device=None):
    """Ratings per row of R (or R^T) for every row: the input of
    als_engine.RowLayout.balanced."""
    _hrec.require_device()
    device = device or torch.device("cuda", torch.cuda.current_device())
    n_rows = n_items if transposed else n_users
    counts = torch.zeros(n_rows, dtype=torch.int64, device=device)
    if n_rows:
        _hrec.synth_row_counts(seed, threshold(density), 0, n_rows, n_users if transposed else n_items, transposed,
                               counts)
    return counts
