"""Device ingest: DataFrame columns -> id codes -> CSR/CSC.

Oracle: numpy's own definitions of the two steps the reference delegates to
Spark (src/als_model.py:51-62) — numpy.unique(return_inverse=True) for the id
encoding and a stable argsort by row for the CSR (Spark keeps duplicate
(user, item) ratings as separate terms). Bit-exact: integer/index work.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hrec():
    from src import _hrec

    return _hrec


def _np_csr(rows, cols, vals, n_rows):
    order = np.argsort(rows, kind="stable")
    indptr = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=n_rows))]).astype(np.int64)
    return indptr, cols[order], vals[order]


@pytest.mark.parametrize("n,lo,hi", [(1, 5, 6), (17, -3, 4), (1000, 0, 50), (100000, -(2 ** 31), 2 ** 31),
                                     (65537, 10 ** 12, 10 ** 12 + 7), (200000, 0, 150000), (4096, 0, 4096),
                                     (3000, -5000, -1000)])
def test_encode_ids_matches_numpy_unique(device, n, lo, hi):
    """Both encode paths: dense id spans (span <= n: presence table + scan)
    and the radix-sort ones (32-bit narrow, 64-bit)."""
    h = _hrec()
    rng = np.random.default_rng(n)
    ids = rng.integers(lo, hi, n, dtype=np.int64)
    d_ids = torch.as_tensor(ids, device=device)
    exp_u, exp_c = np.unique(ids, return_inverse=True)
    assert h.minmax_i64(d_ids) == (int(ids.min()), int(ids.max()))
    # measured range (narrow 32-bit path when it fits), a loose hint, and the
    # unknown-range 64-bit path
    for rng in (None, (int(ids.min()) - 3, int(ids.max()) + 5), (-(2 ** 63), 2 ** 63 - 1)):
        uniq, codes = h.encode_ids(d_ids, rng)
        np.testing.assert_array_equal(uniq.cpu().numpy(), exp_u)
        np.testing.assert_array_equal(codes.cpu().numpy(), exp_c.astype(np.int32))


def test_encode_ids_dense_path_unaligned_views(device):
    """The dense path's 16-B id loads: a view starting one element in (8-B
    aligned only) and an odd length take the scalar loads."""
    h = _hrec()
    rng = np.random.default_rng(5)
    ids = rng.integers(0, 3000, 20001, dtype=np.int64)
    d_ids = torch.as_tensor(ids, device=device)[1:]
    exp_u, exp_c = np.unique(ids[1:], return_inverse=True)
    uniq, codes = h.encode_ids(d_ids, (0, 2999))
    np.testing.assert_array_equal(uniq.cpu().numpy(), exp_u)
    np.testing.assert_array_equal(codes.cpu().numpy(), exp_c.astype(np.int32))


@pytest.mark.parametrize("n,lo,hi", [(2, 0, 1), (3, 0, 2), (1000, 0, 50), (200001, 0, 150000), (600_000, 0, 550_000),
                                     (5000, 0, 10 ** 6), (65537, 10 ** 12, 10 ** 12 + 7),
                                     (100000, -(2 ** 31), 2 ** 31)])
def test_encode_ids_order_flag(device, n, lo, hi):
    """encode_ids(order=True): the ids' order read by the marking pass (dense
    bitmap, dense table) or a descent pass (sorting paths) equals numpy's
    all(ids[:-1] <= ids[1:]) — sorted ids, one descent at every lane / wave /
    block boundary position of the pairs, unsorted — with the same codes; for
    ids in order the row pointer written by the code pass equals the stable
    argsort CSR's indptr, and coo_to_csr(indptr=...) hands it back."""
    h = _hrec()
    rng = np.random.default_rng(n + 1)
    base = np.sort(rng.integers(lo, hi, n, dtype=np.int64))
    cases = [base, rng.permutation(base)]
    for pos in (0, 1, 2, 126, 127, 128, 511, 512, 2 * 256 * 4 - 1, n // 2, n - 2):
        if 0 <= pos < n - 1 and base[pos] != base[pos + 1]:
            x = base.copy()
            x[pos], x[pos + 1] = x[pos + 1], x[pos]
            cases.append(x)
    for ids in cases:
        d_ids = torch.as_tensor(ids, device=device)
        exp_u, exp_c = np.unique(ids, return_inverse=True)
        for r in ((lo, hi), None):
            uniq, codes, in_order, starts = h.encode_ids(d_ids, r, order=True)
            assert in_order == bool(np.all(ids[:-1] <= ids[1:]))
            np.testing.assert_array_equal(uniq.cpu().numpy(), exp_u)
            np.testing.assert_array_equal(codes.cpu().numpy(), exp_c.astype(np.int32))
            assert (starts is not None) == in_order
            if in_order:
                exp_ptr = np.concatenate([[0], np.cumsum(np.bincount(exp_c, minlength=len(exp_u)))])
                np.testing.assert_array_equal(starts.cpu().numpy(), exp_ptr)
                vals = torch.arange(n, dtype=torch.float32, device=device)
                ip, ix, iv = h.coo_to_csr(codes, codes, vals, len(exp_u), alias=True, rows_in_order=True,
                                          indptr=starts)
                assert ip is starts and ix is codes and iv is vals
                ip, _, _ = h.coo_to_csr(codes, codes, vals, len(exp_u) + 3, alias=True, rows_in_order=True,
                                        indptr=starts)  # rows past the last code: empty
                np.testing.assert_array_equal(ip.cpu().numpy(), np.concatenate([exp_ptr, [n, n, n]]))


def test_encode_ids_empty(device):
    h = _hrec()
    uniq, codes = h.encode_ids(torch.zeros(0, dtype=torch.int64, device=device))
    assert uniq.numel() == 0 and codes.numel() == 0


@pytest.mark.parametrize("presorted", [False, True])
@pytest.mark.parametrize("nnz,n_rows,n_cols", [(1, 1, 1), (50, 7, 9), (10000, 3, 500), (200000, 4097, 1000),
                                               (300000, 70000, 50), (1_000_000, 1024, 10), (500_000, 1025, 7),
                                               (3_000_000, 1_500_000, 100)])
def test_coo_to_csr_matches_stable_argsort(device, nnz, n_rows, n_cols, presorted):
    """Both paths: the hand-written stable LSD radix sort (1 pass at <= 10
    bits of row code, 2 at 11-20, 3 at 21; (col, rating) ride as 64-bit
    values between passes), and rows already in order (e.g. ratings grouped
    by user), taken without a sort; rating bit patterns (-0.0, NaN payloads)
    pass unchanged."""
    h = _hrec()
    rng = np.random.default_rng(nnz + n_rows)
    rows = rng.integers(0, n_rows, nnz).astype(np.int32)
    rows[: min(nnz, 5)] = n_rows - 1          # the last row is populated
    if presorted:
        rows = np.sort(rows)
    cols = rng.integers(0, n_cols, nnz).astype(np.int32)
    vals = rng.integers(0, 19, nnz).astype(np.float32)
    vals[::3] += 0.25
    vals[1::7] = -0.0
    vals.view(np.uint32)[2::11] = 0x7fc01234  # a NaN with a payload
    ip, ix, v = h.coo_to_csr(torch.as_tensor(rows, device=device), torch.as_tensor(cols, device=device),
                             torch.as_tensor(vals, device=device), n_rows)
    e_ip, e_ix, e_v = _np_csr(rows, cols, vals, n_rows)
    np.testing.assert_array_equal(ip.cpu().numpy(), e_ip)
    np.testing.assert_array_equal(ix.cpu().numpy(), e_ix)
    np.testing.assert_array_equal(v.cpu().numpy().view(np.uint32), e_v.view(np.uint32))
    # alias=True: rows in order hand back the input columns themselves (no
    # copy); otherwise the same sorted arrays as above
    tc, tv = torch.as_tensor(cols, device=device), torch.as_tensor(vals, device=device)
    ip2, ix2, v2 = h.coo_to_csr(torch.as_tensor(rows, device=device), tc, tv, n_rows, alias=True)
    assert torch.equal(ip2, ip) and torch.equal(ix2, ix) and torch.equal(v2.view(torch.int32), v.view(torch.int32))
    in_order = bool(np.all(np.diff(rows) >= 0))
    assert (ix2.data_ptr() == tc.data_ptr() and v2.data_ptr() == tv.data_ptr()) == in_order


def test_coo_to_csr_empty_rows_and_duplicates(device):
    """Leading, interior and trailing empty rows (the sorted path's row
    starts come from an atomicMin per present row + a suffix min); repeated
    (row, col) pairs stay separate entries in input order."""
    h = _hrec()
    rows = np.array([2, 2, 5, 2, 5, 2], np.int32)
    cols = np.array([1, 1, 0, 3, 0, 1], np.int32)
    vals = np.array([1, 2, 3, 4, 5, 6], np.float32)
    ip, ix, v = h.coo_to_csr(*(torch.as_tensor(a, device=device) for a in (rows, cols, vals)), 8)
    np.testing.assert_array_equal(ip.cpu().numpy(), [0, 0, 0, 4, 4, 4, 6, 6, 6])
    np.testing.assert_array_equal(ix.cpu().numpy(), [1, 1, 3, 1, 0, 0])
    np.testing.assert_array_equal(v.cpu().numpy(), [1, 2, 4, 6, 3, 5])


def test_coo_to_csr_no_entries(device):
    h = _hrec()
    z = torch.zeros(0, dtype=torch.int32, device=device)
    ip, ix, v = h.coo_to_csr(z, z, torch.zeros(0, dtype=torch.float32, device=device), 4)
    np.testing.assert_array_equal(ip.cpu().numpy(), [0, 0, 0, 0, 0])


def test_synthetic_csc_from_csr_via_ingest(device):
    """The CSC built from the synthetic CSR's COO equals the generator's own
    CSC (independent construction of the same matrix)."""
    from src import synthetic

    h = _hrec()
    n_u, n_i, dens = 3000, 700, 0.02
    csr = synthetic.generate(n_u, n_i, dens, False)
    csc = synthetic.generate(n_u, n_i, dens, True)
    counts = (csr.indptr[1:] - csr.indptr[:-1]).cpu()
    urow = torch.repeat_interleave(torch.arange(n_u, dtype=torch.int32), counts).to(device)
    ip, ix, v = h.coo_to_csr(csr.indices, urow, csr.values, n_i)
    assert torch.equal(ip, csc.indptr) and torch.equal(ix, csc.indices) and torch.equal(v, csc.values)


@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 1_000_003, 5_000_000])
def test_exclusive_scan_matches_cumsum(device, n):
    """The in-tree reduce-then-scan (csrc/scan.hip: tile sums, one block over
    the sums, tile scans from their offsets) behind the generator's indptr:
    exact int64 prefix sums at tile boundaries and across many tiles."""
    h = _hrec()
    rng = np.random.default_rng(n)
    c = rng.integers(0, 1 << 40, n, dtype=np.int64)
    got = h.exclusive_scan(torch.as_tensor(c, device=device)).cpu().numpy()
    np.testing.assert_array_equal(got, np.concatenate([[0], np.cumsum(c)]))


def test_minmax_extremes(device):
    h = _hrec()
    x = np.array([5, -(2 ** 63), 2 ** 63 - 1, 0], np.int64)
    assert h.minmax_i64(torch.as_tensor(x, device=device)) == (-(2 ** 63), 2 ** 63 - 1)
    y = np.full(3_000_001, 7, np.int64)
    y[2_999_999] = -1
    assert h.minmax_i64(torch.as_tensor(y, device=device)) == (-1, 7)
