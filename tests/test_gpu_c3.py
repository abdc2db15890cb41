"""GPU: BASELINE configs[2] (c3: 10M users x 1M items, 1 % density, rank 64)
at its real row shapes, against the C oracle (oracle/als_oracle.c, Spark
3.5.1's dspr / dppsv restated).

A c3 item row holds ~1e5 ratings over a 10M-row source matrix; a c3 user
row ~1e4 over 1M items. Each test generates a contiguous slice of rows that
holds more than 2^31 ratings (so int64 CSR offsets above 2^31 are exercised
by the synthetic fill and by the half-sweep's gathers), sweeps it on the
device against the full replicated source factors, and checks sampled rows —
including rows whose ratings start past offset 2^31 — against the oracle:
the CSR row bit-exact, the solved factor row at rtol 1e-5 (f64 Gramian
accumulated in another order; atol 1e-6 of the row's largest entry).
Device memory: ~19 GB of CSR + the source factors; host: the source factors
(2.56 GB for the item side) for the oracle."""
import numpy as np
import pytest
import torch

from oracle import build as obuild

pytestmark = pytest.mark.gpu

N_USERS, N_ITEMS, DENS, K, REG = 10_000_000, 1_000_000, 0.01, 64, 0.1
OFF31 = 1 << 31


def _sweep_and_check(device, transposed, n_rows, n_samples):
    from src import _hrec, synthetic

    n_src = N_USERS if transposed else N_ITEMS
    csr = synthetic.generate(N_USERS, N_ITEMS, DENS, transposed, 0, n_rows)
    assert csr.nnz > OFF31, csr.nnz
    src = torch.empty((n_src, K), dtype=torch.float32, device=device)
    _hrec.als_init_factors(synthetic.SEED_INIT + (0 if transposed else 1), 0, n_src, K, K, src)
    dst = torch.empty((n_rows, K), dtype=torch.float32, device=device)
    _hrec.als_half_sweep(csr.indptr, csr.indices, csr.values, src, K, REG, dst)
    torch.cuda.synchronize()
    indptr = csr.indptr.cpu().numpy()
    # samples: spread over the slice, plus the rows straddling and beyond 2^31
    first_hi = int(np.searchsorted(indptr, OFF31, side="right")) - 1
    rows = np.unique(np.concatenate([
        np.linspace(0, n_rows - 1, n_samples // 2).astype(np.int64),
        np.arange(first_hi - 2, first_hi + 2),
        np.linspace(first_hi, n_rows - 1, n_samples - n_samples // 2 - 4).astype(np.int64)]))
    assert indptr[rows].max() > OFF31 and (indptr[rows] > OFF31).sum() >= n_samples // 3
    src_h = src.cpu().numpy()
    dst_h = dst.cpu().numpy()
    degs, ips, ixs, vvs = [], [0], [], []
    for r in rows:
        ip, ix, vv = obuild.synth_csr(N_USERS, N_ITEMS, DENS, int(transposed), int(r), 1, synthetic.SEED,
                                      synthetic.SEED2)
        lo, hi = int(indptr[r]), int(indptr[r + 1])
        assert hi - lo == ip[1], (r, hi - lo, ip[1])
        assert np.array_equal(csr.indices[lo:hi].cpu().numpy(), ix), r
        assert np.array_equal(csr.values[lo:hi].cpu().numpy(), vv), r
        ips.append(ips[-1] + len(ix))
        ixs.append(ix)
        vvs.append(vv)
        degs.append(hi - lo)
    # one oracle call over all sampled rows (OpenMP across rows)
    want = obuild.half_sweep(np.array(ips, np.int64), np.concatenate(ixs), np.concatenate(vvs), src_h, K, REG)
    for j, r in enumerate(rows):
        np.testing.assert_allclose(dst_h[r], want[j], rtol=1e-5, atol=1e-6 * np.abs(want[j]).max(),
                                   err_msg=f"row {r}")
    return csr.nnz, rows, degs


def test_c3_item_rows_over_10m_users(device):
    """c3 item half-sweep: item rows of ~1e5 ratings each, 22k rows = 2.2e9
    ratings (offsets past 2^31), source = 10M user factors."""
    nnz, rows, degs = _sweep_and_check(device, True, 22_000, 64)
    assert min(degs) > 95_000 and len(rows) >= 60


def test_c3_user_rows_over_1m_items(device):
    """c3 user half-sweep: user rows of ~1e4 ratings each, 220k rows =
    2.2e9 ratings (offsets past 2^31), source = 1M item factors."""
    nnz, rows, degs = _sweep_and_check(device, False, 220_000, 256)
    assert min(degs) > 9_000 and len(rows) >= 250
