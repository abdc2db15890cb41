"""GPU parity of the ALS path at ranks 65..256 (csrc/als_wide.hip: one
workgroup per destination row, register-resident Gramian tiles, blocked
LDL^T) against the C oracle (Spark 3.5.1 ALS restated: f64 dspr Gramian,
dpptrf/dpptrs), plus scoring and init at those widths.

Tolerances (north_star "float scores within 1e-4 rtol"): one half-sweep
rtol 1e-5 / atol 1e-6 (f64 accumulation in a different order, result cast
to f32), fits over several epochs rtol 1e-4; init factors and JVM-exact ALS
scores bit-exact.
"""
import numpy as np
import pytest
import torch
from test_gpu_core import _csr_to_dev, _problem

from oracle import als as oals
from oracle import build as obuild
from oracle import synth as osyn

pytestmark = pytest.mark.gpu


def _h():
    from src import _hrec

    return _hrec


@pytest.mark.parametrize("k,kp", [(65, 96), (96, 96), (100, 128), (128, 128), (150, 192), (192, 192),
                                  (200, 256), (256, 256)])
def test_wide_half_sweep_matches_oracle(device, k, kp):
    h = _h()
    indptr, indices, values, src = _problem(k, 40, 300, k, 90, kp)
    d_ip, d_ix, d_v = _csr_to_dev(indptr, indices, values, device)
    dst = torch.full((40, kp), 3.0, device=device)
    h.als_half_sweep(d_ip, d_ix, d_v, torch.as_tensor(src, device=device), k, 0.1, dst)
    got = dst.cpu().numpy()
    exp = obuild.half_sweep(indptr, indices, values, src[:, :k], k, 0.1)
    np.testing.assert_allclose(got[:, :k], exp, rtol=1e-5, atol=1e-6)
    assert (got[:, k:] == 0).all(), "padding columns must stay zero"
    assert (got[0] == 0).all(), "a row without ratings has no factor"


@pytest.mark.parametrize("kp", [96, 256])
def test_wide_half_sweep_window_boundaries(device, kp):
    """Row lengths around the window size (16 ratings at kp >= 192, 32 below),
    steps of 4, more ratings than rank and fewer (rank-deficient Gramian: the
    lambda * n diagonal keeps it definite), first/last source rows."""
    h = _h()
    k, n_src = kp, 301
    deg = np.array([0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 256, 257, 700])
    rng = np.random.default_rng(3)
    indptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    indices = rng.integers(0, n_src, indptr[-1]).astype(np.int32)
    indices[::7] = n_src - 1
    indices[3::11] = 0
    values = rng.integers(0, 19, indptr[-1]).astype(np.float32)
    src = rng.normal(size=(n_src, kp)).astype(np.float32)
    d_ip, d_ix, d_v = _csr_to_dev(indptr, indices, values, device)
    dst = torch.full((len(deg), kp), 3.0, device=device)
    h.als_half_sweep(d_ip, d_ix, d_v, torch.as_tensor(src, device=device), k, 0.1, dst)
    exp = obuild.half_sweep(indptr, indices, values, src, k, 0.1)
    np.testing.assert_allclose(dst.cpu().numpy(), exp, rtol=1e-5, atol=1e-6)


def test_wide_spark_literal_small(device):
    """Against the literal Spark restatement (scipy dppsv on the packed layout)."""
    h = _h()
    indptr, indices, values, src = _problem(9, 6, 30, 70, 40, 96)
    d_ip, d_ix, d_v = _csr_to_dev(indptr, indices, values, device)
    dst = torch.zeros((6, 96), device=device)
    h.als_half_sweep(d_ip, d_ix, d_v, torch.as_tensor(src, device=device), 70, 0.5, dst)
    exp = oals.half_sweep_spark(indptr, indices, values, src[:, :70], 70, 0.5)
    np.testing.assert_allclose(dst.cpu().numpy()[:, :70], exp, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("k", [100, 256])
def test_wide_engine_fit_matches_oracle(device, k):
    from src import synthetic
    from src.als_engine import DeviceALS

    n_users, n_items, dens = 300, 200, 0.3
    csr = synthetic.generate(n_users, n_items, dens, False)
    csc = synthetic.generate(n_users, n_items, dens, True)
    eng = DeviceALS(n_users, n_items, k, 0.1, csr, csc)
    eng.init_user_factors(synthetic.SEED_INIT)
    U0 = eng.user_factors.cpu().numpy().copy()
    np.testing.assert_array_equal(U0, osyn.init_factors(synthetic.SEED_INIT, 0, n_users, k))
    eng.fit(3)
    ucsr = obuild.synth_csr(n_users, n_items, dens, 0, 0, n_users, synthetic.SEED, synthetic.SEED2)
    icsc = obuild.synth_csr(n_users, n_items, dens, 1, 0, n_items, synthetic.SEED, synthetic.SEED2)
    U, V = oals.fit(ucsr, icsc, U0, k, 0.1, 3, sweep=obuild.half_sweep)
    np.testing.assert_allclose(eng.user_factors.cpu().numpy(), U, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(eng.item_factors.cpu().numpy(), V, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("k,kp", [(100, 128), (256, 256)])
def test_wide_init_and_score_bit_exact(device, k, kp):
    h = _h()
    out = torch.full((21, kp), 7.0, device=device)
    h.als_init_factors(5, 40, 21, k, kp, out)
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got[:, :k], osyn.init_factors(5, 40, 21, k))
    assert (got[:, k:] == 0).all()
    rng = np.random.default_rng(2)
    U = np.zeros((9, kp), np.float32)
    U[:, :k] = rng.normal(size=(9, k))
    V = np.zeros((3000, kp), np.float32)
    V[:, :k] = rng.normal(size=(3000, k))
    Vt = h.transpose(torch.as_tensor(V, device=device))
    rows = torch.arange(9, dtype=torch.int64, device=device)
    s = h.als_score(torch.as_tensor(U, device=device), rows, Vt, None, 3000, k).cpu().numpy()
    np.testing.assert_array_equal(s, oals.score_matrix(U[:, :k], V[:, :k]))
    i, v = h.als_score_topk(torch.as_tensor(U, device=device), rows, Vt, 3000, k, 5)
    order = np.argsort(-s.astype(np.float64), axis=1, kind="stable")[:, :5]
    np.testing.assert_array_equal(i.cpu().numpy(), order)
