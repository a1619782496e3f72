"""The reference's own tests (tests/*.py), run against the MI355X engine.

Broken reference assertions are fixed to the code's actual semantics:
rho has shape (P, 1) (test_output_dim.py:46 expected (1, P))."""
import numpy as np
import pytest

import multi_fidelity_gpflow_amd as M
from conftest import forrester_test_data, sin_multi_output_data

pytestmark = pytest.mark.gpu


def test_scipy_contracts():
    """tests/test_scipy.py:27-50."""
    X, Y = sin_multi_output_data(P=1)
    m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(), M.SquaredExponential())
    assert m.kernel.rho.shape[0] == Y.shape[1]
    K = m.kernel.K(X, X).numpy()
    assert np.all(np.linalg.eigvalsh(K) >= -1e-6)
    mean, var = m.predict_f(X)
    assert mean.shape == Y.shape and var.shape == Y.shape
    initial = float(m.training_loss().numpy())
    m.optimize(max_iters=500, use_adam=False, verbose=False)
    assert float(m.training_loss().numpy()) < initial


def test_lf_variance_contracts():
    """tests/test_lf_variance.py:50-74 (Forrester 60 LF / 20 HF, L-BFGS).

    The reference test is broken as written: its second assertion compares arrays of
    60 and 20 entries (a broadcast error), and under the faithful fp64 restatement its
    first assertion fails too — the second L-BFGS pass trains the noise from 1e-3 up to
    ~2.3e-3, which raises the posterior variance at the LF training points (oracle:
    median ratio ~4.5).  What is checked here instead is the behaviour behind them:
    the noise IS trained in the L-BFGS path (unlike Adam, linear.py:233-234), and the
    posterior variances at LF/HF points equal the oracle's at the trained theta."""
    from oracle import mfgp_oracle as O
    rs = np.random.RandomState(42)
    fo = lambda x: ((6 * x - 2) ** 2) * np.sin(12 * x - 4)
    fl = lambda x: 0.5 * fo(x) + 10 * (x[:, [0]] - 0.5) + 5
    X_L = rs.rand(60, 1)
    X_H = rs.permutation(X_L)[:20]
    Y_L = fl(X_L) + 0.05 * rs.randn(60, 1)
    Y_H = fo(X_H) + 0.01 * rs.randn(20, 1)
    X_L = np.hstack([X_L, np.zeros_like(X_L)])
    X_H = np.hstack([X_H, np.ones_like(X_H)])
    X, Y = np.vstack([X_L, X_H]), np.vstack([Y_L, Y_H])
    m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(), M.SquaredExponential())
    m.optimize(max_iters=500, use_adam=False, verbose=False)
    assert float(m.likelihood.variance.numpy()) != pytest.approx(1e-3, rel=1e-3)
    k = m.kernel
    p = O.MFParams(float(k.kernel_L.variance.numpy()), k.kernel_L.lengthscale_vector(1),
                   float(k.kernel_delta.variance.numpy()), k.kernel_delta.lengthscale_vector(1), k.rho.numpy(),
                   float(m.likelihood.variance.numpy()))
    for Xs in (X_L, X_H):
        _, var = m.predict_f(Xs)
        _, vo = O.gpr_predict_f(X, Y, Xs, p)
        np.testing.assert_allclose(var.numpy(), vo, rtol=1e-7, atol=1e-12)


def test_output_dim_contracts():
    """tests/test_output_dim.py:41-65 with P = 3."""
    X, Y = sin_multi_output_data(P=3)
    m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(), M.SquaredExponential())
    assert m.kernel.rho.numpy().shape == (3, 1)
    before = m.kernel.rho.numpy().copy()
    m.optimize(max_iters=500, use_adam=False, verbose=False)
    after = m.kernel.rho.numpy()
    assert not np.allclose(before, after)
    np.testing.assert_array_equal(after[1:], before[1:])   # only rho[0] is ever used (linear.py:90)


def test_forrest_contracts():
    """tests/test_forrest.py:66-77: 1000 Adam iterations (default lr 0.01)."""
    X, Y = forrester_test_data()
    m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(), M.SquaredExponential())
    m.optimize(max_iters=1000, use_adam=True, verbose=False)
    assert m.kernel.rho.shape == (Y.shape[1], 1)
    K = m.kernel.K(X, X).numpy()
    assert np.all(np.linalg.eigvals(K).real >= -1e-8)
    assert m.loss_history[-1] < m.loss_history[0]


def test_ho2021_multibin_contracts(hbs, kats):
    """tests/test_ho2021_multibin.py:20-154: 100 Adam steps (lr 0.1) then predict."""
    from conftest import HBS_DIR
    from multi_fidelity_gpflow_amd.data import PowerSpecs, multifidelity_training_set
    ps = PowerSpecs()
    ps.read_from_txt(HBS_DIR)
    X, Y, Xt, Yt = multifidelity_training_set(ps)
    m = M.MultiFidelityGPModel(X, Y, M.RBF(lengthscales=np.ones(5), variance=1.0),
                               M.RBF(lengthscales=np.ones(5), variance=1.0))
    m.optimize(max_iters=100, use_adam=True, learning_rate=0.1, unfix_noise_after=50, verbose=False)
    assert len(m.loss_history) == 100
    mean, var = m.predict_f(Xt)
    assert mean.shape == (10, 49) and var.shape == (10, 49)
    err = np.abs(10 ** mean.numpy() / 10 ** Yt - 1).mean(axis=0)
    k = kats["hbs_abs_error_curve"]
    assert abs(err[0] - k["first"]) < k["tol"] and abs(err[-1] - k["last"]) < k["tol"]
    assert int(np.argmin(err)) == k["min_bin"] and abs(err.min() - k["min"]) < k["tol"]
