"""The oracle's analytic LML gradient vs. torch autograd and finite differences."""
import numpy as np
import torch

from oracle import mfgp_oracle as O


def _torch_lml(X, Y, th):
    X = torch.tensor(X)
    Y = torch.tensor(Y)
    vL, lL, vD, lD, rho, noise = th
    f = X[:, -1]
    L1, H1 = (f == 0).double(), (f == 1).double()
    s = L1 + rho * H1

    def rbf(v, l):
        a = X[:, :-1] / l
        r2 = -2 * a @ a.T + ((a * a).sum(1)[:, None] + (a * a).sum(1)[None, :])
        return v * torch.exp(-0.5 * r2)

    K = (s[:, None] * s[None, :]) * rbf(vL, lL) + (H1[:, None] * H1[None, :]) * rbf(vD, lD)
    K = K + noise * torch.eye(len(X), dtype=torch.float64)
    L = torch.linalg.cholesky(K)
    A = torch.linalg.solve_triangular(L, Y, upper=False)
    N, P = Y.shape
    return -0.5 * (A * A).sum() - P * torch.log(torch.diagonal(L)).sum() - 0.5 * N * P * O.LOG2PI


def test_grad_matches_autograd(hbs):
    X, Y = hbs["X"], hbs["Y"]
    rng = np.random.default_rng(0)
    D = X.shape[1] - 1
    p = O.MFParams(1.3, rng.uniform(0.5, 2, D), 0.7, rng.uniform(0.5, 2, D), np.full((Y.shape[1], 1), 0.9), 2e-3)
    lml, g = O.gpr_lml_and_grad(X, Y, p)
    th = [torch.tensor(v, dtype=torch.float64, requires_grad=True)
          for v in (p.vL, p.lL, p.vD, p.lD, p.rho0, p.noise)]
    lt = _torch_lml(X, Y, th)
    lt.backward()
    assert abs(float(lt) - lml) < 1e-9 * abs(lml)
    np.testing.assert_allclose(g["vL"], th[0].grad.item(), rtol=1e-9)
    np.testing.assert_allclose(g["lL"], th[1].grad.numpy(), rtol=1e-8)
    np.testing.assert_allclose(g["vD"], th[2].grad.item(), rtol=1e-9)
    np.testing.assert_allclose(g["lD"], th[3].grad.numpy(), rtol=1e-8)
    np.testing.assert_allclose(g["rho0"], th[4].grad.item(), rtol=1e-9)
    np.testing.assert_allclose(g["noise"], th[5].grad.item(), rtol=1e-9)


def test_grad_finite_difference_forrester():
    from conftest import forrester_test_data
    X, Y = forrester_test_data()
    p = O.MFParams(2.0, np.array([0.3]), 0.5, np.array([0.2]), np.array([[1.7]]), 1e-2)
    lml, g = O.gpr_lml_and_grad(X, Y, p)
    eps = 1e-6
    q = p.copy()
    q.vL += eps
    assert abs((O.gpr_lml(X, Y, q) - lml) / eps - g["vL"]) < 1e-4 * max(1, abs(g["vL"]))
    q = p.copy()
    q.rho = q.rho + eps
    assert abs((O.gpr_lml(X, Y, q) - lml) / eps - g["rho0"]) < 1e-4 * max(1, abs(g["rho0"]))


def test_transforms_roundtrip():
    # TF computes softplus as log(exp(x)+1) (not log1p), so tiny values lose
    # relative precision exactly as in the reference; large values are exact.
    y = np.array([1e-3, 0.5, 1.0, 10.0, 40.0, 1e3])
    np.testing.assert_allclose(O.softplus(O.softplus_inverse(y)), y, rtol=1e-12)
    np.testing.assert_allclose(O.softplus(O.softplus_inverse(1e-9)), 1e-9, rtol=1e-6)
    assert abs(O.softplus_inverse(1.0) - np.log(np.e - 1)) < 1e-15
