"""torch-CPU fp64 restatement of the GPR LML (value, value+grad) — the timed CPU baseline.

TEST INFRASTRUCTURE ONLY — used by ``bench.py``'s ``cpu_baseline`` leg and by
``tests/test_oracle_kats.py`` (which checks it against ``mfgp_oracle``, itself pinned
by the reference's notebook KATs).  The product package never imports it.

Same arithmetic as ``oracle/mfgp_oracle.py`` (``gpr_lml`` / ``gpr_lml_and_grad``,
restating ``mfgpflow/linear.py:55-104`` + GPflow 2.9 ``GPR.log_marginal_likelihood``
and the GradientTape of ``linear.py:205-207``), written with whole-matrix torch ops so
that the CPU baseline uses MKL's threaded Cholesky / TRSM / GEMM rather than NumPy's
per-call overheads: this is the faster fp64 CPU restatement SURVEY §6 timed (28.8
value+grad evals/s on 8 Xeon cores at Goku).  The lengthscale gradient uses
Σ_ij M_ij (x_id − x_jd)² = 2 Σ_i r_i x_id² − 2 x_dᵀ M x_d (M symmetric, r = M·1),
so it is O(N²D) instead of D dense N² passes.
"""
from __future__ import annotations

import math

import torch

LOG2PI = math.log(2.0 * math.pi)


def _rbf(Xs: torch.Tensor, var: float, ls: torch.Tensor) -> torch.Tensor:
    """GPflow square_distance (expanded, no clamp) + SquaredExponential.K."""
    a = Xs / ls
    n2 = (a * a).sum(1)
    r2 = -2.0 * (a @ a.T) + (n2[:, None] + n2[None, :])
    return var * torch.exp(-0.5 * r2)


def _blocks(X: torch.Tensor, vL, lL, vD, lD, rho0, unit=False):
    f = X[:, -1]
    isL = (f == 0).to(X.dtype)
    isH = (f == 1).to(X.dtype)
    s = isL + rho0 * isH
    Xc = X[:, :-1]
    eL = _rbf(Xc, 1.0, lL)
    eD = _rbf(Xc, 1.0, lD)
    if unit:   # exp(-r2/2) too: dK/dv in TF's autodiff form
        return s, isH, Xc, vL * eL, vD * eD, eL, eD
    return s, isH, Xc, vL * eL, vD * eD


def lml(X: torch.Tensor, Y: torch.Tensor, vL, lL, vD, lD, rho0, noise) -> float:
    s, h, _, kL, kD = _blocks(X, vL, lL, vD, lD, rho0)
    K = (s[:, None] * s[None, :]) * kL + (h[:, None] * h[None, :]) * kD
    K.diagonal().add_(noise)
    L = torch.linalg.cholesky(K)
    Z = torch.linalg.solve_triangular(L, Y, upper=False)
    N, P = Y.shape
    return float(-0.5 * (Z * Z).sum() - P * torch.log(L.diagonal()).sum() - 0.5 * N * P * LOG2PI)


def lml_and_grad(X: torch.Tensor, Y: torch.Tensor, vL, lL, vD, lD, rho0, noise):
    """(LML, dLML/d[vL, lL(D), vD, lD(D), rho0, noise]) — constrained parameters, fp64."""
    s, h, Xc, kL, kD, eL, eD = _blocks(X, vL, lL, vD, lD, rho0, unit=True)
    SS = s[:, None] * s[None, :]
    HH = h[:, None] * h[None, :]
    K = SS * kL + HH * kD
    K.diagonal().add_(noise)
    L = torch.linalg.cholesky(K)
    Z = torch.linalg.solve_triangular(L, Y, upper=False)
    N, P = Y.shape
    val = float(-0.5 * (Z * Z).sum() - P * torch.log(L.diagonal()).sum() - 0.5 * N * P * LOG2PI)
    alpha = torch.linalg.solve_triangular(L.T, Z, upper=True)
    W = alpha @ alpha.T - P * torch.cholesky_inverse(L)
    ML = W * SS * kL
    MD = W * HH * kD
    SH = h[:, None] * s[None, :] + s[:, None] * h[None, :]

    def ls_grad(M):
        r = M.sum(1)
        return 2.0 * (r @ (Xc * Xc)) - 2.0 * ((M @ Xc) * Xc).sum(0)

    g = torch.cat([
        (0.5 * (W * SS * eL).sum()).reshape(1),
        0.5 * ls_grad(ML) / lL ** 3,
        (0.5 * (W * HH * eD).sum()).reshape(1),
        0.5 * ls_grad(MD) / lD ** 3,
        (0.5 * (W * SH * kL).sum()).reshape(1),
        (0.5 * W.diagonal().sum()).reshape(1),
    ])
    return val, g


def initial_args(d: int, dtype=torch.float64):
    """The notebook's initial theta: variances/lengthscales/rho 1, noise 1e-3."""
    one = torch.ones(d, dtype=dtype)
    return 1.0, one, 1.0, one.clone(), 1.0, 1e-3
