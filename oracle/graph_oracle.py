"""torch-CPU fp64 restatement of mfgpflow/graph.py — TEST INFRASTRUCTURE ONLY.

GraphMultiFidelityKernel.K / K_diag (graph.py:39-115) and the GPR log-marginal
likelihood / predict_f of GraphMultiFidelityGPModel (graph.py:118-141, GPflow 2.9
GPR), with gradients by torch autograd (torch's Cholesky adjoint is symmetric like
TF's _CholeskyGrad, and the LF-LF block is differentiated entry by entry, so the
asymmetric rho_LF block gets the reference's gradient).  Adam restated as TF 2.10
Keras legacy Adam with a constant float32 learning rate.

Parity: UNPINNED by reference outputs — the reference ships no test, notebook or
recorded value for the graph model; this restates graph.py line by line.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .svgp_oracle import rbf_t, tf_softplus_t
from .mfgp_oracle import softplus_inverse

JITTER = 1e-6


def graph_K(X, X2, prm, jitter=True):
    """graph.py:39-97. prm: v [m+1], l [m+1, D] (index m = delta), rho [m], rhoLF [m, m]."""
    m = prm["rho"].shape[0]
    f1, f2 = X[:, -1].detach(), X2[:, -1].detach()
    A, B = X[:, :-1], X2[:, :-1]
    K = torch.zeros((X.shape[0], X2.shape[0]), dtype=torch.float64)
    k = [rbf_t(A, B, prm["v"][s], prm["l"][s]) for s in range(m + 1)]
    for i in range(m):
        for j in range(m):
            mask = (f1 == i).double()[:, None] * (f2 == j).double()[None, :]
            coef = 1.0 if i == j else prm["rhoLF"][i, j]
            K = K + mask * coef * k[i]
        lh = (f1 == i).double()[:, None] * (f2 == m).double()[None, :]
        hl = (f1 == m).double()[:, None] * (f2 == i).double()[None, :]
        K = K + (lh + hl) * prm["rho"][i] * k[i]
    hh = (f1 == m).double()[:, None] * (f2 == m).double()[None, :]
    khh = sum(k[i] * prm["rho"][i] ** 2 for i in range(m)) + k[m]
    K = K + hh * khh
    if jitter:
        K = K + JITTER * torch.eye(X.shape[0], dtype=torch.float64)
    return K


def graph_Kdiag(X, prm):
    """graph.py:100-115."""
    m = prm["rho"].shape[0]
    f = X[:, -1]
    out = torch.zeros(X.shape[0], dtype=torch.float64)
    for i in range(m):
        out = out + (f == i).double() * prm["v"][i]
    hf = sum(prm["v"][i] * prm["rho"][i] ** 2 for i in range(m)) + prm["v"][m]
    return out + (f == m).double() * hf


def lml(X, Y, prm, noise):
    K = graph_K(X, X, prm) + noise * torch.eye(X.shape[0], dtype=torch.float64)
    L = torch.linalg.cholesky(K)
    Z = torch.linalg.solve_triangular(L, Y, upper=False)
    N, P = Y.shape
    return -0.5 * (Z * Z).sum() - P * torch.log(torch.diagonal(L)).sum() - 0.5 * N * P * math.log(2 * math.pi)


def predict_f(X, Y, Xs, prm, noise):
    """GPR.predict_f(full_cov=False) with K(X, Xs) free of the jitter (see the product docstring)."""
    K = graph_K(X, X, prm) + noise * torch.eye(X.shape[0], dtype=torch.float64)
    L = torch.linalg.cholesky(K)
    Kmn = graph_K(X, Xs, prm, jitter=False)
    A = torch.linalg.solve_triangular(L, Kmn, upper=False)
    V = torch.linalg.solve_triangular(L, Y, upper=False)
    mean = A.T @ V
    var = graph_Kdiag(Xs, prm) - (A * A).sum(0)
    return mean, var


def predict_f_full_cov(X, Y, Xs, prm, noise):
    """GPR.predict_f(full_cov=True): Knn = K(X*, X*) as the kernel computes it (with its 1e-6
    jitter, graph.py:96), cov = Knn − AᵀA (one block for every output)."""
    K = graph_K(X, X, prm) + noise * torch.eye(X.shape[0], dtype=torch.float64)
    L = torch.linalg.cholesky(K)
    Kmn = graph_K(X, Xs, prm, jitter=False)
    A = torch.linalg.solve_triangular(L, Kmn, upper=False)
    V = torch.linalg.solve_triangular(L, Y, upper=False)
    return A.T @ V, graph_K(Xs, Xs, prm) - A.T @ A


class GraphTrainer:
    """GraphMultiFidelityGPModel.optimize(use_adam=True) (graph.py:154-174): Adam (constant
    float32 lr) on the unconstrained kernel variances / lengthscales / rho (Softplus) and
    rho_LF (Sigmoid); the noise stays fixed.  Loss recorded before each update."""

    def __init__(self, X, Y, m, D, lr=0.01, init=None):
        self.X = torch.tensor(X, dtype=torch.float64)
        self.Y = torch.tensor(Y, dtype=torch.float64)
        P = Y.shape[1]
        u1 = float(softplus_inverse(1.0))
        init = init or {}
        sp_inv = lambda v: torch.tensor(np.asarray(softplus_inverse(np.asarray(v, dtype=np.float64))),
                                        dtype=torch.float64)
        self.vars = {
            "v": (sp_inv(init["v"]) if "v" in init else torch.full((m + 1,), u1, dtype=torch.float64)).clone(),
            "l": (sp_inv(init["l"]) if "l" in init else torch.full((m + 1, D), u1, dtype=torch.float64)).clone(),
            "rho": (sp_inv(init["rho"]) if "rho" in init else torch.full((m, P), u1, dtype=torch.float64)).clone(),
            "rhoLF": torch.tensor(np.log(init.get("rhoLF", 0.5 * np.ones((m, m))))
                                  - np.log1p(-np.asarray(init.get("rhoLF", 0.5 * np.ones((m, m))))),
                                  dtype=torch.float64),
        }
        for v in self.vars.values():
            v.requires_grad_(True)
        self.noise = torch.tensor(float(init.get("noise", 1e-3)), dtype=torch.float64)
        self.lr = float(np.float32(lr))
        self.b1, self.b2, self.eps = float(np.float32(0.9)), float(np.float32(0.999)), 1e-7
        self.m = {k: torch.zeros_like(v) for k, v in self.vars.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.vars.items()}
        self.t = 0

    def params(self):
        V = self.vars
        return dict(v=tf_softplus_t(V["v"]), l=tf_softplus_t(V["l"]), rho=tf_softplus_t(V["rho"])[:, 0],
                    rhoLF=torch.sigmoid(V["rhoLF"]))

    def loss(self):
        return -lml(self.X, self.Y, self.params(), self.noise)

    def step(self):
        loss = self.loss()
        grads = torch.autograd.grad(loss, list(self.vars.values()))
        self.t += 1
        alpha = self.lr * math.sqrt(1.0 - self.b2 ** self.t) / (1.0 - self.b1 ** self.t)
        with torch.no_grad():
            for (k, var), g in zip(self.vars.items(), grads):
                self.m[k] += (g - self.m[k]) * (1.0 - self.b1)
                self.v[k] += (g * g - self.v[k]) * (1.0 - self.b2)
                var -= (self.m[k] * alpha) / (torch.sqrt(self.v[k]) + self.eps)
        return float(loss.detach())
