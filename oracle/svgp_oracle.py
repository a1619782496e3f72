"""fp64 torch-CPU restatement of the reference's SVGP path — TEST INFRASTRUCTURE ONLY.

Used by tests/ to check the HIP SVGP ELBO (value) and, through torch autograd,
to reproduce the reference's recorded SingleBinSVGP training trace.  Parity:
PINNED by the notebook KAT (demo matter power single bin.ipynb:156-159: −ELBO
after Adam steps 0/10/20/30), see tests/golden/kats.json.

Restates (GPflow 2.9.0, not vendored): SVGP.elbo with whiten=True,
covariances Kuu (+default_jitter 1e-6) / Kuf / Kff for
SharedIndependentInducingVariables over SeparateIndependent and
LinearCoregionalization kernels, conditionals.util.base_conditional_with_lm,
posteriors mix_latent_gp, kullback_leiblers.gauss_kl (K=None),
likelihoods.Gaussian._variational_expectations; TF 2.10 Keras Adam with a
float32 CosineDecay schedule.  Reference call sites: mfgpflow/singlebin_svgp.py:20-97,
mfgpflow/linear_svgp.py:73-203.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .mfgp_oracle import cosine_decay_f32, softplus_inverse

LOG2PI = math.log(2.0 * math.pi)
JITTER = 1e-6
_THR = math.log(np.finfo(np.float64).eps) + 2.0


def tf_softplus_t(x: torch.Tensor) -> torch.Tensor:
    """tf.math.softplus (log(exp(x)+1) with eps thresholds) in torch fp64."""
    ex = torch.exp(torch.clamp(x, max=700.0))
    return torch.where(x > -_THR, x, torch.where(x < _THR, ex, torch.log(ex + 1.0)))


def rbf_t(a, b, var, ls):
    a = a / ls
    b = b / ls
    r2 = -2.0 * (a @ b.T) + ((a * a).sum(-1)[:, None] + (b * b).sum(-1)[None, :])
    return var * torch.exp(-0.5 * r2)


def mf_K_t(X, X2, kp):
    """mfgpflow/linear.py:55-104 (rows with fidelity not exactly 0/1 are zero)."""
    f1, f2 = X[:, -1].detach(), X2[:, -1].detach()
    L1, H1 = (f1 == 0).double(), (f1 == 1).double()
    L2, H2 = (f2 == 0).double(), (f2 == 1).double()
    rho = kp["rho"]
    s1 = L1 + rho * H1
    s2 = L2 + rho * H2
    kL = rbf_t(X[:, :-1], X2[:, :-1], kp["vL"], kp["lL"])
    kD = rbf_t(X[:, :-1], X2[:, :-1], kp["vD"], kp["lD"])
    return (s1[:, None] * s2[None, :]) * kL + (H1[:, None] * H2[None, :]) * kD


def mf_Kdiag_t(X, kp):
    f = X[:, -1].detach()
    rho = kp["rho"]
    return torch.where(f == 0, kp["vL"] * torch.ones_like(f),
                       torch.where(f == 1, kp["vL"] * rho ** 2 + kp["vD"], torch.zeros_like(f)))


def latent_moments(X, Z, kps, q_mu, q_sqrt):
    """Whitened SVGP conditional per latent -> g_mu, g_var [N, L]."""
    gm, gv = [], []
    M = Z.shape[0]
    for l, kp in enumerate(kps):
        Kuu = mf_K_t(Z, Z, kp) + JITTER * torch.eye(M, dtype=torch.float64)
        Kuf = mf_K_t(Z, X, kp)
        Kff = mf_Kdiag_t(X, kp)
        Lm = torch.linalg.cholesky(Kuu)
        A = torch.linalg.solve_triangular(Lm, Kuf, upper=False)
        Lq = torch.tril(q_sqrt[l])
        LTA = Lq.T @ A
        gm.append(A.T @ q_mu[:, l])
        gv.append(Kff - (A * A).sum(0) + (LTA * LTA).sum(0))
    return torch.stack(gm, 1), torch.stack(gv, 1)


def latent_cov(X, Z, kps, q_mu, q_sqrt):
    """GPflow base_conditional_with_lm(full_cov=True, white=True) per latent:
    g_mu [N, L], g_cov [L, N, N] = Knn - A^T A + (Lq^T A)^T (Lq^T A), A = Lm^{-1} Kuf (no jitter on Knn)."""
    gm, gc = [], []
    M = Z.shape[0]
    for l, kp in enumerate(kps):
        Kuu = mf_K_t(Z, Z, kp) + JITTER * torch.eye(M, dtype=torch.float64)
        Kuf = mf_K_t(Z, X, kp)
        Knn = mf_K_t(X, X, kp)
        Lm = torch.linalg.cholesky(Kuu)
        A = torch.linalg.solve_triangular(Lm, Kuf, upper=False)
        LTA = torch.tril(q_sqrt[l]).T @ A
        gm.append(A.T @ q_mu[:, l])
        gc.append(Knn - A.T @ A + LTA.T @ LTA)
    return torch.stack(gm, 1), torch.stack(gc, 0)


def mix_cov(g_cov, g_var, W, full_cov, full_output_cov):
    """GPflow mix_latent_gp covariance branches (W None: independent outputs, P = L):
    full_cov only -> [P, N, N]; full_output_cov only -> [N, P, P]; both -> [N, P, N, P]."""
    L = g_cov.shape[0]
    Wm = torch.eye(L, dtype=torch.float64) if W is None else W
    if full_cov and full_output_cov:
        return torch.einsum("pl,ql,lab->apbq", Wm, Wm, g_cov)
    if full_cov:
        return torch.einsum("pl,lab->pab", Wm * Wm, g_cov)
    return torch.einsum("pl,ql,al->apq", Wm, Wm, g_var)


def elbo_t(X, Y, Z, kps, q_mu, q_sqrt, W, noise, num_data=None):
    """GPflow SVGP.elbo (Gaussian likelihood, whiten=True). W=None -> SeparateIndependent.

    noise must be an fp64 tensor: a torch.tensor(python_float) is fp32 and turns the constant
    -0.5 log(2 pi) - 0.5 log(noise) into an fp32 scalar (1.6e-8 off a term, 1.2e-3 over Goku's N P)."""
    if not (torch.is_tensor(noise) and noise.dtype == torch.float64):
        raise TypeError("elbo_t: noise must be a float64 tensor")
    gm, gv = latent_moments(X, Z, kps, q_mu, q_sqrt)
    if W is not None:
        fm, fv = gm @ W.T, gv @ (W * W).T
    else:
        fm, fv = gm, gv
    ve = (-0.5 * LOG2PI - 0.5 * torch.log(noise) - 0.5 * ((Y - fm) ** 2 + fv) / noise).sum()
    Lq = torch.tril(q_sqrt)
    M, L = q_mu.shape
    kl = 0.5 * ((q_mu ** 2).sum() - M * L + (Lq ** 2).sum()
                - torch.log(torch.diagonal(Lq, dim1=-2, dim2=-1) ** 2).sum())
    scale = (num_data / X.shape[0]) if num_data else 1.0
    return ve * scale - kl, kl, ve


class SingleBinTrainer:
    """SingleBinSVGP (singlebin_svgp.py:20-97) training restated with torch autograd.

    Unconstrained variables: q_mu [M, P]; q_sqrt lower-triangle entries (FillTriangular);
    Z [M, D+1] (fidelity column gets a zero gradient); per-bin kernel_L/kernel_delta
    variance + lengthscales and rho (Softplus); likelihood variance (Shift(1e-6) o Softplus)."""

    def __init__(self, X, Y, Z, lr=0.1, max_iters=2000):
        self.X = torch.tensor(X, dtype=torch.float64)
        self.Y = torch.tensor(Y, dtype=torch.float64)
        M, Dp1 = Z.shape
        D = Dp1 - 1
        P = Y.shape[1]
        self.M, self.P, self.D = M, P, D
        u1 = float(softplus_inverse(1.0))
        self.vars = {
            "q_mu": torch.zeros((M, P), dtype=torch.float64, requires_grad=True),
            "q_sqrt_tri": torch.tensor(np.tile(np.eye(M)[np.tril_indices(M)] * 0.1, (P, 1)), requires_grad=True),
            "Z": torch.tensor(Z, dtype=torch.float64, requires_grad=True),
            "vL": torch.full((P,), u1, dtype=torch.float64, requires_grad=True),
            "lL": torch.full((P, D), u1, dtype=torch.float64, requires_grad=True),
            "vD": torch.full((P,), u1, dtype=torch.float64, requires_grad=True),
            "lD": torch.full((P, D), u1, dtype=torch.float64, requires_grad=True),
            "rho": torch.full((P,), u1, dtype=torch.float64, requires_grad=True),
            "noise": torch.tensor(float(softplus_inverse(1.0 - 1e-6)), dtype=torch.float64, requires_grad=True),
        }
        self.tri = np.tril_indices(M)
        self.sched = cosine_decay_f32(lr, max_iters)
        self.b1, self.b2, self.eps = float(np.float32(0.9)), float(np.float32(0.999)), 1e-7
        self.m = {k: torch.zeros_like(v) for k, v in self.vars.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.vars.items()}
        self.t = 0

    def constrained(self):
        V = self.vars
        q_sqrt = torch.zeros((self.P, self.M, self.M), dtype=torch.float64)
        q_sqrt[:, self.tri[0], self.tri[1]] = V["q_sqrt_tri"]
        kps = [dict(vL=tf_softplus_t(V["vL"][p]), lL=tf_softplus_t(V["lL"][p]), vD=tf_softplus_t(V["vD"][p]),
                    lD=tf_softplus_t(V["lD"][p]), rho=tf_softplus_t(V["rho"][p])) for p in range(self.P)]
        noise = tf_softplus_t(V["noise"]) + 1e-6
        return V["Z"], kps, V["q_mu"], q_sqrt, noise

    def neg_elbo(self):
        Z, kps, q_mu, q_sqrt, noise = self.constrained()
        return -elbo_t(self.X, self.Y, Z, kps, q_mu, q_sqrt, None, noise)[0]

    def step(self):
        loss = self.neg_elbo()
        grads = torch.autograd.grad(loss, list(self.vars.values()))
        lr = self.sched(self.t)
        self.t += 1
        alpha = lr * math.sqrt(1.0 - self.b2 ** self.t) / (1.0 - self.b1 ** self.t)
        with torch.no_grad():
            for (k, var), g in zip(self.vars.items(), grads):
                self.m[k] += (g - self.m[k]) * (1.0 - self.b1)
                self.v[k] += (g * g - self.v[k]) * (1.0 - self.b2)
                var -= (self.m[k] * alpha) / (torch.sqrt(self.v[k]) + self.eps)
        return float(loss.detach())


def initialize_W_ref(output_dim, num_latents, window_fraction=0.3, scale=0.5):
    """mfgpflow/linear_svgp.py:17-48 (structured diagonal W, P x L)."""
    W = np.zeros((output_dim, num_latents))
    window = max(int(output_dim * window_fraction), 2)
    stride = max(output_dim // (num_latents - 1), 1) if num_latents > 1 else 1
    for j in range(num_latents):
        center = min(int(j * stride), output_dim - 1)
        for i in range(output_dim):
            if abs(i - center) < window / 2:
                W[i, j] = np.exp(-0.1 * abs(i - center))
    return W * scale


class LatentTrainer(SingleBinTrainer):
    """LatentMFCoregionalizationSVGP.optimize (linear_svgp.py:153-203) restated with torch
    autograd: W trainable (w_type='diagonal'), q_sqrt = I per latent, noise 1.0,
    num_data = N, loss = -ELBO + (kl_multiplier - 1) KL recorded before each update."""

    def __init__(self, X, Y, kw, lr=0.005, max_iters=10000, kl_multiplier=1.0):
        from sklearn.cluster import KMeans
        Z = KMeans(n_clusters=kw["num_inducing"], random_state=42).fit(X).cluster_centers_
        L, P = kw["num_latents"], kw["num_outputs"]
        super().__init__(X, Y, Z, lr=lr, max_iters=max_iters)
        M, D = Z.shape[0], Z.shape[1] - 1
        u1 = float(softplus_inverse(1.0))
        self.P = L   # per-latent parameter blocks below are sized by L
        self.vars.update({
            "q_mu": torch.zeros((M, L), dtype=torch.float64, requires_grad=True),
            "q_sqrt_tri": torch.tensor(np.tile(np.eye(M)[np.tril_indices(M)], (L, 1)), requires_grad=True),
            "vL": torch.full((L,), u1, dtype=torch.float64, requires_grad=True),
            "lL": torch.full((L, D), u1, dtype=torch.float64, requires_grad=True),
            "vD": torch.full((L,), u1, dtype=torch.float64, requires_grad=True),
            "lD": torch.full((L, D), u1, dtype=torch.float64, requires_grad=True),
            "rho": torch.full((L,), u1, dtype=torch.float64, requires_grad=True),
            "W": torch.tensor(initialize_W_ref(P, L, kw.get("window_fraction", 0.4), kw.get("scale", 0.2)),
                              requires_grad=True),
        })
        self.m = {k: torch.zeros_like(v) for k, v in self.vars.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.vars.items()}
        self.klm = kl_multiplier

    def neg_elbo(self):
        Z, kps, q_mu, q_sqrt, noise = self.constrained()
        e, kl, _ = elbo_t(self.X, self.Y, Z, kps, q_mu, q_sqrt, self.vars["W"], noise, num_data=self.X.shape[0])
        return -e + (self.klm - 1.0) * kl

    def optimize(self, history, max_iters, lr):
        """One LatentMFCoregionalizationSVGP.optimize call (linear_svgp.py:169,194): a FRESH Keras Adam
        (zero moments, iteration counter 0) over CosineDecay(lr, max_iters), stepping
        `for i in range(len(history), max_iters)`; appends the pre-step losses to `history`."""
        self.sched = cosine_decay_f32(lr, max_iters)
        self.m = {k: torch.zeros_like(v) for k, v in self.vars.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.vars.items()}
        self.t = 0
        for _ in range(len(history), max_iters):
            history.append(self.step())
        return history
