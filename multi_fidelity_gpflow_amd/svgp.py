"""Sparse variational multi-fidelity emulators (value path on the MI355X engine).

* ``LatentMFCoregionalizationSVGP`` — mfgpflow/linear_svgp.py:64-221: L latent
  LinearMultiFidelityKernels mixed by W (LinearCoregionalization), KMeans
  inducing points, whitened q(u).
* ``SingleBinSVGP`` — mfgpflow/singlebin_svgp.py:13-135: one LinearMultiFidelityKernel
  per output bin (SeparateIndependent), q_sqrt = 0.1 I.

``elbo``, ``prior_kl`` and ``predict_f`` run in libmfgp.so (mfgp_svgp_elbo /
mfgp_svgp_predict: batched K_uu factor, fused K_uf K_uu^{-1} products, mixing,
variational expectations, KL).  The ELBO gradient on the device is the next row of
SURVEY §8(f) (#2); ``optimize`` raises until it lands.
"""
from __future__ import annotations

import copy
import pickle

import numpy as np
import torch

from .engine import Engine, theta_size, to_dev
from .kernels import LinearCoregionalization, LinearMultiFidelityKernel, SeparateIndependent
from .models import CholeskyError, Gaussian
from .params import Module, Parameter, as_result, parameter_dict, multiple_assign

DEFAULT_JITTER = 1e-6


def initialize_W(output_dim, num_latents, window_fraction=0.3, scale=0.5):
    """Structured diagonal W (P x L) — linear_svgp.py:17-48."""
    W = np.zeros((output_dim, num_latents))
    window = max(int(output_dim * window_fraction), 2)
    stride = max(output_dim // (num_latents - 1), 1) if num_latents > 1 else 1
    for j in range(num_latents):
        center = min(int(j * stride), output_dim - 1)
        for i in range(output_dim):
            dist = abs(i - center)
            if dist < window / 2:
                W[i, j] = np.exp(-0.1 * dist)
    return W * scale


def initialize_W_pca(Y, output_dim, num_latents, perturb=0.01, seed=None):
    """PCA-based W — linear_svgp.py:50-62."""
    from sklearn.decomposition import PCA
    pca = PCA(n_components=num_latents)
    pca.fit(Y)
    W = pca.components_.T
    W = W / np.linalg.norm(W, axis=0)
    rng = np.random if seed is None else np.random.RandomState(seed)
    return W + perturb * rng.randn(*W.shape)


def kmeans_inducing(X, num_inducing, random_state=42):
    """KMeans(n_clusters, random_state=42).fit(X).cluster_centers_ (host, one-time init)."""
    from sklearn.cluster import KMeans
    return KMeans(n_clusters=num_inducing, random_state=random_state).fit(X).cluster_centers_


class _SVGPBase(Module):
    """Shared state: kernel (multi-output), Z, q_mu [M, L], q_sqrt [L, M, M], likelihood."""

    def _setup(self, Z, q_mu, q_sqrt, likelihood, num_data):
        self.inducing_variable = Parameter(np.asarray(Z, dtype=np.float64))
        self.q_mu = Parameter(np.asarray(q_mu, dtype=np.float64))
        self.q_sqrt = Parameter(np.asarray(q_sqrt, dtype=np.float64))
        self.likelihood = likelihood
        self.num_data = num_data
        self.loss_history = []

    @property
    def num_latent_gps(self) -> int:
        return self.q_mu.shape[1]

    def _W(self):
        return None

    def _dev_state(self):
        eng = Engine.get()
        D = self.inducing_variable.shape[1] - 1
        Z = to_dev(self.inducing_variable.numpy(), eng.device)
        thetas = self.kernel.latent_thetas(D, eng.device)
        q_mu = to_dev(self.q_mu.numpy(), eng.device)
        q_sqrt = to_dev(np.tril(self.q_sqrt.numpy()), eng.device)
        W = self._W()
        W = None if W is None else to_dev(W, eng.device)
        return eng, Z, thetas, q_mu, q_sqrt, W

    def _elbo_parts(self, data):
        X, Y = data
        eng, Z, thetas, q_mu, q_sqrt, W = self._dev_state()
        Xd, Yd = to_dev(X, eng.device), to_dev(Y, eng.device)
        scale = (self.num_data / Xd.shape[0]) if self.num_data else 1.0
        out, g_mu, g_var, info = eng.svgp_elbo(Xd, Yd, Z, thetas, q_mu, q_sqrt, W,
                                               float(self.likelihood.variance.numpy()), scale, DEFAULT_JITTER)
        if int(info.max().item()) != 0:
            raise CholeskyError("elbo: Cholesky of K_uu was not successful")
        return out

    def elbo(self, data):
        """GPflow SVGP.elbo: sum of variational expectations (x num_data / N) - KL."""
        return as_result(self._elbo_parts(data)[0].clone())

    def training_loss(self, data):
        return as_result(-self.elbo(data))

    def prior_kl(self):
        """gauss_kl(q_mu, q_sqrt) with the whitened N(0, I) prior."""
        L = np.tril(self.q_sqrt.numpy())
        q = self.q_mu.numpy()
        M, Lat = q.shape
        d = np.diagonal(L, axis1=-2, axis2=-1)
        return 0.5 * (np.sum(q * q) - M * Lat + np.sum(L * L) - np.sum(np.log(d * d)))

    def predict_f(self, Xnew, full_cov=False, full_output_cov=False):
        if full_cov or full_output_cov:
            raise NotImplementedError("SVGP predict_f(full_cov=True) is not provided by the MI355X engine yet")
        eng, Z, thetas, q_mu, q_sqrt, W = self._dev_state()
        Xs = to_dev(Xnew, eng.device)
        f_mu, f_var, _, _, info = eng.svgp_predict(Xs, Z, thetas, q_mu, q_sqrt, W, self.num_outputs, DEFAULT_JITTER)
        if int(info.max().item()) != 0:
            raise CholeskyError("predict_f: Cholesky of K_uu was not successful")
        return as_result(f_mu), as_result(f_var)

    def predict_y(self, Xnew, full_cov=False, full_output_cov=False):
        mean, var = self.predict_f(Xnew, full_cov, full_output_cov)
        return mean, as_result(var + float(self.likelihood.variance.numpy()))

    def optimize(self, *args, **kwargs):
        raise NotImplementedError(
            "SVGP training needs the ELBO gradient on the device (SURVEY §8(f) row 2, next round); "
            "elbo / predict_f run on the MI355X engine now")

    def save_model(self, filename):
        """parameter_dict pickled (linear_svgp.py:206-212) — our own file format."""
        with open(filename, "wb") as f:
            pickle.dump(parameter_dict(self), f)


class LatentMFCoregionalizationSVGP(_SVGPBase):
    """mfgpflow/linear_svgp.py:64-151 constructor semantics."""

    def __init__(self, X, Y, kernel_L, kernel_delta, num_latents, num_inducing, num_outputs, use_rho=True,
                 heterosed=False, loss_type='gaussian', w_type='diagonal', window_fraction=0.4, scale=0.2):
        if heterosed:
            raise NotImplementedError("heteroscedastic likelihoods are out of scope (SURVEY §2)")
        self.num_outputs = num_outputs
        self.num_latents = num_latents
        self.loss_type = loss_type
        if w_type == 'pca':
            W = Parameter(initialize_W_pca(np.asarray(Y)[:, :num_outputs], num_outputs, num_latents))
        elif w_type == 'diagonal':
            W = Parameter(initialize_W(num_outputs, num_latents, window_fraction=window_fraction, scale=scale))
        elif w_type == 'fixed_independent':
            W = Parameter(np.eye(num_outputs, num_latents), trainable=False)
        else:
            raise ValueError(f"Unknown w_type: {w_type}. Choose from 'pca', 'diagonal', or 'fixed_independent'.")
        kernels = [LinearMultiFidelityKernel(copy.deepcopy(kernel_L), copy.deepcopy(kernel_delta), num_output_dims=1,
                                             use_rho=use_rho) for _ in range(num_latents)]
        self.kernel = LinearCoregionalization(kernels, W=W)
        Z = kmeans_inducing(np.asarray(X), num_inducing, 42)
        M = Z.shape[0]
        self._setup(Z, np.zeros((M, num_latents)), np.tile(np.eye(M)[None], (num_latents, 1, 1)),
                    Gaussian(variance=1.0), np.asarray(X).shape[0])
        self.kl_history = []

    def _W(self):
        return self.kernel.W.numpy()


class SingleBinSVGP(_SVGPBase):
    """mfgpflow/singlebin_svgp.py:20-62 constructor semantics (Z values are ignored;
    KMeans is recomputed with Z.shape[0] clusters, singlebin_svgp.py:50-51)."""

    def __init__(self, X, Y, kernel_L, kernel_delta, num_outputs, Z, random_state=42):
        self.num_outputs = num_outputs
        kernels = [LinearMultiFidelityKernel(copy.deepcopy(kernel_L), copy.deepcopy(kernel_delta), num_output_dims=1)
                   for _ in range(num_outputs)]
        self.kernel = SeparateIndependent(kernels)
        Zi = kmeans_inducing(np.asarray(X), np.asarray(Z).shape[0], random_state)
        M = Zi.shape[0]
        self._setup(Zi, np.zeros((M, num_outputs)), np.repeat(np.eye(M)[None], num_outputs, axis=0) * 0.1,
                    Gaussian(), None)

    @staticmethod
    def load_model(filename, X, Y, kernel_L, kernel_delta, num_outputs, Z):
        model = SingleBinSVGP(X, Y, kernel_L, kernel_delta, num_outputs, Z)
        with open(filename, "rb") as f:
            multiple_assign(model, pickle.load(f))
        return model
