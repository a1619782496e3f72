"""GPflow-compatible kernels whose arithmetic runs in libmfgp.so.

* ``SquaredExponential`` / ``RBF`` — gpflow.kernels.SquaredExponential (K1, rbf mode).
* ``LinearMultiFidelityKernel`` — mfgpflow/linear.py:12-136 (K1, multi-fidelity mode):
  ``K(X, X2=None, ith_output_dim=0)`` and ``K_diag(X, ith_output_dim=0)``.
* ``LinearCoregionalization`` / ``SeparateIndependent`` — the multi-output
  containers of GPflow used by mfgpflow/linear_svgp.py:122 and
  mfgpflow/singlebin_svgp.py:47.
"""
from __future__ import annotations

import copy

import numpy as np
import torch

from .engine import Engine, resolve_dtype, theta_size, to_dev
from .params import Module, Parameter, as_result, positive, set_trainable


class Kernel(Module):
    """gpflow.kernels.Kernel call protocol: ``kernel(X, X2=None, full_cov=True)``."""

    def __call__(self, X, X2=None, *, full_cov: bool = True, presliced: bool = False):
        if not full_cov:
            if X2 is not None:
                raise ValueError("Ambiguous inputs: `not full_cov` and `X2` are not compatible.")
            return self.K_diag(X)
        return self.K(X, X2)


class SquaredExponential(Kernel):
    """gpflow.kernels.SquaredExponential: k(x, x') = variance * exp(-|x - x'|^2 / (2 l^2))."""

    def __init__(self, variance=1.0, lengthscales=1.0, active_dims=None):
        self.variance = Parameter(variance, transform=positive())
        self.lengthscales = Parameter(lengthscales, transform=positive())
        self.active_dims = active_dims

    @property
    def ard(self) -> bool:
        return self.lengthscales.shape != ()

    def lengthscale_vector(self, d: int) -> np.ndarray:
        ls = self.lengthscales.numpy()
        return np.broadcast_to(ls, (d,)).astype(np.float64) if ls.ndim == 0 else ls.astype(np.float64)

    def _params(self, d, device):
        return torch.tensor(np.concatenate([[float(self.variance.numpy())], self.lengthscale_vector(d)]),
                            dtype=torch.float64, device=device)

    def K(self, X, X2=None):
        eng = Engine.get()
        X1 = to_dev(X, eng.device)
        X2d = X1 if X2 is None else to_dev(X2, eng.device)
        return as_result(eng.rbf_gram(X1, X2d, self._params(X1.shape[1], eng.device)))

    def K_diag(self, X):
        eng = Engine.get()
        n = np.shape(X)[0]
        return as_result(torch.full((n,), float(self.variance.numpy()), dtype=torch.float64, device=eng.device))


RBF = SquaredExponential


class LinearMultiFidelityKernel(Kernel):
    """Kennedy–O'Hagan AR(1) multi-fidelity kernel (mfgpflow/linear.py:12-136).

    f_H(x) = rho f_L(x) + delta(x):  K = [K_LL, rho K_LH; rho K_HL, rho^2 K_HH + K_delta].
    The last input column is the fidelity flag (0.0 = LF, 1.0 = HF; anything else
    gives zero rows, linear.py:67-70).  ``rho`` has shape (num_output_dims, 1) but
    the model-level calls only ever use rho[0] (linear.py:90).
    """

    def __init__(self, kernel_L, kernel_delta, num_output_dims, use_rho=True):
        self.kernel_L = kernel_L
        self.kernel_delta = kernel_delta
        self.rho = Parameter(np.ones((num_output_dims, 1)), transform=positive())
        if not use_rho:
            set_trainable(self.rho, False)

    # -- theta layout of include/mfgp.h: [vL, lL(d), vD, lD(d), rho, noise]
    def theta_vector(self, d: int, ith_output_dim: int = 0, noise: float = 0.0) -> np.ndarray:
        return np.concatenate([
            [float(self.kernel_L.variance.numpy())], self.kernel_L.lengthscale_vector(d),
            [float(self.kernel_delta.variance.numpy())], self.kernel_delta.lengthscale_vector(d),
            [float(self.rho.numpy()[ith_output_dim, 0])], [noise]])

    def theta(self, d: int, device, ith_output_dim: int = 0, noise: float = 0.0) -> torch.Tensor:
        return torch.tensor(self.theta_vector(d, ith_output_dim, noise), dtype=torch.float64, device=device)

    def K(self, X, X2=None, ith_output_dim=0, dtype=None):
        """linear.py:55-104 (fp64, as the reference forces); dtype="float32" selects the fp32 path
        (this engine's addition, include/mfgp.h mfgp_mf_gram_ex)."""
        eng = Engine.get()
        dt = resolve_dtype(dtype)
        X1 = to_dev(X, eng.device, dt)
        X2d = X1 if X2 is None else to_dev(X2, eng.device, dt)
        d = X1.shape[1] - 1
        return as_result(eng.mf_gram(X1, X2d, self.theta(d, eng.device, ith_output_dim)))

    def K_diag(self, X, ith_output_dim=0):
        eng = Engine.get()
        X1 = to_dev(X, eng.device)
        d = X1.shape[1] - 1
        return as_result(eng.mf_kdiag(X1, self.theta(d, eng.device, ith_output_dim)))


class GraphMultiFidelityKernel(Kernel):
    """Graph-structured multi-fidelity kernel (mfgpflow/graph.py:7-115): m LF sources
    (fidelity flags 0..m-1) and HF (flag m), f_H = sum_i rho_i f_Li + delta.

    LF-LF block (i, j) = rho_LF[i, j] k_i (i != j; 1 on the diagonal) — the row source's
    kernel, so K is not symmetric unless rho_LF is; LF-HF = rho_i k_i; HF-HF =
    sum_i rho_i^2 k_i + k_delta; K(X, X2) carries the reference's 1e-6 I jitter
    (graph.py:96), K_diag does not.  Only rho[:, 0] is used (ith_output_dim = 0).
    """

    JITTER = 1e-6

    def __init__(self, kernel_Ls, kernel_delta, num_LF, num_output_dims):
        from .params import Sigmoid
        self.num_LF = int(num_LF)
        self.kernel_Ls = list(kernel_Ls)
        self.kernel_delta = kernel_delta
        self.rho = Parameter(np.ones((self.num_LF, num_output_dims)), transform=positive())
        self.rho_LF = Parameter(0.5 * np.ones((self.num_LF, self.num_LF)), transform=Sigmoid())

    def theta_entries(self, d: int):
        """(Parameter, index) for every theta entry of the include/mfgp.h graph layout (noise excluded)."""
        ents = []
        for k in self.kernel_Ls + [self.kernel_delta]:
            ents.append((k.variance, None))
            ents += [(k.lengthscales, None if k.lengthscales.shape == () else (i,)) for i in range(d)]
        ents += [(self.rho, (i, 0)) for i in range(self.num_LF)]
        ents += [(self.rho_LF, (i, j)) for i in range(self.num_LF) for j in range(self.num_LF)]
        return ents

    def theta_vector(self, d: int, noise: float = 0.0) -> np.ndarray:
        vals = []
        for prm, idx in self.theta_entries(d):
            v = prm.numpy()
            vals.append(float(v if idx is None else v[idx]))
        return np.array(vals + [noise])

    def K(self, X, X2=None, ith_output_dim=0):
        eng = Engine.get()
        X1 = to_dev(X, eng.device)
        X2d = X1 if X2 is None else to_dev(X2, eng.device)
        if X1.shape[0] != X2d.shape[0]:
            # graph.py:96 adds tf.eye(n1) to an [n1, n2] matrix: the reference raises here
            raise ValueError("GraphMultiFidelityKernel.K(X, X2) with len(X) != len(X2): the reference adds "
                             "tf.eye(len(X)) to K and fails the same way")
        d = X1.shape[1] - 1
        th = torch.tensor(self.theta_vector(d), dtype=torch.float64, device=eng.device)
        return as_result(eng.gmf_gram(self.num_LF, X1, X2d, th, diag_add=self.JITTER))

    def K_diag(self, X, ith_output_dim=0):
        eng = Engine.get()
        X1 = to_dev(X, eng.device)
        d = X1.shape[1] - 1
        th = torch.tensor(self.theta_vector(d), dtype=torch.float64, device=eng.device)
        return as_result(eng.gmf_kdiag(self.num_LF, X1, th))


class Combination(Kernel):
    def __init__(self, kernels):
        self.kernels = list(kernels)

    @property
    def num_latent_gps(self) -> int:
        return len(self.kernels)

    def latent_thetas(self, d: int, device) -> torch.Tensor:
        return torch.tensor(np.stack([k.theta_vector(d) for k in self.kernels]), dtype=torch.float64, device=device)


class SeparateIndependent(Combination):
    """gpflow.kernels.SeparateIndependent (singlebin_svgp.py:47)."""

    def K(self, X, X2=None, full_output_cov=False):
        """[L, N, N2] (GPflow SeparateIndependent.K, full_output_cov=False)."""
        if full_output_cov:
            raise NotImplementedError("SeparateIndependent.K(full_output_cov=True) is not used by the reference")
        return as_result(torch.stack([k.K(X, X2).as_subclass(torch.Tensor) for k in self.kernels], dim=0))

    def K_diag(self, X, full_output_cov=False):
        """[N, L] (GPflow SeparateIndependent.K_diag, full_output_cov=False)."""
        if full_output_cov:
            raise NotImplementedError("SeparateIndependent.K_diag(full_output_cov=True) is not used by the reference")
        return as_result(torch.stack([k.K_diag(X).as_subclass(torch.Tensor) for k in self.kernels], dim=1))


class LinearCoregionalization(Combination):
    """gpflow.kernels.LinearCoregionalization (linear_svgp.py:122): f = W g."""

    def __init__(self, kernels, W):
        super().__init__(kernels)
        self.W = W if isinstance(W, Parameter) else Parameter(W)

    @property
    def num_latent_gps(self) -> int:
        return self.W.shape[-1]


def deepcopy_kernel(k):
    """copy.deepcopy of a kernel (linear_svgp.py:121 deep-copies per latent)."""
    return copy.deepcopy(k)
