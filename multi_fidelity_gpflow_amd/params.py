"""GPflow-compatible parameters, transforms and result tensors.

Mirrors the parts of ``gpflow.Parameter`` / ``gpflow.utilities.positive`` /
``set_trainable`` that the reference uses (mfgpflow/linear.py:6,47-52,154,218;
linear_svgp.py:109-115).  Values are kept on the host in float64 (they are a
handful of scalars); the transforms follow TF/TFP exactly so the constrained
values agree bit-for-bit with the device-side transform in k_finalize:

  Softplus forward  = tf.math.softplus     (log(exp(x)+1), eps thresholds)
  Softplus inverse  = tfp.math.softplus_inverse
  positive(lower)   = Shift(lower) ∘ Softplus   (lower=None -> plain Softplus)
"""
from __future__ import annotations

import math

import numpy as np
import torch

_THR = math.log(np.finfo(np.float64).eps) + 2.0


def tf_softplus(x):
    x = np.asarray(x, dtype=np.float64)
    ex = np.exp(np.minimum(x, 700.0))
    return np.where(x > -_THR, x, np.where(x < _THR, ex, np.log(ex + 1.0)))


def tf_softplus_inverse(y):
    y = np.asarray(y, dtype=np.float64)
    small = y < math.exp(_THR)
    large = y > -_THR
    safe = np.where(small | large, 1.0, y)
    val = safe + np.log(-np.expm1(-safe))
    return np.where(small, np.log(np.where(small, y, 1.0)), np.where(large, y, val))


class Sigmoid:
    """tfp.bijectors.Sigmoid (graph.py:36 rho_LF): forward 1/(1+exp(-u)), inverse log(y) - log1p(-y)."""

    lower = None

    def forward(self, u):
        return 1.0 / (1.0 + np.exp(-np.asarray(u, dtype=np.float64)))

    def inverse(self, v):
        v = np.asarray(v, dtype=np.float64)
        return np.log(v) - np.log1p(-v)

    def dforward(self, u):
        y = self.forward(u)
        return y * (1.0 - y)


class Softplus:
    """tfp.bijectors.Softplus, optionally chained with Shift(lower)."""

    def __init__(self, lower: float | None = None):
        self.lower = lower

    def forward(self, u):
        v = tf_softplus(u)
        return v + self.lower if self.lower else v

    def inverse(self, v):
        v = np.asarray(v, dtype=np.float64)
        return tf_softplus_inverse(v - self.lower if self.lower else v)

    def dforward(self, u):
        """TF SoftplusGrad form 1 / (exp(-u) + 1)."""
        return 1.0 / (np.exp(-np.asarray(u, dtype=np.float64)) + 1.0)

    def forward_grad(self, u):
        return 1.0 / (np.exp(-np.asarray(u, dtype=np.float64)) + 1.0)


def positive(lower: float | None = None) -> Softplus:
    """gpflow.utilities.positive (default positive_minimum 0.0 -> plain Softplus)."""
    return Softplus(lower if lower else None)


class Parameter:
    """A (possibly constrained) trainable value: gpflow.Parameter analogue."""

    def __init__(self, value, transform: Softplus | None = None, trainable: bool = True, name: str | None = None):
        self.transform = transform
        self.name = name
        self.trainable = trainable
        self._u = np.array(self._inv(np.asarray(value, dtype=np.float64)), dtype=np.float64)

    # -- transforms
    def _inv(self, v):
        return self.transform.inverse(v) if self.transform else np.array(v, dtype=np.float64)

    def _fwd(self, u):
        return self.transform.forward(u) if self.transform else np.array(u, dtype=np.float64)

    # -- gpflow-like surface
    def numpy(self) -> np.ndarray:
        return np.asarray(self._fwd(self._u), dtype=np.float64)

    def value(self) -> np.ndarray:
        return self.numpy()

    def assign(self, value):
        v = np.asarray(value, dtype=np.float64)
        self._u = np.array(self._inv(np.broadcast_to(v, self._u.shape)), dtype=np.float64)

    @property
    def unconstrained_variable(self) -> np.ndarray:
        return self._u

    @unconstrained_variable.setter
    def unconstrained_variable(self, u):
        self._u = np.array(u, dtype=np.float64).reshape(self._u.shape)

    @property
    def shape(self):
        return self._u.shape

    @property
    def dtype(self):
        return np.float64

    def __array__(self, dtype=None):
        v = self.numpy()
        return v.astype(dtype) if dtype is not None else v

    def __float__(self):
        return float(self.numpy())

    def __repr__(self):
        return f"Parameter(value={self.numpy()!r}, trainable={self.trainable})"


class Module:
    """Minimal gpflow.Module: parameters discovered by attribute traversal."""

    def _submodules(self):
        for k in sorted(vars(self)):
            v = getattr(self, k)
            if isinstance(v, (Module, Parameter)):
                yield k, v
            elif isinstance(v, (list, tuple)):
                for i, e in enumerate(v):
                    if isinstance(e, (Module, Parameter)):
                        yield f"{k}[{i}]", e

    def parameters_with_names(self, prefix=""):
        seen = set()
        out = []

        def rec(mod, pre):
            for k, v in mod._submodules():
                if id(v) in seen:
                    continue
                seen.add(id(v))
                name = f"{pre}.{k}" if pre else k
                if isinstance(v, Parameter):
                    out.append((name, v))
                else:
                    rec(v, name)

        rec(self, prefix)
        return out

    @property
    def parameters(self):
        return tuple(p for _, p in self.parameters_with_names())

    @property
    def trainable_parameters(self):
        return tuple(p for p in self.parameters if p.trainable)

    @property
    def trainable_variables(self):
        return self.trainable_parameters


def set_trainable(obj, flag: bool):
    """gpflow.utilities.set_trainable for a Parameter or every Parameter of a Module."""
    if isinstance(obj, Parameter):
        obj.trainable = flag
    elif isinstance(obj, Module):
        for p in obj.parameters:
            p.trainable = flag
    else:
        raise TypeError(f"cannot set_trainable on {type(obj)}")


def parameter_dict(module: Module) -> dict:
    """gpflow.utilities.parameter_dict analogue: '.path' -> constrained numpy value."""
    return {"." + n: p.numpy().copy() for n, p in module.parameters_with_names()}


def multiple_assign(module: Module, params: dict):
    """gpflow.utilities.multiple_assign analogue."""
    named = {"." + n: p for n, p in module.parameters_with_names()}
    for k, v in params.items():
        if k not in named:
            raise KeyError(f"unknown parameter path {k}")
        named[k].assign(v)


class MFTensor(torch.Tensor):
    """torch.Tensor whose .numpy() works on device tensors (TF eager-tensor habit of
    the reference's callers: ``mean.numpy()``, ``loss.numpy()``)."""

    def numpy(self, *args, **kwargs):  # noqa: D401
        return torch.Tensor.numpy(self.detach().cpu().as_subclass(torch.Tensor), *args, **kwargs)


def as_result(t: torch.Tensor) -> MFTensor:
    return t.as_subclass(MFTensor)
