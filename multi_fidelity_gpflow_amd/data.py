"""Reference on-disk dataset format (host-side input preparation).

Restates mfgpflow/data_loader.py:278-360 (PowerSpecs.read_from_txt and the
*_norm properties) and mfgpflow/latin_hypercube.py:141-164 (map_to_unit_cube)
without the h5py dependency of the reference module.  This is host glue, not
part of the accelerated path.
"""
from __future__ import annotations

import os

import numpy as np


def map_to_unit_cube(param_vec, param_limits):
    """latin_hypercube.py:141-164: clip to the limits, then map into [0, 1]."""
    param_vec = np.array(param_vec, dtype=np.float64, copy=True)
    lo, hi = param_limits[:, 0], param_limits[:, 1]
    if not (np.all(param_vec - 1e-16 <= hi) and np.all(param_vec + 1e-16 >= lo)):
        raise ValueError("parameter vector outside its limits")
    param_vec = np.minimum(np.maximum(param_vec, lo), hi)
    return (param_vec - lo) / (hi - lo)


def map_to_unit_cube_list(param_vec_list, param_limits):
    return np.array([map_to_unit_cube(p, param_limits) for p in param_vec_list])


def input_normalize(params, param_limits):
    """gpemulator_singlebin.py:24-41 (_map_params_to_unit_cube)."""
    return map_to_unit_cube_list(params, param_limits)


class PowerSpecs:
    """Multi-fidelity P(k) training/test sets in the reference's txt layout."""

    def __init__(self, folder: str = "data/50_LR_3_HR/", n_fidelities: int = 2):
        self.n_fidelities = n_fidelities

    def read_from_txt(self, folder: str = "data/50_LR_3_HR/"):
        self.X_train, self.Y_train = [], []
        for i in range(self.n_fidelities):
            self.X_train.append(np.loadtxt(os.path.join(folder, f"train_input_fidelity_{i}.txt")))
            self.Y_train.append(np.loadtxt(os.path.join(folder, f"train_output_fidelity_{i}.txt")))
        self.parameter_limits = np.loadtxt(os.path.join(folder, "input_limits.txt"))
        self.X_test = [np.loadtxt(os.path.join(folder, "test_input.txt"))]
        self.Y_test = [np.loadtxt(os.path.join(folder, "test_output.txt"))]
        self.kf = np.loadtxt(os.path.join(folder, "kf.txt"))
        assert len(self.kf) == self.Y_test[0].shape[1]
        assert len(self.kf) == self.Y_train[0].shape[1]

    @property
    def X_train_norm(self):
        return [input_normalize(x, self.parameter_limits) for x in self.X_train]

    @property
    def X_test_norm(self):
        return [input_normalize(x, self.parameter_limits) for x in self.X_test]

    @property
    def Y_train_norm(self):
        """LF outputs minus their per-bin sample mean; HF outputs unchanged."""
        out = [y - y.mean(axis=0) for y in self.Y_train[:-1]]
        out.append(self.Y_train[-1])
        return out


def multifidelity_training_set(data: PowerSpecs):
    """Append the fidelity column (0 = LF, 1 = HF) and stack (test_ho2021_multibin.py:29-35)."""
    X_LF, Y_LF = data.X_train_norm[0], data.Y_train_norm[0]
    X_HF, Y_HF = data.X_train_norm[1], data.Y_train_norm[1]
    X = np.vstack([np.hstack([X_LF, np.zeros((len(X_LF), 1))]), np.hstack([X_HF, np.ones((len(X_HF), 1))])])
    Y = np.vstack([Y_LF, Y_HF])
    Xt = data.X_test_norm[0]
    return X, Y, np.hstack([Xt, np.ones((len(Xt), 1))]), data.Y_test[0]


def synthetic_multifidelity(n_lf=16384, n_hf=2048, d=10, p=512, n_test=2048, seed=20251015):
    """The synthetic scale-up configuration of SURVEY §8(d) (the reference has none):
    X ~ U[0,1]^d, Y_L[:, p] = f_p(x) + 0.01 eps, Y_H = 1.2 f_p(x) + 0.1 g_p(x) + 0.005 eps,
    f_p, g_p = (1/sqrt(d)) sum_k sin(2 pi k_pk x_k + phi_pk), k ~ U[0.5, 1.5], phi ~ U[0, 2 pi].
    Returns (X [n_lf+n_hf, d+1] with the fidelity column, Y, X_test [n_test, d+1] HF, Y_test)."""
    rng = np.random.default_rng(seed)
    kf, pf = rng.uniform(0.5, 1.5, (p, d)), rng.uniform(0, 2 * np.pi, (p, d))
    kg, pg = rng.uniform(0.5, 1.5, (p, d)), rng.uniform(0, 2 * np.pi, (p, d))

    def f(x, k, ph):
        return np.sin(2 * np.pi * x[:, None, :] * k[None] + ph[None]).sum(-1) / np.sqrt(d)

    XL = rng.uniform(0, 1, (n_lf, d))
    XH = rng.uniform(0, 1, (n_hf, d))
    Xt = rng.uniform(0, 1, (n_test, d))
    YL = f(XL, kf, pf) + 0.01 * rng.standard_normal((n_lf, p))
    YH = 1.2 * f(XH, kf, pf) + 0.1 * f(XH, kg, pg) + 0.005 * rng.standard_normal((n_hf, p))
    Yt = 1.2 * f(Xt, kf, pf) + 0.1 * f(Xt, kg, pg)
    X = np.vstack([np.hstack([XL, np.zeros((n_lf, 1))]), np.hstack([XH, np.ones((n_hf, 1))])])
    return X, np.vstack([YL, YH]), np.hstack([Xt, np.ones((n_test, 1))]), Yt
