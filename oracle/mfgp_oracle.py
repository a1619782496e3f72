"""fp64 NumPy/SciPy restatement of the reference's multi-fidelity GP hot path.

TEST INFRASTRUCTURE ONLY — this module is the parity checker for the HIP
path and the timed CPU baseline in ``bench.py``.  The product package never
imports it.

Parity status: PINNED.  The reference (``mfgpflow`` on GPflow 2.9.0 /
TensorFlow 2.10) cannot be imported in this container (``ModuleNotFoundError:
No module named 'gpflow'`` — an ordinary missing dependency, not a permission
denial; there is no network to install it).  The restatement below is pinned
against every numeric value the reference itself recorded (notebook outputs,
committed as ``tests/golden/kats.json``): initial LMLs (HBS, Goku), Adam LML
trajectories, the Forrester L-BFGS ρ, and the SingleBinSVGP −ELBO sequence.

Third-party algorithms restated here (not vendored in /root/reference):
  gpflow==2.9.0 (requirements.txt:2): kernels.SquaredExponential,
      utilities.ops.square_distance, models.GPR.log_marginal_likelihood /
      predict_f, conditionals.base_conditional, optimizers.Scipy,
      likelihoods.Gaussian (variance lower bound 1e-6), utilities.positive.
  tensorflow==2.10 (requirements.txt:9): tf.math.softplus, Keras (legacy) Adam
      ResourceApplyAdam update, CosineDecay schedule.
  tensorflow-probability~=0.18: bijectors.Softplus / Shift, softplus_inverse.

Reference call sites are cited per function.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np
import scipy.linalg as sla

LOG2PI = math.log(2.0 * math.pi)
_SP_THRESH = math.log(np.finfo(np.float64).eps) + 2.0   # TF softplus_op.h threshold


# ---------------------------------------------------------------- transforms
def softplus(x):
    """tf.math.softplus (tensorflow/core/kernels/softplus_op.h): log(exp(x)+1)
    with the eps-based large/small thresholds."""
    x = np.asarray(x, dtype=np.float64)
    ex = np.exp(np.minimum(x, 700.0))
    return np.where(x > -_SP_THRESH, x, np.where(x < _SP_THRESH, ex, np.log(ex + 1.0)))


def softplus_grad(x):
    """TF SoftplusGrad: 1 / (exp(-x) + 1)."""
    x = np.asarray(x, dtype=np.float64)
    return 1.0 / (np.exp(-x) + 1.0)


def softplus_inverse(y):
    """tfp.math.softplus_inverse (TFP 0.18)."""
    y = np.asarray(y, dtype=np.float64)
    too_small = y < math.exp(_SP_THRESH)
    too_large = y > -_SP_THRESH
    safe = np.where(too_small | too_large, 1.0, y)
    val = safe + np.log(-np.expm1(-safe))
    return np.where(too_small, np.log(np.where(too_small, y, 1.0)), np.where(too_large, y, val))


NOISE_SHIFT = 1e-6   # gpflow.likelihoods.Gaussian variance lower bound (Shift(1e-6) ∘ Softplus)


# ---------------------------------------------------------------- data prep
def map_to_unit_cube(x, limits):
    """mfgpflow/latin_hypercube.py:141-164 (clip to limits, then affine map)."""
    x = np.array(x, dtype=np.float64, copy=True)
    lo, hi = limits[:, 0], limits[:, 1]
    x = np.where(x > hi, hi, x)
    x = np.where(x < lo, lo, x)
    return (x - lo) / (hi - lo)


def load_powerspecs(folder):
    """mfgpflow/data_loader.py:288-360 (PowerSpecs.read_from_txt + *_norm):
    X normalised into the unit cube by input_limits.txt; LF outputs mean-subtracted
    per bin; HF outputs unchanged.  Returns the training X with the fidelity
    column appended (test_ho2021_multibin.py:32-35)."""
    ld = lambda n: np.loadtxt(os.path.join(folder, n))
    lim = ld("input_limits.txt")
    xl, xh = ld("train_input_fidelity_0.txt"), ld("train_input_fidelity_1.txt")
    yl, yh = ld("train_output_fidelity_0.txt"), ld("train_output_fidelity_1.txt")
    xt, yt = ld("test_input.txt"), ld("test_output.txt")
    xl_n = np.array([map_to_unit_cube(r, lim) for r in xl])
    xh_n = np.array([map_to_unit_cube(r, lim) for r in xh])
    xt_n = np.array([map_to_unit_cube(r, lim) for r in xt])
    yl_n = yl - yl.mean(axis=0)
    X = np.vstack([np.hstack([xl_n, np.zeros((len(xl_n), 1))]),
                   np.hstack([xh_n, np.ones((len(xh_n), 1))])])
    Y = np.vstack([yl_n, yh])
    Xt = np.hstack([xt_n, np.ones((len(xt_n), 1))])
    return dict(X=X, Y=Y, Xtest=Xt, Ytest=yt, kf=ld("kf.txt"))


# ---------------------------------------------------------------- kernels
def square_distance(a, b):
    """gpflow 2.9 utilities/ops.py:square_distance (X2 given branch, no clamp):
    dist = -2 a·bᵀ + (‖a‖² ⊕ ‖b‖²)."""
    as_ = np.sum(a * a, axis=-1)
    bs = np.sum(b * b, axis=-1)
    return -2.0 * (a @ b.T) + (as_[:, None] + bs[None, :])


def rbf_K(X1, X2, variance, lengthscales):
    """gpflow.kernels.SquaredExponential.K = variance·exp(-½ r²) on X/ℓ."""
    ls = np.asarray(lengthscales, dtype=np.float64)
    return variance * np.exp(-0.5 * square_distance(X1 / ls, X2 / ls))


@dataclass
class MFParams:
    """Constrained hyper-parameters of LinearMultiFidelityKernel + Gaussian noise."""
    vL: float
    lL: np.ndarray
    vD: float
    lD: np.ndarray
    rho: np.ndarray                  # (P, 1); only rho[0,0] is ever used (linear.py:90)
    noise: float = 1e-3

    @property
    def rho0(self):
        return float(np.asarray(self.rho).reshape(-1)[0])

    @staticmethod
    def initial(D, P=1, noise=1e-3):
        return MFParams(1.0, np.ones(D), 1.0, np.ones(D), np.ones((P, 1)), noise)

    def copy(self):
        return MFParams(self.vL, np.array(self.lL), self.vD, np.array(self.lD),
                        np.array(self.rho), self.noise)


def mf_K(X, X2, p: MFParams):
    """mfgpflow/linear.py:55-104 LinearMultiFidelityKernel.K — masks, gathers and
    scatters of the four blocks; rows whose fidelity is not exactly 0 or 1 stay 0."""
    X = np.asarray(X, dtype=np.float64)
    X2 = X if X2 is None else np.asarray(X2, dtype=np.float64)
    mL, mH = np.where(X[:, -1] == 0)[0], np.where(X[:, -1] == 1)[0]
    m2L, m2H = np.where(X2[:, -1] == 0)[0], np.where(X2[:, -1] == 1)[0]
    XL, XH, X2L, X2H = X[mL, :-1], X[mH, :-1], X2[m2L, :-1], X2[m2H, :-1]
    rho = p.rho0
    K = np.zeros((X.shape[0], X2.shape[0]))
    K[np.ix_(mL, m2L)] = rbf_K(XL, X2L, p.vL, p.lL)
    K[np.ix_(mL, m2H)] = rbf_K(XL, X2H, p.vL, p.lL) * rho
    K[np.ix_(mH, m2L)] = rbf_K(XH, X2L, p.vL, p.lL) * rho
    K[np.ix_(mH, m2H)] = rbf_K(XH, X2H, p.vL, p.lL) * (rho * rho) + rbf_K(XH, X2H, p.vD, p.lD)
    return K


def mf_Kdiag(X, p: MFParams):
    """mfgpflow/linear.py:106-136 LinearMultiFidelityKernel.K_diag."""
    f = np.asarray(X)[:, -1]
    rho = p.rho0
    return np.where(f == 0, p.vL, np.where(f == 1, p.vL * (rho ** 2) + p.vD, 0.0))


# ---------------------------------------------------------------- GPR
def gpr_lml(X, Y, p: MFParams):
    """gpflow GPR.log_marginal_likelihood (inherited at linear.py:138/153):
    L = chol(K + σ²I); Σ_p multivariate_normal(y_p | 0, L)."""
    K = mf_K(X, None, p)
    K[np.diag_indices_from(K)] += p.noise
    L = np.linalg.cholesky(K)
    A = sla.solve_triangular(L, Y, lower=True)
    N, P = Y.shape
    return float(-0.5 * np.sum(A * A) - P * np.sum(np.log(np.diag(L))) - 0.5 * N * P * LOG2PI)


def _pair_blocks(X, p: MFParams):
    f = X[:, -1]
    isL, isH = (f == 0).astype(float), (f == 1).astype(float)
    s = isL + p.rho0 * isH
    h = isH
    XL = X[:, :-1]
    kL = rbf_K(XL, XL, p.vL, p.lL)
    kD = rbf_K(XL, XL, p.vD, p.lD)
    return s, h, isL + isH, XL, kL, kD


def gpr_lml_and_grad(X, Y, p: MFParams):
    """LML and its analytic gradient w.r.t. the CONSTRAINED hyper-parameters.

    Equivalent to GradientTape through linear.py:206 (value) — ∂LML/∂θ =
    ½ Σ_ij W_ij ∂K_ij/∂θ with W = ααᵀ − P·K⁻¹, α = K⁻¹Y.
    Returns (lml, dict(vL, lL[D], vD, lD[D], rho0, noise))."""
    X = np.asarray(X, dtype=np.float64)
    N, P = Y.shape
    K = mf_K(X, None, p)
    K[np.diag_indices_from(K)] += p.noise
    L = np.linalg.cholesky(K)
    Z = sla.solve_triangular(L, Y, lower=True)
    lml = float(-0.5 * np.sum(Z * Z) - P * np.sum(np.log(np.diag(L))) - 0.5 * N * P * LOG2PI)
    alpha = sla.solve_triangular(L.T, Z, lower=False)
    Linv = sla.solve_triangular(L, np.eye(N), lower=True)
    Kinv = Linv.T @ Linv
    W = alpha @ alpha.T - P * Kinv
    s, h, valid, Xc, kL, kD = _pair_blocks(X, p)
    SS = np.outer(s, s)
    HH = np.outer(h, h)
    SH = np.outer(h, s) + np.outer(s, h)
    g = {}
    # dK/dv = exp(-r2/2): TF's autodiff of v * exp(-r2/2) (GPflow SquaredExponential.K), finite
    # where v underflows to 0 (the division form K / v gave 0/0 at L-BFGS line-search points)
    eL = rbf_K(Xc, Xc, 1.0, p.lL)
    eD = rbf_K(Xc, Xc, 1.0, p.lD)
    g["vL"] = 0.5 * np.sum(W * SS * eL)
    g["vD"] = 0.5 * np.sum(W * HH * eD)
    g["rho0"] = 0.5 * np.sum(W * SH * kL)
    D = Xc.shape[1]
    gl, gd = np.zeros(D), np.zeros(D)
    for d in range(D):
        diff2 = (Xc[:, d][:, None] - Xc[:, d][None, :]) ** 2
        gl[d] = 0.5 * np.sum(W * SS * kL * diff2) / p.lL[d] ** 3
        gd[d] = 0.5 * np.sum(W * HH * kD * diff2) / p.lD[d] ** 3
    g["lL"], g["lD"] = gl, gd
    g["noise"] = 0.5 * np.trace(W)
    return lml, g


def gpr_predict_f(X, Y, Xnew, p: MFParams):
    """gpflow GPR.predict_f(full_cov=False) → base_conditional(white=False)
    (verbatim mirror at linear.py:237-286). Variance is tiled over the P outputs."""
    K = mf_K(X, None, p)
    K[np.diag_indices_from(K)] += p.noise
    Lm = np.linalg.cholesky(K)
    Kmn = mf_K(X, Xnew, p)
    A = sla.solve_triangular(Lm, Kmn, lower=True)
    var = mf_Kdiag(Xnew, p) - np.sum(A * A, axis=0)
    A2 = sla.solve_triangular(Lm.T, A, lower=False)
    mean = A2.T @ Y
    return mean, np.tile(var[:, None], (1, Y.shape[1]))


def gpr_predict_f_full_cov(X, Y, Xnew, p: MFParams):
    """gpflow GPR.predict_f(full_cov=True) → base_conditional(full_cov=True, white=False):
    fvar = Knn − AᵀA with Knn = K(X*, X*), tiled to [P, N*, N*]."""
    K = mf_K(X, None, p)
    K[np.diag_indices_from(K)] += p.noise
    Lm = np.linalg.cholesky(K)
    Kmn = mf_K(X, Xnew, p)
    A = sla.solve_triangular(Lm, Kmn, lower=True)
    cov = mf_K(Xnew, None, p) - A.T @ A
    mean = sla.solve_triangular(Lm.T, A, lower=False).T @ Y
    return mean, np.tile(cov[None], (Y.shape[1], 1, 1))


# ---------------------------------------------------------------- unconstrained vector
def pack_unconstrained(p: MFParams, with_noise=False):
    """Trainable unconstrained vector [vL, lL(D), vD, lD(D), rho0, (noise)]."""
    u = [softplus_inverse(p.vL)], softplus_inverse(p.lL), [softplus_inverse(p.vD)], \
        softplus_inverse(p.lD), [softplus_inverse(p.rho0)]
    u = np.concatenate([np.atleast_1d(np.asarray(a, dtype=np.float64)) for a in u])
    if with_noise:
        u = np.concatenate([u, [softplus_inverse(p.noise - NOISE_SHIFT)]])
    return u


def unpack_unconstrained(u, template: MFParams, with_noise=False):
    D = len(template.lL)
    q = template.copy()
    q.vL = float(softplus(u[0]))
    q.lL = softplus(u[1:1 + D])
    q.vD = float(softplus(u[1 + D]))
    q.lD = softplus(u[2 + D:2 + 2 * D])
    rho = np.array(q.rho, dtype=np.float64)
    rho.reshape(-1)[0] = softplus(u[2 + 2 * D])
    q.rho = rho
    if with_noise:
        q.noise = float(softplus(u[3 + 2 * D]) + NOISE_SHIFT)
    return q


def softplus_backprop(g, u):
    """TF SoftplusGrad as autodiff applies it: upstream / (exp(-u) + 1)."""
    return g / (np.exp(-np.asarray(u, dtype=np.float64)) + 1.0)


def grad_unconstrained(u, g, with_noise=False):
    """Chain rule through Softplus (TF SoftplusGrad form)."""
    gc = np.concatenate([[g["vL"]], g["lL"], [g["vD"]], g["lD"], [g["rho0"]]]
                        + ([[g["noise"]]] if with_noise else []))
    return softplus_backprop(gc, u)


# ---------------------------------------------------------------- optimisers
def _f32(x):
    return float(np.float32(x))


class AdamTF210:
    """Keras (legacy OptimizerV2, TF 2.10) Adam → ResourceApplyAdam:
    m += (g-m)(1-β1); v += (g²-v)(1-β2); var -= lr·√(1-β2ᵗ)/(1-β1ᵗ) · m/(√v+ε).

    OptimizerV2 stores learning_rate / beta_1 / beta_2 as float32 hyper variables
    (add_weight default dtype) and casts them to the fp64 var dtype, so the
    effective lr is float32(0.1) = 0.10000000149…; ε stays a python float.
    With this rounding the HBS trajectory matches the recorded notebook output
    to ≤2e-15 through iteration 500 (it turns chaotic after ≈520)."""

    def __init__(self, lr=0.001, beta1=0.9, beta2=0.999, eps=1e-7, schedule=None):
        self.lr, self.b1, self.b2 = _f32(lr), _f32(beta1), _f32(beta2)
        self.eps, self.schedule = eps, schedule
        self.t = 0
        self.m = self.v = None

    def step(self, u, g):
        if self.m is None:
            self.m, self.v = np.zeros_like(u), np.zeros_like(u)
        lr = self.schedule(self.t) if self.schedule is not None else self.lr
        self.t += 1
        b1p, b2p = self.b1 ** self.t, self.b2 ** self.t
        alpha = lr * math.sqrt(1.0 - b2p) / (1.0 - b1p)
        self.m += (g - self.m) * (1.0 - self.b1)
        self.v += (g * g - self.v) * (1.0 - self.b2)
        return u - (self.m * alpha) / (np.sqrt(self.v) + self.eps)


def cosine_decay_f32(initial_lr, decay_steps):
    """tf.keras.optimizers.schedules.CosineDecay (TF 2.10, alpha=0): computed in
    float32 (dtype of the python-float initial lr), then cast to float64."""
    def sched(step):
        lr0 = np.float32(initial_lr)
        frac = np.float32(min(step, decay_steps)) / np.float32(decay_steps)
        cosd = np.float32(0.5) * (np.float32(1.0) + np.cos(np.float32(math.pi) * frac, dtype=np.float32))
        return float(np.float32(lr0 * cosd))
    return sched


def adam_train(X, Y, p0: MFParams, max_iters=1000, learning_rate=0.1, record=None):
    """MultiFidelityGPModel.optimize(use_adam=True) — linear.py:190-221.
    The noise stays fixed (set_trainable after tf.function tracing is a no-op;
    SURVEY Appendix C-2). loss_history holds the pre-step −LML."""
    u = pack_unconstrained(p0)
    opt = AdamTF210(lr=learning_rate)
    hist = []
    for _ in range(max_iters):
        p = unpack_unconstrained(u, p0)
        lml, g = gpr_lml_and_grad(X, Y, p)
        hist.append(-lml)
        u = opt.step(u, grad_unconstrained(u, {k: -np.asarray(v) for k, v in g.items()}))
    return unpack_unconstrained(u, p0), np.array(hist)


def lbfgs_train(X, Y, p0: MFParams, max_iters=1000, return_trace=False):
    """optimize(use_adam=False) — linear.py:223-234 through gpflow.optimizers.Scipy:
    L-BFGS-B (jac=True) over the concatenated UNCONSTRAINED trainables in tf.Module
    attribute order [lL(D), vL, lD(D), vD, rho (all P), (noise)], first with the
    noise fixed, then again with it trainable.  The unconstrained values persist
    between the two passes; the noise is always Shift(1e-6) o Softplus of its
    variable (so its initial value is softplus(softplus_inverse(1e-3 - 1e-6)) + 1e-6).
    The objective is degenerate (the noise runs to its 1e-6 floor), so the end
    point is sensitive to 1e-16-level arithmetic differences."""
    from scipy.optimize import minimize

    D = len(p0.lL)
    P = np.asarray(p0.rho).reshape(-1).size
    u = {"lL": softplus_inverse(p0.lL), "vL": np.atleast_1d(softplus_inverse(p0.vL)),
         "lD": softplus_inverse(p0.lD), "vD": np.atleast_1d(softplus_inverse(p0.vD)),
         "rho": softplus_inverse(np.asarray(p0.rho, dtype=np.float64).reshape(-1)),
         "noise": np.atleast_1d(softplus_inverse(p0.noise - NOISE_SHIFT))}

    def params():
        return MFParams(float(softplus(u["vL"][0])), softplus(u["lL"]), float(softplus(u["vD"][0])),
                        softplus(u["lD"]), softplus(u["rho"]).reshape(P, 1),
                        float(softplus(u["noise"][0]) + NOISE_SHIFT))

    trace = []
    for phase in (0, 1):
        keys = ["lL", "vL", "lD", "vD", "rho"] + (["noise"] if phase else [])
        sizes = [u[k].size for k in keys]

        def unpack(x):
            o = 0
            for k, n in zip(keys, sizes):
                u[k] = np.array(x[o:o + n])
                o += n

        def fg(x):
            unpack(x)
            lml, g = gpr_lml_and_grad(X, Y, params())
            gd = {"lL": g["lL"], "vL": [g["vL"]], "lD": g["lD"], "vD": [g["vD"]],
                  "rho": np.r_[g["rho0"], np.zeros(P - 1)], "noise": [g["noise"]]}
            trace.append(-lml)
            return -lml, np.concatenate([softplus_backprop(-np.asarray(gd[k], dtype=np.float64), u[k]) for k in keys])

        res = minimize(fg, np.concatenate([u[k] for k in keys]), jac=True, method="L-BFGS-B",
                       options={"maxiter": max_iters})
        unpack(res.x)
    return (params(), np.array(trace)) if return_trace else params()
