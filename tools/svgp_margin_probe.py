"""Diagnostic (VERDICT r5 missing #3 / weak #4): where the SVGP value path's ~1e-8 relative ELBO
margin against the torch-CPU oracle comes from.  The Goku single-bin state of
tests/test_gpu_svgp.py::test_goku_singlebin_grad_vs_autograd (qscale 0.1); the device's value path
(mfgp_svgp_elbo) is run once and its workspace read back (svgp_layout's offsets, mfgp_svgp.hip), so
every stage is compared with the oracle's on the same inputs:
  Kuu, Kuf         the device Gram tiles vs the oracle's mf_K_t
  Li               the device L^{-1} (step sequence) vs inv(cholesky(Kuu_oracle))
  sum A^2          Li Kuf column sums (the explicit-inverse form) vs the oracle's triangular solve
  g_var, g_mu      the device's latent moments vs the oracle's latent_moments
and the same A / sum A^2 re-formed on the CPU from the DEVICE Kuu / Kuf by (a) inv(chol) and
(b) a triangular solve, which separates the Gram's rounding from A's formation.

  python tools/svgp_margin_probe.py       (GPU; writes gpurun_out/svgp_margin_probe.json)
"""
import json
import os
import sys

import numpy as np
import scipy.linalg as sla
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import multi_fidelity_gpflow_amd as M  # noqa: E402
from multi_fidelity_gpflow_amd.engine import Engine  # noqa: E402
from oracle import svgp_oracle as S  # noqa: E402
from oracle.mfgp_oracle import load_powerspecs  # noqa: E402
from conftest import GOKU_DIR  # noqa: E402


def layout(nb, n, m, l):
    """svgp_layout (mfgp_svgp.hip): byte offsets of Kuu, R, Xo, Dd, ldiag, Lq, C, Kuf."""
    Tm, Tn = -(-m // nb), -(-n // nb)
    mpad, npad = Tm * nb, Tn * nb
    mm = mpad * mpad
    off, res = 0, {}
    for name, cnt in (("Kuu", mm * l), ("R", mm * l), ("Xo", mm * l), ("Dd", Tm * nb * nb * l), ("ldiag", mpad * l),
                      ("Lq", mm * l), ("C", mm * l), ("Kuf", mpad * npad * l)):
        off = (off + 255) & ~255
        res[name] = (off // 8, cnt)
        off += cnt * 8
    return res, mpad, npad


def main():
    g = load_powerspecs(GOKU_DIR)
    X, Y = g["X"], g["Y"]
    Zfix = np.load(os.path.join(ROOT, "tests", "golden", "goku_kmeans_z300.npy"))
    m = M.SingleBinSVGP(X, Y, M.SquaredExponential(lengthscales=np.ones(10)),
                        M.SquaredExponential(lengthscales=np.ones(10)), 64, Z=np.zeros((300, 11)))
    m.inducing_variable.assign(Zfix)
    rng = np.random.default_rng(7)
    L, Mi = 64, 300
    m.q_mu.assign(rng.standard_normal((Mi, L)) * 0.5)
    m.q_sqrt.assign(np.tril(rng.standard_normal((L, Mi, Mi)) * 0.01) + 0.1 * np.eye(Mi)[None])
    eng = Engine.get()
    cap = {}
    orig = eng.svgp_elbo

    def spy(*a, **k):
        r = orig(*a, **k)
        torch.cuda.synchronize()
        cap["res"] = [t.cpu().numpy() for t in r]
        cap["wsd"] = eng._ws["svgp"].cpu().numpy().view(np.float64)   # the workspace the call used
        return r

    eng.svgp_elbo = spy
    e_dev = float(m.elbo((X, Y)))
    eng.svgp_elbo = orig
    Z = torch.tensor(Zfix)
    D = 10
    kps = []
    for k in m.kernel.kernels:
        t = k.theta_vector(D)
        kps.append(dict(vL=torch.tensor(t[0]), lL=torch.tensor(t[1:1 + D]), vD=torch.tensor(t[1 + D]),
                        lD=torch.tensor(t[2 + D:2 + 2 * D]), rho=torch.tensor(t[2 + 2 * D])))
    q_mu = torch.tensor(m.q_mu.numpy())
    q_sqrt = torch.tensor(m.q_sqrt.numpy())
    noise = torch.tensor(float(m.likelihood.variance.numpy()), dtype=torch.float64)
    noise32 = torch.tensor(float(m.likelihood.variance.numpy()))   # the old test helper's fp32 scalar
    Xt, Yt = torch.tensor(X), torch.tensor(Y)
    e_or, _, _ = S.elbo_t(Xt, Yt, Z, kps, q_mu, q_sqrt, None, noise)
    e_or = float(e_or)
    gm_o, gv_o = S.latent_moments(Xt, Z, kps, q_mu, q_sqrt)
    out, gmu_d, gvar_d, info = cap["res"]
    e_o, kl_o, ve_o = [float(v) for v in S.elbo_t(Xt, Yt, Z, kps, q_mu, q_sqrt, None, noise)]
    nz = float(noise)
    ve_np = float((-0.5 * S.LOG2PI - 0.5 * np.log(nz) - 0.5 * ((Y - gmu_d.T) ** 2 + gvar_d.T) / nz).sum())
    ve_onp = float((-0.5 * S.LOG2PI - 0.5 * np.log(nz) - 0.5 * ((Y - gm_o.numpy()) ** 2 + gv_o.numpy()) / nz).sum())
    Lq = np.tril(q_sqrt.numpy())
    kl_np = 0.5 * float((q_mu.numpy() ** 2).sum() - Mi * L + (Lq ** 2).sum()
                        - np.log(np.diagonal(Lq, axis1=1, axis2=2) ** 2).sum())
    parts = {"device": {"elbo": float(out[0]), "kl": float(out[1]), "ve": float(out[2])},
             "oracle": {"elbo": e_o, "kl": kl_o, "ve": ve_o},
             "numpy_from_device_moments": {"ve": ve_np}, "numpy_from_oracle_moments": {"ve": ve_onp},
             "numpy_kl": kl_np, "noise": nz,
             # what torch.tensor(python_float) (fp32) made of the oracle's per-term constant, times N P
             "fp32_noise_constant_shift": float(Y.size * (float(-0.5 * S.LOG2PI - 0.5 * torch.log(noise32))
                                                          - (-0.5 * S.LOG2PI - 0.5 * np.log(nz))))}
    rep = {"elbo_dev": e_dev, "elbo_oracle": e_or, "elbo_rel": abs(e_dev - e_or) / abs(e_or),
           "g_var_abs_max": float(np.abs(gvar_d.T - gv_o.numpy()).max()),
           "g_var_sum_err": float((gvar_d.T - gv_o.numpy()).sum()),
           "g_mu_abs_max": float(np.abs(gmu_d.T - gm_o.numpy()).max()), "parts": parts}
    w = cap["wsd"]
    n = X.shape[0]
    lay, mpad, npad = layout(32, n, Mi, L)
    per = []
    for l in (0, 1, 17, 63):
        kp = kps[l]
        Kuu_o = (S.mf_K_t(Z, Z, kp) + S.JITTER * torch.eye(Mi, dtype=torch.float64)).numpy()
        Kuf_o = S.mf_K_t(Z, Xt, kp).numpy()
        o, _ = lay["Kuf"]
        Kuf_d = w[o + l * mpad * npad: o + (l + 1) * mpad * npad].reshape(mpad, npad)[:Mi, :n]
        o, _ = lay["Xo"]
        Li_d = w[o + l * mpad * mpad: o + (l + 1) * mpad * mpad].reshape(mpad, mpad)[:Mi, :Mi]
        Lo = np.linalg.cholesky(Kuu_o)
        A_o = sla.solve_triangular(Lo, Kuf_o, lower=True)
        Li_o = sla.solve_triangular(Lo, np.eye(Mi), lower=True)
        q_o = (A_o * A_o).sum(0)
        A_dev = np.tril(Li_d) @ Kuf_d            # the device's explicit-inverse form, CPU arithmetic
        q_dev = (A_dev * A_dev).sum(0)
        A_dt = sla.solve_triangular(np.linalg.inv(np.tril(Li_d)), Kuf_d, lower=True)
        # A from the oracle's factor and the DEVICE's Kuf: the Gram's own share
        A_gk = sla.solve_triangular(Lo, Kuf_d, lower=True)
        A_gi = Li_o @ Kuf_o                       # the oracle factor, explicit inverse
        per.append({"latent": l,
                    "Kuf_rel": float(np.abs(Kuf_d - Kuf_o).max() / np.abs(Kuf_o).max()),
                    "Li_rel": float(np.abs(np.tril(Li_d) - Li_o).max() / np.abs(Li_o).max()),
                    "Li_absmax": float(np.abs(Li_o).max()),
                    "sumA2_dev_form": float(np.abs(q_dev - q_o).max()),
                    "sumA2_oracleL_devKuf": float(np.abs((A_gk * A_gk).sum(0) - q_o).max()),
                    "sumA2_oracleL_inverse": float(np.abs((A_gi * A_gi).sum(0) - q_o).max()),
                    "sumA2_devL_trsm": float(np.abs((A_dt * A_dt).sum(0) - q_o).max()),
                    "g_var_dev": float(np.abs(gvar_d[l] - gv_o.numpy()[:, l]).max())})
    rep["latents"] = per
    print(json.dumps(rep, indent=1))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "svgp_margin_probe.json"), "w") as f:
        json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
