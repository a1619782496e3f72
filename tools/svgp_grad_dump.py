"""Dump one Goku single-bin and one HBS latent SVGP value + gradient (all outputs) to an .npz, for
bitwise A/B of library builds:  MFGP_LIB_PATH=<lib> python tools/svgp_grad_dump.py OUT.npz
then  python tools/svgp_grad_dump.py --compare A.npz B.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def dump(out):
    import multi_fidelity_gpflow_amd as M
    from conftest import GOKU_DIR, HBS_DIR
    from oracle.mfgp_oracle import load_powerspecs
    res = {}
    g = load_powerspecs(GOKU_DIR)
    X, Y = g["X"], g["Y"]
    Zfix = np.load(os.path.join(ROOT, "tests", "golden", "goku_kmeans_z300.npy"))
    m = M.SingleBinSVGP(X, Y, M.SquaredExponential(lengthscales=np.ones(10)),
                        M.SquaredExponential(lengthscales=np.ones(10)), 64, Z=np.zeros((300, 11)))
    m.inducing_variable.assign(Zfix)
    rng = np.random.default_rng(7)
    m.q_mu.assign(rng.standard_normal((300, 64)) * 0.5)
    m.q_sqrt.assign(np.tril(rng.standard_normal((64, 300, 300)) * 0.01) + 0.1 * np.eye(300)[None])
    e, gd = m.elbo_and_grad((X, Y))
    res["goku_elbo"] = np.array(e)
    for k, v in gd.items():
        res["goku_" + k] = np.asarray(v)
    h = load_powerspecs(HBS_DIR)
    X, Y = h["X"], h["Y"]
    D, P = X.shape[1] - 1, Y.shape[1]
    m = M.LatentMFCoregionalizationSVGP(X, Y, M.SquaredExponential(lengthscales=np.ones(D)),
                                        M.SquaredExponential(lengthscales=np.ones(D)), num_latents=5,
                                        num_inducing=30, num_outputs=P, w_type='diagonal')
    e, gd = m.elbo_and_grad((X, Y))
    res["hbs_elbo"] = np.array(e)
    for k, v in gd.items():
        res["hbs_" + k] = np.asarray(v)
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        same = np.array_equal(A[k], B[k])
        d = float(np.abs(A[k] - B[k]).max() / max(np.abs(A[k]).max(), 1e-300))
        print(f"{k:16s} {'bitwise' if same else 'DIFF'} rel {d:.1e}")
        bad += not same
    print("all bitwise equal" if not bad else f"{bad} arrays differ")


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1])
