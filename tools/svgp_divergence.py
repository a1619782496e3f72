"""Where the Goku SingleBinSVGP device trajectory leaves the oracle's (diagnostic, GPU box):
step-by-step -ELBO and parameter differences between the device trainer (libmfgp.so) and the
torch-autograd oracle trainer (oracle/svgp_oracle.py SingleBinTrainer), both from the committed
KMeans centres, plus the step-0 gradient error per parameter group.
    python tools/svgp_divergence.py [steps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import multi_fidelity_gpflow_amd as M                         # noqa: E402
from oracle import mfgp_oracle as O                           # noqa: E402
from oracle import svgp_oracle as S                           # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 31
    d = O.load_powerspecs(os.path.join(ROOT, "tests", "golden", "data",
                                       "matter_power_1128_Box1000_Part750_36_Box1000_Part3000_z0"))
    X, Y = d["X"], d["Y"]
    D, P = X.shape[1] - 1, Y.shape[1]
    Zf = np.load(os.path.join(ROOT, "tests", "golden", "goku_kmeans_z300.npy"))
    m = M.SingleBinSVGP(X, Y, M.SquaredExponential(lengthscales=np.ones(D)),
                        M.SquaredExponential(lengthscales=np.ones(D)), P, Z=np.zeros((300, D + 1)))
    m.inducing_variable.assign(Zf)
    # step-0 gradients: device vs autograd through the oracle
    e, gd = m.elbo_and_grad((X, Y))
    from test_gpu_svgp import _autograd_grads
    eo, ga = _autograd_grads(m, X, Y)
    print(f"step-0 ELBO rel err {abs(e - eo) / abs(eo):.2e}")
    for k, ref in ga.items():
        got = np.asarray(gd[k]).reshape(np.shape(ref))
        scale = max(np.abs(ref).max(), 1e-30)
        rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)
        print(f"  grad {k:7s} max|err|/max|ref| {np.abs(got - ref).max() / scale:.2e}   "
              f"median elementwise rel {np.median(rel):.2e}")
    if "theta" in ga:
        th_err = np.abs(np.asarray(gd["theta"]) - ga["theta"]) / np.maximum(np.abs(ga["theta"]).max(0), 1e-300)
        print("  theta columns max err / column scale:", np.array2string(th_err.max(0), precision=1))
    tr = M.svgp._SVGPTrainer(m, (X, Y), max_iters=1000, initial_lr=0.1, graph=False)
    orc = S.SingleBinTrainer(X, Y, Zf, lr=0.1, max_iters=1000)
    for i in range(steps):
        tr.run(1)
        orc.step()
        dev = -tr.elbo_now()
        ref = float(orc.neg_elbo().detach())
        Z, kps, q_mu, q_sqrt, noise = orc.constrained()
        dZ = np.abs(tr.view(tr.c, "Z").cpu().numpy() - Z.detach().numpy()).max()
        dq = np.abs(tr.view(tr.c, "q_mu").cpu().numpy() - q_mu.detach().numpy()).max()
        th = tr.view(tr.c, "theta").cpu().numpy()
        lL = np.stack([kp["lL"].detach().numpy() for kp in kps])
        dl = np.abs(th[:, 1:1 + D] - lL).max() / np.abs(lL).max()
        print(f"step {i:2d}  -ELBO dev {dev:.12e}  oracle {ref:.12e}  rel {abs(dev - ref) / abs(ref):.1e}  "
              f"|dZ| {dZ:.1e}  |dq_mu| {dq:.1e}  |dlL|rel {dl:.1e}", flush=True)


if __name__ == "__main__":
    main()
