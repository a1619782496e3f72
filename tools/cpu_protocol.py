"""The CPU baseline's full protocol, timed once: the notebook's Goku training --
1000 Keras-Adam steps at lr 0.1 on the LML value+gradient (noise fixed, as the reference's Adam path
leaves it) -- then predict_f(X_test), on the host cores of the machine this runs on, with the
torch-MKL fp64 restatement (oracle/torch_oracle.py) and the oracle's Adam (oracle/mfgp_oracle.py).
bench.py's cpu_baseline reports the evals/s of a bounded sample; this measures the whole protocol.

  python tools/cpu_protocol.py [OUT.json] [--steps N]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import host_cpus, load_goku  # noqa: E402
from oracle import mfgp_oracle as O  # noqa: E402
from oracle import torch_oracle as TO  # noqa: E402


def main():
    out = next((a for a in sys.argv[1:] if a.endswith(".json")), None)
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 1000
    X, Y, Xt, _ = load_goku()
    D, P = X.shape[1] - 1, Y.shape[1]
    cores, src = host_cpus()
    torch.set_num_threads(cores)
    Xd, Yd = torch.as_tensor(X), torch.as_tensor(Y)
    p0 = O.MFParams.initial(D, P)
    u = O.pack_unconstrained(p0)
    opt = O.AdamTF210(lr=0.1)
    hist = []
    t0 = time.perf_counter()
    for _ in range(steps):
        p = O.unpack_unconstrained(u, p0)
        lml, g = TO.lml_and_grad(Xd, Yd, p.vL, torch.as_tensor(p.lL), p.vD, torch.as_tensor(p.lD), p.rho0, p.noise)
        g = g.numpy()
        hist.append(-lml)
        gl = {"vL": -g[0], "lL": -g[1:1 + D], "vD": -g[1 + D], "lD": -g[2 + D:2 + 2 * D], "rho0": -g[2 + 2 * D]}
        u = opt.step(u, O.grad_unconstrained(u, gl))
    t_train = time.perf_counter() - t0
    t1 = time.perf_counter()
    mean, var = O.gpr_predict_f(X, Y, Xt, O.unpack_unconstrained(u, p0))
    t_pred = time.perf_counter() - t1
    res = {"protocol": f"Goku {steps} Keras-Adam steps (lr 0.1, noise fixed) + predict_f(X_test), fp64 on the CPU",
           "train_s": round(t_train, 3), "predict_s": round(t_pred, 3), "train_predict_s": round(t_train + t_pred, 3),
           "steps": steps, "evals_per_s": round(steps / t_train, 3), "cores": cores, "cores_source": src,
           "loss_first_last": [float(hist[0]), float(hist[-1])],
           "implementation": "oracle/torch_oracle.py lml_and_grad (MKL) + oracle/mfgp_oracle.py AdamTF210; "
                             "predict: oracle/mfgp_oracle.py gpr_predict_f (NumPy)",
           "published_m1_cpu_s": 142.36}
    line = json.dumps(res)
    print(line)
    if out:
        with open(out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
