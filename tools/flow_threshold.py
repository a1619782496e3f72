"""Where the persistent flow starts to pay: Cholesky phase time (hipEvents, ms) of one fp64 LML
value+grad evaluation with the flow (k_chol_flow) and with the launch-per-step schedule
(k_chol_step x T), over problem sizes.  Diagnostic (GPU box): python tools/flow_threshold.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multi_fidelity_gpflow_amd.engine import Engine, gpr_phase_times   # noqa: E402


def main():
    eng = Engine.get()
    rng = np.random.default_rng(3)
    D, P = 5, 49
    for n in (53, 96, 160, 224, 288, 352, 416, 512, 768):
        X = rng.uniform(size=(n, D + 1))
        X[:, -1] = (np.arange(n) >= n - max(3, n // 16)).astype(float)
        Y = rng.normal(size=(n, P))
        Xd = torch.tensor(X, device=eng.device)
        Yd = torch.tensor(Y, device=eng.device)
        th = torch.tensor(np.concatenate([[1.0], np.full(D, 0.5), [0.3], np.full(D, 0.5), [1.2, 1e-3]]),
                          device=eng.device)
        res = {}
        for flow in (True, False):
            eng.set_flow(flow)
            for _ in range(3):
                gpr_phase_times(eng, Xd, Yd, th)
            t = np.mean([gpr_phase_times(eng, Xd, Yd, th) for _ in range(20)], axis=0)
            res[flow] = t
        eng.set_flow(True)
        print(f"n={n:4d} T={(n + 31) // 32:2d}  chol flow {res[True][2] * 1e3:7.1f} us  steps {res[False][2] * 1e3:7.1f} us"
              f"  | total flow {sum(res[True]) * 1e3:7.1f}  steps {sum(res[False]) * 1e3:7.1f}", flush=True)


if __name__ == "__main__":
    main()
