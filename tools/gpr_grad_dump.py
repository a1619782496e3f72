"""Dump GPR LML value + gradient outputs (Goku and HBS at a few theta, every schedule the handle
offers: flow / steps / tiny) to an .npz, for bitwise A/B of library builds:
  MFGP_LIB_PATH=<lib> python tools/gpr_grad_dump.py OUT.npz ;  python tools/gpr_grad_dump.py --compare A B"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def dump(out):
    import torch
    from multi_fidelity_gpflow_amd.engine import Engine
    from conftest import GOKU_DIR, HBS_DIR
    from oracle.mfgp_oracle import load_powerspecs
    eng = Engine.get()
    res = {}
    rng = np.random.default_rng(3)
    for name, dd in (("goku", GOKU_DIR), ("hbs", HBS_DIR)):
        g = load_powerspecs(dd)
        X = torch.tensor(g["X"], device=eng.device)
        Y = torch.tensor(g["Y"], device=eng.device)
        d = X.shape[1] - 1
        for s in range(3):
            th = np.concatenate([[0.5 + rng.random()], 0.5 + rng.random(d), [0.1 + rng.random()], 0.5 + rng.random(d),
                                 [0.5 + rng.random()], [1e-3]])
            t = torch.tensor(th, dtype=torch.float64, device=eng.device)
            for flow in (True, False):
                eng.set_flow(flow)
                o, info = eng.gpr_lml(X, Y, t, want_grad=True)
                torch.cuda.synchronize()
                res[f"{name}_{s}_{'flow' if flow else 'steps'}"] = o.cpu().numpy().copy()
        eng.set_flow(True)
    np.savez(out, **res)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        A, B = np.load(sys.argv[2]), np.load(sys.argv[3])
        bad = 0
        for k in A.files:
            same = np.array_equal(A[k], B[k])
            d = float(np.abs(A[k] - B[k]).max() / max(np.abs(A[k]).max(), 1e-300))
            print(f"{k:18s} {'bitwise' if same else 'DIFF'} rel {d:.1e}")
            bad += not same
        print("all bitwise equal" if not bad else f"{bad} arrays differ")
    else:
        dump(sys.argv[1])
