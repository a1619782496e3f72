"""Synth-size fp32 value-only LML and predict with and without the fp64 refinement (for rocprof).
    python tools/refine_synth.py [reps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multi_fidelity_gpflow_amd as M                               # noqa: E402
from multi_fidelity_gpflow_amd.data import synthetic_multifidelity  # noqa: E402
from multi_fidelity_gpflow_amd.engine import Engine                 # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
eng = Engine.get()
X, Y, Xt, _ = synthetic_multifidelity()
d = X.shape[1] - 1
m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(d)),
                           M.SquaredExponential(lengthscales=np.ones(d)), dtype="float32")
for r in (False, True):
    eng.set_f32_refine(r)
    for what in ("lml", "predict"):
        f = (lambda: m.log_marginal_likelihood()) if what == "lml" else (lambda: m.predict_f(Xt))
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        print(f"synth refine={r} {what}: {(time.perf_counter() - t0) / reps * 1e3:.1f} ms", flush=True)
