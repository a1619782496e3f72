"""Times the fp32 Synth step (AdamSession, hipGraph replay, lookahead on) over panel widths and
reserved CUs.  Usage (GPU box): python tools/f32_sweep_knobs.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import multi_fidelity_gpflow_amd as M  # noqa: E402
from multi_fidelity_gpflow_amd.data import synthetic_multifidelity  # noqa: E402
from multi_fidelity_gpflow_amd.engine import Engine  # noqa: E402

torch.cuda.set_device(0)
eng = Engine.get()
X, Y, _, _ = synthetic_multifidelity()
d = X.shape[1] - 1
m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(d)),
                           M.SquaredExponential(lengthscales=np.ones(d)), dtype="float32")
for panel, rv in [(int(a), int(b)) for a, b in (x.split(":") for x in sys.argv[1:])] or \
        [(4, 32), (6, 32), (8, 32), (4, 48), (8, 48), (2, 32)]:
    eng.set_f32_panel(panel)
    eng.set_f32_reserve(rv)
    sess = m.adam_session(0.1, 8, graph=True, graph_chunk=2)
    sess.run(2)
    sess.prepare(4)
    sess.sync()
    t0 = time.time()
    sess.run(4)
    sess.sync()
    print(f"panel={panel} reserve={rv}: {(time.time() - t0) / 4 * 1e3:.1f} ms/step", flush=True)
