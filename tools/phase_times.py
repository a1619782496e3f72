"""Per-phase device times of one Goku LML value+grad evaluation (hipEvents on the launch stream).
Diagnostic: python tools/phase_times.py [reps]  (MFGP_LIB_PATH selects a variant build)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multi_fidelity_gpflow_amd.engine import Engine, gpr_phase_times   # noqa: E402
from oracle import mfgp_oracle as O                                    # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
d = O.load_powerspecs(os.path.join(ROOT, "tests", "golden", "data",
                                   "matter_power_1128_Box1000_Part750_36_Box1000_Part3000_z0"))
eng = Engine.get()
X = torch.tensor(d["X"], device=eng.device)
Y = torch.tensor(d["Y"], device=eng.device)
D = d["X"].shape[1] - 1
th = torch.tensor(np.concatenate([[1.0], np.ones(D), [1.0], np.ones(D), [1.0, 1e-3]]), device=eng.device)
gpr_phase_times(eng, X, Y, th)
acc = np.zeros(5)
for _ in range(reps):
    acc += np.array(gpr_phase_times(eng, X, Y, th))
print(os.environ.get("MFGP_LIB_PATH", "default"), " ".join(f"{n}={v * 1e3 / reps:.1f}us" for n, v in
      zip(["pre", "gram", "chol", "grad", "fin"], acc)))
