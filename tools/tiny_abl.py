"""Kernel-time ablation of k_gpr_tiny (diagnostic, GPU box): HBS LML value + gradient calls in a
loop, run under rocprofv3 with the variant libraries of tools/build_variants.py
(TINY_STOP = k: the kernel returns after phase k).
    MFGP_LIB_PATH=... rocprofv3 --kernel-trace --stats -- python tools/tiny_abl.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import HBS  # noqa: E402
from multi_fidelity_gpflow_amd.data import PowerSpecs, multifidelity_training_set  # noqa: E402
from multi_fidelity_gpflow_amd.engine import Engine  # noqa: E402

ps = PowerSpecs()
ps.read_from_txt(HBS)
X, Y, _, _ = multifidelity_training_set(ps)
eng = Engine.get()
D = X.shape[1] - 1
Xd, Yd = torch.tensor(X, device=eng.device), torch.tensor(Y, device=eng.device)
th = torch.tensor(np.concatenate([[1.0], np.ones(D), [1.0], np.ones(D), [1.0, 1e-3]]), device=eng.device)
for _ in range(200):
    eng.gpr_lml(Xd, Yd, th, want_grad=True)
torch.cuda.synchronize()
print("done")
