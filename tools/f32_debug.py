"""Debug probe of the fp32 diagonal-block factor: one 128 x 128 tile (n = 128, p = 1), workspace
inspected against numpy (L = chol(K + s2 I), D = L^-1, ldiag)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from multi_fidelity_gpflow_amd.data import synthetic_multifidelity  # noqa: E402
from multi_fidelity_gpflow_amd.engine import Engine  # noqa: E402
from oracle import mfgp_oracle as O  # noqa: E402

torch.cuda.set_device(0)
eng = Engine.get()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
X, Y, _, _ = synthetic_multifidelity(n - n // 4, n // 4, 10, 1, 8, seed=1)
Xd = torch.tensor(X, dtype=torch.float32, device=eng.device)
Yd = torch.tensor(Y, dtype=torch.float32, device=eng.device)
p0 = O.MFParams.initial(10, 1)
theta = torch.tensor(np.concatenate([[1.0], np.ones(10), [1.0], np.ones(10), [1.0], [1e-3]]), dtype=torch.float64,
                     device=eng.device)
nb = eng.gpr_workspace_bytes(n, 1, 10, torch.float32)
ws = torch.zeros(nb, dtype=torch.uint8, device=eng.device)
out, info = eng.gpr_lml(Xd, Yd, theta, want_grad=False, ws=ws)
torch.cuda.synchronize()
print("info", info.item(), "lml", out[0].item(), "oracle", O.gpr_lml(X, Y, p0))
T = -(-n // 128)
npad = 128 * T
rows = (T + 1) * 128   # want_grad=0: A + Y^T rows
Mbytes = rows * npad * 4
M = ws[:Mbytes].view(torch.float32).reshape(rows, npad).cpu().numpy()
off = (Mbytes + 255) // 256 * 256
Dd = ws[off:off + T * 128 * 128 * 4].view(torch.float32).reshape(T, 128, 128).cpu().numpy()
off2 = (off + T * 128 * 128 * 4 + 255) // 256 * 256
ld = ws[off2:off2 + npad * 8].view(torch.float64).cpu().numpy()
K = O.mf_K(X, None, p0)
K[np.diag_indices_from(K)] += 1e-3
Kp = np.eye(npad)
Kp[:n, :n] = K
L = np.linalg.cholesky(Kp)
D0 = np.linalg.inv(L[:128, :128])
Lg = np.tril(M[:128, :128])
print("ldiag err", np.max(np.abs(ld[:128] - np.diag(L)[:128])), "ldiag[:8]", ld[:8], "ref", np.diag(L)[:8])
print("L00 err", np.max(np.abs(Lg - L[:128, :128])))
print("D0 err", np.max(np.abs(Dd[0] - D0)), "D0 upper max", np.max(np.abs(np.triu(Dd[0], 1))))
for s in range(4):
    for t in range(s + 1):
        e = np.max(np.abs(Lg[32 * s:32 * s + 32, 32 * t:32 * t + 32] - L[32 * s:32 * s + 32, 32 * t:32 * t + 32]))
        f = np.max(np.abs(Dd[0][32 * s:32 * s + 32, 32 * t:32 * t + 32] - D0[32 * s:32 * s + 32, 32 * t:32 * t + 32]))
        print(f"block ({s},{t}) L err {e:.2e} D err {f:.2e}")
