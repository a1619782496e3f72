"""Timeline of the flow set-up launch (k_gram_flow) at Goku: per-role start / work done / end
relative to the earliest workgroup start (us).  Diagnostic only (GPU box):
    python tools/gram_trace.py [reps]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multi_fidelity_gpflow_amd import _lib                       # noqa: E402
from multi_fidelity_gpflow_amd.engine import Engine             # noqa: E402
from oracle import mfgp_oracle as O                             # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    d = O.load_powerspecs(os.path.join(ROOT, "tests", "golden", "data",
                                       "matter_power_1128_Box1000_Part750_36_Box1000_Part3000_z0"))
    X, Y = d["X"], d["Y"]
    eng = Engine.get()
    lib = eng.lib
    _lib.check(lib.mfgp_set_flow(eng.h, 2), "mfgp_set_flow")
    n, p, D = X.shape[0], Y.shape[1], X.shape[1] - 1
    Xd = torch.tensor(X, device=eng.device)
    Yd = torch.tensor(Y, device=eng.device)
    th = torch.tensor(np.concatenate([[1.0], np.ones(D), [1.0], np.ones(D), [1.0, 1e-3]]), device=eng.device)
    off, cnt = C.c_size_t(), C.c_int()
    _lib.check(lib.mfgp_gpr_flow_trace(eng.h, n, p, D, C.byref(off), C.byref(cnt)), "trace")
    T = (n + 31) // 32
    nb = (T * 32 + 63) // 64
    nblk = nb * (nb + 1) // 2
    for r in range(reps):
        eng.gpr_lml(Xd, Yd, th, want_grad=True)
        torch.cuda.synchronize()
        ws = eng._ws["gpr"]
        g = ws[off.value + 8 * (cnt.value - 5 * (T * (T + 1) // 2 + 4)): off.value + 8 * cnt.value].view(torch.int64).cpu().numpy()
        grid = nblk + 3
        h = g[3 * grid: 3 * grid + 2 * (nblk + 1)].reshape(-1, 2).astype(np.float64)   # [unused, staged]
        g = g[:3 * (T * (T + 1) // 2 + 4)].reshape(-1, 3)[:nblk + 3].astype(np.float64)
        z = g[:, 0].min()
        g = (g - z) / 100.0
        h = (h - z) / 100.0
        print(f"        blocks staged med {np.median(h[1:nblk + 1, 1]):.2f} max {h[1:nblk + 1, 1].max():.2f};"
              f" factor staged {h[0, 1]:.2f}")
        fa, b = g[0], g[1:nblk + 1]
        print(f"rep {r}: blocks start med {np.median(b[:, 0]):.2f} max {b[:, 0].max():.2f} | entries med "
              f"{np.median(b[:, 1]):.2f} max {b[:, 1].max():.2f} | end med {np.median(b[:, 2]):.2f} max {b[:, 2].max():.2f}")
        for k, name in ((0, "factor"), (nblk + 1, "owner"), (nblk + 2, "order")):
            print(f"        {name:6s} start {g[k, 0]:.2f} work-done {g[k, 1]:.2f} end {g[k, 2]:.2f}")


if __name__ == "__main__":
    main()
