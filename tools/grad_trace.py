"""Phase timeline of k_grad's workgroups (diagnostic) from a trace build of the library
(tools/experiments/grad_trace.patch: s_memrealtime stamps at entry, after the m-loop, after the
epilogue's staging, after the per-entry partial sums, after the reduction, after the next
evaluation's sentinel refill):
  MFGP_LIB_PATH=ablibs/lib_kgrtrace.so python tools/grad_trace.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import multi_fidelity_gpflow_amd as M
    from multi_fidelity_gpflow_amd import _lib
    from multi_fidelity_gpflow_amd.engine import Engine
    from conftest import GOKU_DIR
    from oracle.mfgp_oracle import load_powerspecs
    g = load_powerspecs(GOKU_DIR)
    X, Y = g["X"], g["Y"]
    m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(10)),
                               M.SquaredExponential(lengthscales=np.ones(10)))
    eng = Engine.get()
    Xd = torch.tensor(X, device=eng.device)
    Yd = torch.tensor(Y, device=eng.device)
    th = torch.tensor(m._theta_map().theta(), dtype=torch.float64, device=eng.device)
    for _ in range(5):
        eng.gpr_lml(Xd, Yd, th, want_grad=True)
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = np.zeros((1024, 8), dtype=np.int64)
    assert lib.mfgp_debug_kgr_trace(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
    n = int((buf[:, 0] != 0).sum())
    t = buf[:n, :6].astype(np.float64) * 10e-3
    t -= t[:, 0].min()
    print(f"k_grad: {n} workgroups, span {t[:, 5].max():.1f} us; start quantiles",
          " ".join(f"{q:.1f}" for q in np.percentile(t[:, 0], [0, 25, 50, 75, 100])))
    for a, b, lab in ((0, 1, "m-loop (operand stream + MFMA)"), (1, 2, "epilogue staging + sync"),
                      (2, 3, "dK contraction + partials + sync"), (3, 4, "entry reduction"),
                      (4, 5, "next evaluation's sentinel refill")):
        v = t[:, b] - t[:, a]
        print(f"  {lab:36s} median {np.median(v):6.2f} us  p90 {np.percentile(v, 90):6.2f}  max {v.max():6.2f}")
    life = t[:, 5] - t[:, 0]
    print(f"  lifetime median {np.median(life):.2f} us, max {life.max():.2f}; last end {t[:, 5].max():.1f} us")


if __name__ == "__main__":
    main()
