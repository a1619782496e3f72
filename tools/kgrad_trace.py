"""Phase timeline of k_kgrad's workgroups from a trace build (diagnostic; the build adds
s_memrealtime stamps per wave and mfgp_debug_kg_trace, see tools/experiments/kgrad_trace.patch):
  MFGP_LIB_PATH=ablibs/lib_trace.so python tools/kgrad_trace.py"""
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
    from conftest import GOKU_DIR
    from oracle.mfgp_oracle import load_powerspecs
    g = load_powerspecs(GOKU_DIR)
    X, Y = g["X"], g["Y"]
    Zfix = np.load(os.path.join(ROOT, "tests", "golden", "goku_kmeans_z300.npy"))
    m = M.SingleBinSVGP(X, Y, M.SquaredExponential(lengthscales=np.ones(10)),
                        M.SquaredExponential(lengthscales=np.ones(10)), 64, Z=np.zeros((300, 11)))
    m.inducing_variable.assign(Zfix)
    for _ in range(3):
        m.elbo_and_grad((X, Y))
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = np.zeros((2, 4096, 4, 32), dtype=np.int64)
    assert lib.mfgp_debug_kg_trace(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
    seq, labels = [0, 1, 2], ["prologue: loads + sync", "prologue: Z rows, norms"]
    for c in range(4):
        kq = 3 + 6 * c
        seq += [kq + j for j in range(6)]
        labels += [f"c{c - 1} pairs (LF + HF)" if c else "-", f"c{c} barrier 1", f"c{c} X rows -> LDS",
                   f"c{c} barrier 2", f"c{c} B operand + norms", f"c{c} barrier 3"]
    seq += [27, 28]
    labels += ["c3 pairs (LF + HF)", "epilogue"]
    for k, name, nwg in ((0, "Kuf", 3200), (1, "Kuu", 1280)):
        t = buf[k, :nwg].astype(np.float64) * 10e-3   # 100 MHz ticks -> us
        t -= t[:, :, 0].min()
        start, end = t[:, :, 0].min(1), t[:, :, 28].max(1)
        print(f"== {name}: {nwg} workgroups, kernel span {end.max():.1f} us, workgroup lifetime "
              f"median {np.median(end - start):.1f} us")
        for i in range(1, len(seq)):
            v = t[:, :, seq[i]] - t[:, :, seq[i - 1]]
            lab = labels[i - 1]
            print(f"   {lab:22s} median {np.median(v):6.2f} us  wave-0 median {np.median(v[:, 0]):6.2f}  "
                  f"p90 {np.percentile(v, 90):6.2f}")


if __name__ == "__main__":
    main()
