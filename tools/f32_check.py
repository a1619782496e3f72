"""Exploratory check of the fp32 path (mfgp_*_ex with MFGP_F32): accuracy against the fp64
oracle at small sizes, against the fp64 HIP path at the Synth size, and per-phase timings.
Usage (GPU box): python tools/f32_check.py [--full]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import multi_fidelity_gpflow_amd as M  # noqa: E402
from multi_fidelity_gpflow_amd.data import synthetic_multifidelity  # noqa: E402
from multi_fidelity_gpflow_amd.engine import Engine, gpr_phase_times_ex  # noqa: E402
from oracle import mfgp_oracle as O  # noqa: E402


def model(X, Y, dtype):
    d = X.shape[1] - 1
    return M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(d)),
                                  M.SquaredExponential(lengthscales=np.ones(d)), dtype=dtype)


def small(n_lf, n_hf, p, panel):
    eng = Engine.get()
    eng.set_f32_panel(panel)
    X, Y, Xt, _ = synthetic_multifidelity(n_lf, n_hf, 10, p, 64, seed=1)
    m32 = model(X, Y, "float32")
    l32, g32 = m32.log_marginal_likelihood_and_grad()
    p0 = O.MFParams.initial(10, p)
    lo, go = O.gpr_lml_and_grad(X, Y, p0)
    gov = np.concatenate([[go["vL"]], go["lL"], [go["vD"]], go["lD"], [go["rho0"]], [go["noise"]]])
    mu32, v32 = m32.predict_f(Xt)
    mo, vo = O.gpr_predict_f(X, Y, Xt, p0)
    print(f"small n={X.shape[0]} p={p} panel={panel}: LML f32 {l32:.6f} oracle {lo:.6f} rel {abs(l32-lo)/abs(lo):.2e}; "
          f"grad maxrel {np.max(np.abs(g32-gov))/np.max(np.abs(gov)):.2e}; "
          f"mean maxabs {np.max(np.abs(mu32.numpy()-mo)):.2e} (|mean| {np.max(np.abs(mo)):.2e}); "
          f"var maxabs {np.max(np.abs(v32.numpy()[:, 0]-vo[:, 0])):.2e}", flush=True)


def full():
    eng = Engine.get()
    eng.set_f32_panel(4)
    X, Y, Xt, _ = synthetic_multifidelity()
    t0 = time.time()
    m32 = model(X, Y, "float32")
    l32, g32 = m32.log_marginal_likelihood_and_grad()
    torch.cuda.synchronize()
    print(f"full f32 first call {time.time()-t0:.2f}s LML {l32:.6f}", flush=True)
    eng32, X32, Y32 = m32._device_data()
    theta = torch.tensor(m32._theta_map().theta(), dtype=torch.float64, device=eng.device)
    for _ in range(2):
        ph = gpr_phase_times_ex(eng, X32, Y32, theta)
    tot = sum(v[0] for v in ph.values())
    print("phases (ms, TF/s, launches):", {k: (round(v[0], 3), round(v[1] / (v[0] * 1e-3) / 1e12, 2) if v[0] else 0,
                                              v[2]) for k, v in ph.items()}, f"total {tot:.2f} ms", flush=True)
    for la in (0, 1):
        eng.set_f32_lookahead(bool(la))
        m32.log_marginal_likelihood_and_grad()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(3):
            lx, gx = m32.log_marginal_likelihood_and_grad()
        torch.cuda.synchronize()
        print(f"lookahead={la}: f32 value+grad {(time.time()-t0)/3*1e3:.1f} ms/eval (host-synced), LML {lx:.6f} "
              f"same-as-serial {lx == l32 and np.array_equal(gx, g32)}", flush=True)
    for graph, la, rv in ((False, 0, 0), (True, 0, 0), (True, 1, 0), (True, 1, 8), (True, 1, 16), (True, 1, 32)):
        eng.set_f32_lookahead(bool(la))
        eng.set_f32_reserve(rv)
        sess = m32.adam_session(0.1, 8, graph=graph, graph_chunk=2)
        sess.run(2)
        sess.prepare(4)
        sess.sync()
        t0 = time.time()
        sess.run(4)
        sess.sync()
        print(f"adam session graph={graph} lookahead={la} reserve={rv}: {(time.time()-t0)/4*1e3:.1f} ms/step",
              flush=True)
    eng.set_f32_lookahead(True)
    # additivity over output columns
    la, _ = model(X, Y[:, :256], "float32").log_marginal_likelihood_and_grad()
    lb, _ = model(X, Y[:, 256:], "float32").log_marginal_likelihood_and_grad()
    print(f"additivity: {l32:.6f} vs {la+lb:.6f} rel {abs(l32-la-lb)/abs(l32):.2e}", flush=True)
    if "--f64" in sys.argv:
        t0 = time.time()
        m64 = model(X, Y, None)
        l64, g64 = m64.log_marginal_likelihood_and_grad()
        torch.cuda.synchronize()
        print(f"f64 HIP path {time.time()-t0:.2f}s LML {l64:.6f}; f32 rel {abs(l32-l64)/abs(l64):.2e}; "
              f"grad maxrel {np.max(np.abs(g32-g64))/np.max(np.abs(g64)):.2e}", flush=True)
        print("g32", np.array2string(g32, precision=4), "\ng64", np.array2string(g64, precision=4), flush=True)


if __name__ == "__main__":
    torch.cuda.set_device(0)
    for (nl, nh, p) in ((200, 50, 3), (500, 100, 20)):
        for panel in (1, 4):
            small(nl, nh, p, panel)
    small(2000, 300, 130, 2)
    if "--full" in sys.argv:
        full()
