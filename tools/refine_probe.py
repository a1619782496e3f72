import sys, time, numpy as np, torch
sys.path.insert(0, '.')
import multi_fidelity_gpflow_amd as M
from multi_fidelity_gpflow_amd.data import synthetic_multifidelity
from multi_fidelity_gpflow_amd.engine import Engine
from oracle import mfgp_oracle as O
eng = Engine.get()
X, Y, Xt, _ = synthetic_multifidelity(2000, 300, 10, 130, 64, seed=1)
p0 = O.MFParams.initial(10, 130)
lo, _ = O.gpr_lml_and_grad(X, Y, p0)
mo, vo = O.gpr_predict_f(X, Y, Xt, p0)
d = X.shape[1] - 1
m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(d)), M.SquaredExponential(lengthscales=np.ones(d)), dtype="float32")
for r in (False, True):
    eng.set_f32_refine(r)
    lv = float(m.log_marginal_likelihood())
    mean, var = m.predict_f(Xt)
    print("refine", r, "lml", lv, "ref", lo, "rel", abs(lv - lo) / abs(lo), "mean rel", np.max(np.abs(mean.numpy() - mo)) / np.max(np.abs(mo)), flush=True)
# Synth size: cost of the refinement (value-only LML and predict, fp32), timed with events
Xs, Ys, Xts, _ = synthetic_multifidelity()
ms = M.MultiFidelityGPModel(Xs, Ys, M.SquaredExponential(lengthscales=np.ones(d)), M.SquaredExponential(lengthscales=np.ones(d)), dtype="float32")
for r in (False, True):
    eng.set_f32_refine(r)
    for what in ("lml", "predict"):
        f = (lambda: ms.log_marginal_likelihood()) if what == "lml" else (lambda: ms.predict_f(Xts))
        f(); torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        print(f"synth refine={r} {what}: {(time.perf_counter() - t0) / 3 * 1e3:.1f} ms", flush=True)
