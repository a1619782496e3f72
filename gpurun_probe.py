import sys, time, numpy as np, torch
sys.path.insert(0, '.')
from oracle import mfgp_oracle as O
import multi_fidelity_gpflow_amd as M
from multi_fidelity_gpflow_amd.engine import Engine
eng = Engine.get()
print("mfma selftest:\n", eng.selftest_mfma()[:4, :6])
A = np.arange(16)[:, None] * 4 + np.arange(4)[None, :] + 1.0
B = 100.0 * np.arange(4)[:, None] + np.arange(16)[None, :]
print("expected:\n", (A @ B)[:4, :6], "\nmaxdiff", np.abs(eng.selftest_mfma() - A @ B).max())
for nb in (32, 64):
    eng.set_tile(nb)
    for name in ["50_LR_3_HR", "matter_power_1128_Box1000_Part750_36_Box1000_Part3000_z0"]:
        d = O.load_powerspecs("tests/golden/data/" + name)
        X, Y = d["X"], d["Y"]
        D = X.shape[1] - 1
        p = O.MFParams.initial(D, Y.shape[1])
        p.vL, p.rho = 1.3, np.full((Y.shape[1], 1), 0.8); p.lL = np.linspace(0.5, 2, D)
        m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(D)), M.SquaredExponential(lengthscales=np.ones(D)))
        m.kernel.kernel_L.variance.assign(p.vL); m.kernel.kernel_L.lengthscales.assign(p.lL); m.kernel.rho.assign(p.rho)
        K = m.kernel.K(X).numpy(); Ko = O.mf_K(X, None, p)
        print(nb, name, "gram maxabs", np.abs(K - Ko).max())
        Kd = m.kernel.K_diag(X).numpy(); print("  kdiag", np.abs(Kd - O.mf_Kdiag(X, p)).max())
        Kc = O.mf_K(X, None, p) + p.noise * np.eye(len(X))
        Linv, ld, info = eng.potrf_inv(torch.tensor(Kc, device='cuda'))
        Lo = np.linalg.cholesky(Kc); print("  potrf_inv info", info.item(), "Linv err", np.abs(Linv.cpu().numpy() @ Lo - np.eye(len(X))).max(), "ldiag", np.abs(ld.cpu().numpy() - np.diag(Lo)).max())
        t = time.time(); l = float(m.log_marginal_likelihood()); 
        lo, go = O.gpr_lml_and_grad(X, Y, p)
        print("  lml", l, lo, (l - lo) / abs(lo))
        l2, g = m.log_marginal_likelihood_and_grad()
        gov = np.concatenate([[go['vL']], go['lL'], [go['vD']], go['lD'], [go['rho0']], [go['noise']]])
        print("  grad relerr", np.max(np.abs(g - gov) / (np.abs(gov) + 1e-8)))
        mean, var = m.predict_f(d["Xtest"]); mo, vo = O.gpr_predict_f(X, Y, d["Xtest"], p)
        print("  pred mean err", np.abs(mean.numpy() - mo).max(), "var err", np.abs(var.numpy() - vo).max())
        torch.cuda.synchronize(); t = time.time()
        for _ in range(20): out, info = eng.gpr_lml(*m._device_data()[1:], torch.tensor(m._theta_map().theta(), device='cuda'), True)
        torch.cuda.synchronize(); print("  value+grad ms (eager)", (time.time() - t) / 20 * 1e3)
eng.set_tile(32)
d = O.load_powerspecs("tests/golden/data/50_LR_3_HR")
m = M.MultiFidelityGPModel(d["X"], d["Y"], M.SquaredExponential(lengthscales=np.ones(5)), M.SquaredExponential(lengthscales=np.ones(5)))
t = time.time(); m.optimize(max_iters=1000, learning_rate=0.1); torch.cuda.synchronize(); print("HBS 1000 adam s", time.time() - t)
kat = {100:5108.897743849085, 500:5254.116876204594, 900:5292.602815722793}
for k, v in kat.items(): print(k, -m.loss_history[k], (-m.loss_history[k] - v) / v)
d = O.load_powerspecs("tests/golden/data/matter_power_1128_Box1000_Part750_36_Box1000_Part3000_z0")
m = M.MultiFidelityGPModel(d["X"], d["Y"], M.SquaredExponential(lengthscales=np.ones(10)), M.SquaredExponential(lengthscales=np.ones(10)))
t = time.time(); m.optimize(max_iters=1000, learning_rate=0.1); torch.cuda.synchronize(); print("Goku 1000 adam s", time.time() - t)
kat = {0: 95216.01782973186, 100:139100.27740368416, 500:142611.01593941066, 900:143468.40684723994}
for k, v in kat.items(): print(k, -m.loss_history[k], (-m.loss_history[k] - v) / v)
t = time.time(); m.optimize(max_iters=1000, learning_rate=0.1, verbose=False); torch.cuda.synchronize(); print("Goku 1000 adam s (warm)", time.time() - t)
