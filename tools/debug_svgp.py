import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import multi_fidelity_gpflow_amd as M
from oracle.mfgp_oracle import load_powerspecs
from oracle import svgp_oracle as S
import test_gpu_svgp as T
d = load_powerspecs('tests/golden/data/50_LR_3_HR')
X, Y = d['X'], d['Y']
m = M.SingleBinSVGP(X, Y, M.SquaredExponential(lengthscales=np.ones(5)), M.SquaredExponential(lengthscales=np.ones(5)), 49, Z=np.zeros((50, 6)))
e, gd = m.elbo_and_grad((X, Y))
eo, ga = T._autograd_grads(m, X, Y)
print("elbo gpu", e, "oracle", eo)
for k in ga:
    ref = ga[k]; got = np.asarray(gd[k]).reshape(ref.shape)
    print(k, "max|ref|", np.abs(ref).max(), "rel err", np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))
tr = M.svgp._SVGPTrainer(m, (X, Y), max_iters=2000, initial_lr=0.1, graph=False)
tr.run(1); tr.grad(); tr.sync()
print("gpu after 1 step", -float(tr.out[0].item()), "loss_hist[0]", float(tr.loss_hist[0].item()))
Z = __import__('sklearn.cluster', fromlist=['KMeans']).KMeans(n_clusters=50, random_state=42).fit(X).cluster_centers_
ot = S.SingleBinTrainer(X, Y, Z, lr=0.1, max_iters=2000)
l0 = ot.step(); print("oracle loss0", l0, "after 1 step", float(ot.neg_elbo().detach()))
print("step", int(tr.step_t.item()), "lr[0]", float(tr.lr[0].item()), "n trainable", int(tr.trainable.sum().item()), "of", tr.n)
