"""GraphMultiFidelityKernel / GraphMultiFidelityGPModel (mfgpflow/graph.py)
on the HIP path vs. the torch-CPU restatement oracle/graph_oracle.py.

Parity is UNPINNED by reference outputs (the reference has no graph-model test or recorded
value); the oracle restates graph.py line by line, including its asymmetric LF-LF block
(rho_LF[i, j] k_i) and the 1e-6 jitter inside K.  Tolerances: K entries 1e-13 abs; LML
1e-11 rel; gradient 1e-8 rel of the largest component; Adam trajectory 1e-9 rel."""
import numpy as np
import pytest
import torch

import multi_fidelity_gpflow_amd as M
from oracle import graph_oracle as GO

pytestmark = pytest.mark.gpu


def _data(m=2, D=3, P=4, sizes=(40, 30, 12), seed=3):
    rng = np.random.default_rng(seed)
    Xs, Ys = [], []
    w = rng.standard_normal((D, P))
    for s, n in enumerate(sizes[:m + 1]):
        x = rng.uniform(0, 1, (n, D))
        y = np.sin(3 * x @ w) * (1 + 0.3 * s) + 0.05 * rng.standard_normal((n, P))
        Xs.append(np.hstack([x, np.full((n, 1), float(s))]))
        Ys.append(y)
    return np.vstack(Xs), np.vstack(Ys)


def _model(X, Y, m, D, asym=True, seed=5):
    """Valid (PD) parameters: the graph kernel's LF-LF block is rho_LF (x) k only when the LF
    sources share k (graph.py uses the row source's kernel); rho_LF's upper triangle is
    free (the factorization reads the lower one) and is set asymmetric to exercise the
    entry-by-entry gradient."""
    rng = np.random.default_rng(seed)
    lsh, vsh = 0.5 + rng.random(D), 0.5 + rng.random()
    kLs = [M.SquaredExponential(lengthscales=lsh.copy(), variance=vsh) for _ in range(m)]
    kd = M.SquaredExponential(lengthscales=0.5 + rng.random(D), variance=0.2 + 0.3 * rng.random())
    mod = M.GraphMultiFidelityGPModel(X, Y, kLs, kd)
    mod.kernel.rho.assign(0.6 + rng.random((m, Y.shape[1])))
    if asym:
        r = 0.2 + 0.3 * rng.random((m, m))
        mod.kernel.rho_LF.assign(r)
    return mod


def _oracle_params(mod, D):
    k = mod.kernel
    ks = k.kernel_Ls + [k.kernel_delta]
    f64 = dict(dtype=torch.float64)
    return dict(v=torch.tensor([float(kk.variance.numpy()) for kk in ks], **f64),
                l=torch.tensor(np.stack([kk.lengthscale_vector(D) for kk in ks]), **f64),
                rho=torch.tensor(k.rho.numpy()[:, 0], **f64), rhoLF=torch.tensor(k.rho_LF.numpy(), **f64))


@pytest.mark.parametrize("m,asym", [(1, False), (2, True), (3, True)])
def test_graph_K_and_Kdiag(m, asym):
    D = 3
    X, Y = _data(m, D)
    mod = _model(X, Y, m, D, asym)
    prm = _oracle_params(mod, D)
    Xt = torch.tensor(X)
    np.testing.assert_allclose(mod.kernel.K(X).numpy(), GO.graph_K(Xt, Xt, prm).numpy(), rtol=0, atol=1e-13)
    np.testing.assert_allclose(mod.kernel.K_diag(X).numpy(), GO.graph_Kdiag(Xt, prm).numpy(), rtol=0, atol=1e-14)
    with pytest.raises(ValueError):
        mod.kernel.K(X, X[:5])


@pytest.mark.parametrize("m,asym", [(1, False), (2, True), (3, True)])
def test_graph_lml_and_grad(m, asym):
    D = 3
    X, Y = _data(m, D)
    mod = _model(X, Y, m, D, asym)
    lml, g = mod.log_marginal_likelihood_and_grad()
    prm = _oracle_params(mod, D)
    for v in prm.values():
        v.requires_grad_(True)
    noise = torch.tensor(1e-3, dtype=torch.float64, requires_grad=True)
    lo = GO.lml(torch.tensor(X), torch.tensor(Y), prm, noise)
    lo.backward()
    assert abs(lml - float(lo)) < 1e-11 * abs(float(lo))
    grl = prm["rhoLF"].grad.numpy().ravel() if prm["rhoLF"].grad is not None else np.zeros(m * m)
    go = np.concatenate([np.concatenate([[prm["v"].grad[s]], prm["l"].grad[s].numpy()]) for s in range(m + 1)]
                        + [prm["rho"].grad.numpy(), grl, [noise.grad]])
    np.testing.assert_allclose(g, go, rtol=0, atol=1e-8 * np.abs(go).max())


def test_graph_adam_matches_oracle():
    m, D = 2, 3
    X, Y = _data(m, D)
    mod = _model(X, Y, m, D, asym=True)
    k = mod.kernel
    init = dict(v=[float(kk.variance.numpy()) for kk in k.kernel_Ls + [k.kernel_delta]],
                l=np.stack([kk.lengthscales.numpy() for kk in k.kernel_Ls + [k.kernel_delta]]),
                rho=k.rho.numpy(), rhoLF=k.rho_LF.numpy())
    tr = GO.GraphTrainer(X, Y, m, D, lr=0.01, init=init)
    ref = [tr.step() for _ in range(20)]
    mod.optimize(max_iters=20, learning_rate=0.01, use_adam=True, graph=True, graph_chunk=10)
    np.testing.assert_allclose(mod.loss_history, ref, rtol=1e-9)
    prm = tr.params()
    np.testing.assert_allclose(k.rho_LF.numpy()[~np.eye(m, dtype=bool)],
                               prm["rhoLF"].detach().numpy()[~np.eye(m, dtype=bool)], rtol=1e-8)


def test_graph_predict_and_lbfgs():
    m, D = 2, 3
    X, Y = _data(m, D)
    Xs = np.hstack([np.random.default_rng(9).uniform(0, 1, (7, D)), np.full((7, 1), float(m))])
    mod = _model(X, Y, m, D, asym=True)
    mean, var = mod.predict_f(Xs)
    mo, vo = GO.predict_f(torch.tensor(X), torch.tensor(Y), torch.tensor(Xs), _oracle_params(mod, D),
                          torch.tensor(1e-3, dtype=torch.float64))
    np.testing.assert_allclose(mean.numpy(), mo.numpy(), rtol=0, atol=1e-9 * max(1.0, np.abs(mo.numpy()).max()))
    np.testing.assert_allclose(var.numpy()[:, 0], vo.numpy(), rtol=0, atol=1e-9)
    # L-BFGS (graph.py:176-188) with one LF source: the graph K stays a valid covariance for
    # any parameters (with m >= 2 sources L-BFGS can step into rho_LF / kernel combinations
    # whose lower triangle is not PD, where the reference's Cholesky raises as well).
    X1, Y1 = _data(1, D)
    mod1 = _model(X1, Y1, 1, D, asym=False)
    l0 = float(mod1.training_loss())
    mod1.optimize(max_iters=30, use_adam=False)
    assert float(mod1.training_loss()) < l0 and np.isfinite(mod1.loss_history).all()
