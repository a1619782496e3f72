"""HIP path (libmfgp.so through the C-ABI) vs. the CPU oracle and the reference KATs.

Tolerances (fp64): Gram entries 1e-13 abs; LML 1e-11 rel; gradient 1e-8 rel (of the
largest component); posterior mean/var 1e-9 abs; Adam trajectories 1e-10 rel through
iteration 500 (the reference dynamics turn chaotic after ~520).  The north-star bar is
1e-5 relative for posteriors."""
import numpy as np
import pytest
import torch

import multi_fidelity_gpflow_amd as M
from multi_fidelity_gpflow_amd.engine import Engine
from oracle import mfgp_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from multi_fidelity_gpflow_amd.build import build_lib
    build_lib()
    e = Engine.get()
    yield e
    e.set_tile(32)


@pytest.fixture(params=[(32, True, False), (32, False, False), (64, False, False), (32, False, True)],
                ids=["nb32-flow", "nb32-steps", "nb64", "nb32-tiny"])
def tile(request, eng):
    """Tile size and LML schedule: the persistent dataflow launch (k_chol_flow, NB = 32), the
    launch-per-step sequence (k_chol_step), or the one-launch small-problem kernel (k_gpr_tiny:
    n, p <= 64 -- HBS, Forrester; larger problems take the step sequence under this id)."""
    nb, flow, tiny = request.param
    eng.set_tile(nb)
    eng.set_flow(flow, any_size=True)   # the flow even below its default size threshold
    eng.set_tiny(tiny)
    yield nb
    eng.set_tile(32)
    eng.set_flow(True)
    eng.set_tiny(True)   # the library default


def _params(D, P, seed=0, scale=1.0):
    rng = np.random.default_rng(seed)
    return O.MFParams(1.0 + 0.5 * rng.random() * scale, 0.5 + 1.5 * rng.random(D) * scale, 0.3 + rng.random() * scale,
                      0.5 + rng.random(D) * scale, np.full((P, 1), 0.7 + 0.6 * rng.random() * scale), 1e-3)


def _model(X, Y, p: O.MFParams):
    D = X.shape[1] - 1
    m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(D)),
                               M.SquaredExponential(lengthscales=np.ones(D)))
    m.kernel.kernel_L.variance.assign(p.vL)
    m.kernel.kernel_L.lengthscales.assign(p.lL)
    m.kernel.kernel_delta.variance.assign(p.vD)
    m.kernel.kernel_delta.lengthscales.assign(p.lD)
    m.kernel.rho.assign(p.rho)
    m.likelihood.variance.assign(p.noise)
    return m


def _oracle_params(m) -> O.MFParams:
    k = m.kernel
    D = m.input_dim
    return O.MFParams(float(k.kernel_L.variance.numpy()), k.kernel_L.lengthscale_vector(D),
                      float(k.kernel_delta.variance.numpy()), k.kernel_delta.lengthscale_vector(D),
                      k.rho.numpy(), float(m.likelihood.variance.numpy()))


def test_mfma_f64_layout(eng):
    A = np.arange(16)[:, None] * 4 + np.arange(4)[None, :] + 1.0
    B = 100.0 * np.arange(4)[:, None] + np.arange(16)[None, :]
    np.testing.assert_array_equal(eng.selftest_mfma(), A @ B)


@pytest.mark.parametrize("which", ["hbs", "goku"])
def test_mf_gram(which, tile, hbs, goku):
    d = hbs if which == "hbs" else goku
    X = d["X"]
    p = _params(X.shape[1] - 1, d["Y"].shape[1], seed=1)
    m = _model(X, d["Y"], p)
    np.testing.assert_allclose(m.kernel.K(X).numpy(), O.mf_K(X, None, p), rtol=0, atol=1e-13)
    # rectangular, mixed fidelities on both sides, LF+HF test rows
    X2 = np.vstack([d["Xtest"], np.hstack([d["Xtest"][:, :-1], np.zeros((len(d["Xtest"]), 1))])])
    np.testing.assert_allclose(m.kernel.K(X, X2).numpy(), O.mf_K(X, X2, p), rtol=0, atol=1e-13)
    np.testing.assert_allclose(m.kernel.K_diag(X2).numpy(), O.mf_Kdiag(X2, p), rtol=0, atol=1e-15)


def test_fractional_fidelity_rows_are_zero(eng, hbs):
    """linear.py:67-70 exact masks: a KMeans centre with fidelity 0.9999999999999999 gets a zero row."""
    X = hbs["X"][:20].copy()
    X[3, -1] = 0.9999999999999999
    X[7, -1] = 0.5
    p = _params(5, 1, seed=2)
    m = _model(X, np.zeros((20, 1)), p)
    K = m.kernel.K(X).numpy()
    np.testing.assert_array_equal(K[3], 0.0)
    np.testing.assert_array_equal(K[:, 7], 0.0)
    np.testing.assert_allclose(K, O.mf_K(X, None, p), rtol=0, atol=1e-14)
    assert m.kernel.K_diag(X).numpy()[3] == 0.0


def test_rbf_gram(eng):
    rng = np.random.default_rng(3)
    A, B = rng.random((70, 4)), rng.random((33, 4))
    k = M.SquaredExponential(variance=1.7, lengthscales=np.array([0.3, 0.8, 1.1, 2.0]))
    np.testing.assert_allclose(k.K(A, B).numpy(), O.rbf_K(A, B, 1.7, [0.3, 0.8, 1.1, 2.0]), rtol=0, atol=1e-14)
    k2 = M.SquaredExponential(variance=0.5, lengthscales=0.7)       # isotropic
    np.testing.assert_allclose(k2(A).numpy(), O.rbf_K(A, A, 0.5, 0.7), rtol=0, atol=1e-14)
    np.testing.assert_allclose(k2(A, full_cov=False).numpy(), np.full(70, 0.5))


@pytest.mark.parametrize("n,batch", [(1, 1), (5, 2), (32, 1), (33, 3), (64, 1), (65, 2), (300, 2)])
def test_potrf_inv(n, batch, tile, eng):
    rng = np.random.default_rng(n)
    G = rng.standard_normal((batch, n, n))
    A = G @ G.transpose(0, 2, 1) / n + np.eye(n) * 0.5
    Linv, ld, info = eng.potrf_inv(torch.tensor(A, device=eng.device))
    assert info.cpu().numpy().tolist() == [0] * batch
    for b in range(batch):
        L = np.linalg.cholesky(A[b])
        np.testing.assert_allclose(Linv[b].cpu().numpy() @ L, np.eye(n), atol=1e-11)
        np.testing.assert_allclose(ld[b].cpu().numpy(), np.diag(L), rtol=1e-13)
        assert np.all(np.triu(Linv[b].cpu().numpy(), 1) == 0)


def test_non_pd_reports_info_and_raises(eng, hbs):
    A = np.eye(40)
    A[17, 17] = -1.0
    _, _, info = eng.potrf_inv(torch.tensor(A, device=eng.device))
    assert int(info.item()) == 18                 # LAPACK-style 1-based row
    bad = _model(hbs["X"], hbs["Y"], _params(5, 49))
    bad.kernel.kernel_L.variance.assign(1e300)    # overflowing trailing updates -> non-finite pivot
    with pytest.raises(M.CholeskyError):
        bad.log_marginal_likelihood()


@pytest.mark.parametrize("which,seed", [("hbs", None), ("hbs", 4), ("goku", None), ("goku", 5), ("forrester", 6)])
def test_lml_and_grad(which, seed, tile, hbs, goku):
    if which == "forrester":
        from conftest import forrester_test_data
        X, Y = forrester_test_data()
    else:
        d = hbs if which == "hbs" else goku
        X, Y = d["X"], d["Y"]
    D, P = X.shape[1] - 1, Y.shape[1]
    p = O.MFParams.initial(D, P) if seed is None else _params(D, P, seed=seed)
    m = _model(X, Y, p)
    po = _oracle_params(m)
    lo, go = O.gpr_lml_and_grad(X, Y, po)
    assert abs(float(m.log_marginal_likelihood()) - lo) < 1e-11 * abs(lo)
    l, g = m.log_marginal_likelihood_and_grad()
    gov = np.concatenate([[go["vL"]], go["lL"], [go["vD"]], go["lD"], [go["rho0"]], [go["noise"]]])
    assert abs(l - lo) < 1e-11 * abs(lo)
    np.testing.assert_allclose(g, gov, rtol=0, atol=1e-8 * np.abs(gov).max())


def test_lml_kats(hbs, goku, kats, eng):
    for d, key in ((hbs, "hbs_lml_initial"), (goku, "goku_lml_initial")):
        m = _model(d["X"], d["Y"], O.MFParams.initial(d["X"].shape[1] - 1, d["Y"].shape[1]))
        v = float(m.log_marginal_likelihood())
        assert abs(v - kats[key]["value"]) < 1e-12 * abs(v)


@pytest.mark.parametrize("which", ["hbs", "goku"])
def test_predict_f(which, tile, hbs, goku):
    d = hbs if which == "hbs" else goku
    p = _params(d["X"].shape[1] - 1, d["Y"].shape[1], seed=7)
    m = _model(d["X"], d["Y"], p)
    po = _oracle_params(m)
    for Xs in (d["Xtest"], d["X"][::7]):
        mean, var = m.predict_f(Xs)
        mo, vo = O.gpr_predict_f(d["X"], d["Y"], Xs, po)
        assert mean.shape == mo.shape and var.shape == vo.shape
        np.testing.assert_allclose(mean.numpy(), mo, rtol=0, atol=1e-9 * max(1, np.abs(mo).max()))
        np.testing.assert_allclose(var.numpy(), vo, rtol=0, atol=1e-9)


@pytest.mark.parametrize("n_lf,n_hf,p", [(20, 5, 1), (60, 20, 3), (1128, 36, 64), (1400, 100, 40)])
def test_flow_matches_step_schedule(n_lf, n_hf, p, eng):
    """k_chol_flow (one persistent launch) and the launch-per-step k_chol_step sequence compute
    the same LML and gradient (different MFMA summation orders: rounding-level agreement),
    T = 1, 3, 37 and 47 tiles; also checks the flow really is the default schedule."""
    rng = np.random.default_rng(n_lf + p)
    D = 4
    X = np.vstack([np.hstack([rng.random((n_lf, D)), np.zeros((n_lf, 1))]),
                   np.hstack([rng.random((n_hf, D)), np.ones((n_hf, 1))])])
    Y = np.sin(X[:, :D] @ rng.standard_normal((D, p)) * 3.0)
    m = _model(X, Y, _params(D, p, seed=3))
    assert eng.flow() or torch.cuda.get_device_properties(0).multi_processor_count < 2
    vals = []
    for flow in (True, False):
        eng.set_flow(flow, any_size=True)
        vals.append(m.log_marginal_likelihood_and_grad())
    eng.set_flow(True)
    assert abs(vals[0][0] - vals[1][0]) < 1e-11 * abs(vals[1][0])
    np.testing.assert_allclose(vals[0][1], vals[1][1], rtol=0, atol=1e-9 * np.abs(vals[1][1]).max())
    lo, go = O.gpr_lml_and_grad(X, Y, _oracle_params(m))
    assert abs(vals[0][0] - lo) < 1e-10 * abs(lo)


def test_schedule_tables_rebuilt_when_clobbered(eng):
    """k_gram keeps the k_grad task order and the k_chol_flow owner table in the workspace with a
    key + content hash and skips rebuilding them when both are intact (sched_cached).  A stale
    table must never be used: results are bit-identical after (a) a call at another size, (b)
    one corrupted table entry below an intact key, (c) the whole workspace overwritten."""
    rng = np.random.default_rng(11)
    D, p = 4, 2

    def model(n_lf, n_hf):
        X = np.vstack([np.hstack([rng.random((n_lf, D)), np.zeros((n_lf, 1))]),
                       np.hstack([rng.random((n_hf, D)), np.ones((n_hf, 1))])])
        Y = np.sin(X[:, :D] @ rng.standard_normal((D, p)) * 3.0)
        return _model(X, Y, _params(D, p, seed=5))

    big, small = model(900, 300), model(60, 30)
    ref = big.log_marginal_likelihood_and_grad()
    ws = eng.workspace("gpr", 0)
    keys = {}
    for name, magic in (("order", 0x4F524431), ("owner", 0x464C4F57)):
        hits = np.nonzero(ws.view(torch.int32).cpu().numpy() == magic)[0]
        assert len(hits) >= 1, name
        keys[name] = int(hits[-1])

    def same(v):
        assert v[0] == ref[0]
        np.testing.assert_array_equal(v[1], ref[1])

    same(big.log_marginal_likelihood_and_grad())            # cached tables
    small.log_marginal_likelihood_and_grad()                # (a) other shape: rebuilt, then back
    same(big.log_marginal_likelihood_and_grad())
    for name, k in keys.items():                            # (b) one entry below an intact key
        w32 = ws.view(torch.int32)
        w32[k - 7] = w32[k - 7] ^ 0x5A5A
        same(big.log_marginal_likelihood_and_grad())
    ws.view(torch.int32).random_(0, 1 << 30)                # (c) everything overwritten
    same(big.log_marginal_likelihood_and_grad())


def test_tile_size_invariance(eng, goku):
    m = _model(goku["X"], goku["Y"], _params(10, 64, seed=8))
    vals = []
    for nb in (32, 64):
        eng.set_tile(nb)
        vals.append(m.log_marginal_likelihood_and_grad())
    eng.set_tile(32)
    assert abs(vals[0][0] - vals[1][0]) < 1e-12 * abs(vals[0][0])
    np.testing.assert_allclose(vals[0][1], vals[1][1], rtol=0, atol=1e-9 * np.abs(vals[0][1]).max())


@pytest.mark.parametrize("which", ["hbs", "goku"])
def test_adam_trajectory_kats(which, hbs, goku, kats, eng):
    d = hbs if which == "hbs" else goku
    key = "hbs_adam_lr0.1_lml" if which == "hbs" else "goku_adam_lr0.1_lml"
    D = d["X"].shape[1] - 1
    m = M.MultiFidelityGPModel(d["X"], d["Y"], M.SquaredExponential(lengthscales=np.ones(D)),
                               M.SquaredExponential(lengthscales=np.ones(D)))
    m.optimize(max_iters=1000, use_adam=True, learning_rate=0.1, unfix_noise_after=500, verbose=False)
    assert len(m.loss_history) == 1000
    # Bit-level region (<= 500): 1e-10.  The dynamics turn chaotic near iteration 520 (a 1e-13
    # perturbation grows to 1e-6 by 540, tests/test_oracle_kats.py) and then re-converge: the HIP
    # path measured 3.4e-8 / 4.1e-9 / 3.1e-9 at HBS 600 / 700 / 800 (round 2), so 600-800 are held
    # to 1e-7; iteration 900 (the oracle itself is 1.5e-5 off at Goku) keeps 1e-4.
    errs = {}
    for k, v in kats[key]["values"].items():
        k = int(k)
        errs[k] = abs(-m.loss_history[k] - v) / abs(v)
    print(which, {k: f"{e:.2e}" for k, e in sorted(errs.items())})
    for k, e in errs.items():
        tol = 1e-10 if k <= 500 else (1e-7 if k <= 800 else 1e-4)
        assert e < tol, (k, e, tol)
    # noise never trained in the Adam path (Appendix C-2)
    assert float(m.likelihood.variance.numpy()) == pytest.approx(1e-3, rel=1e-12)


def test_flow_trace_mode_stays_in_its_workspace(eng):
    """in trace mode (mfgp_set_flow(h, 2)) k_gram_flow writes a per-workgroup
    timeline at the end of the workspace; its region is sized from the k_gram_flow grid
    (flow_gram_dbg_count).  At T = 132 tiles (n = 4200, a grid of ~2300 set-up workgroups) every
    byte past the reported workspace size must stay untouched, and the trace mode must not change
    the results."""
    from multi_fidelity_gpflow_amd import _lib
    rng = np.random.default_rng(31)
    n_lf, n_hf, p, D = 3900, 300, 4, 3
    X = np.vstack([np.hstack([rng.random((n_lf, D)), np.zeros((n_lf, 1))]),
                   np.hstack([rng.random((n_hf, D)), np.ones((n_hf, 1))])])
    Y = np.sin(X[:, :D] @ rng.standard_normal((D, p)) * 3.0)
    Xd, Yd = torch.tensor(X, device=eng.device), torch.tensor(Y, device=eng.device)
    th = torch.tensor(np.concatenate([[1.0], np.full(D, 0.3), [0.5], np.full(D, 0.4), [0.9, 1e-3]]), device=eng.device)
    nbytes = eng.gpr_workspace_bytes(X.shape[0], p, D)
    ws = torch.full((nbytes + (1 << 20),), 0x5A, dtype=torch.uint8, device=eng.device)
    ref, _ = eng.gpr_lml(Xd, Yd, th, want_grad=True, ws=ws)
    ref = ref.cpu().numpy().copy()
    _lib.check(eng.lib.mfgp_set_flow(eng.h, 2), "mfgp_set_flow")
    try:
        got, info = eng.gpr_lml(Xd, Yd, th, want_grad=True, ws=ws)
        torch.cuda.synchronize()
    finally:
        eng.set_flow(True)
    assert int(info.item()) == 0
    assert bool((ws[nbytes:] == 0x5A).all())
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_graph_and_eager_agree(hbs, eng):
    hs = []
    for graph in (True, False):
        m = M.MultiFidelityGPModel(hbs["X"], hbs["Y"], M.SquaredExponential(lengthscales=np.ones(5)),
                                   M.SquaredExponential(lengthscales=np.ones(5)))
        m.optimize(max_iters=120, learning_rate=0.1, verbose=False, graph=graph)
        hs.append(np.array(m.loss_history))
    np.testing.assert_array_equal(hs[0], hs[1])


@pytest.mark.parametrize("flow", [True, False, "tiny"], ids=["flow", "steps", "tiny"])
def test_lbfgs_forrester_kat(kats, eng, flow):
    """notebooks/demo.ipynb:233,257: rho 1.99976989, noise 1e-06 after GPflow's two L-BFGS
    passes.  With the variance gradients in TF's autodiff form (dK/dv = exp(-r2/2), finite
    where the line search drives v to 0; the division form K / v gave NaN there) the device
    stops 2.7e-5 off with the launch-per-step Cholesky (the default below 8 tiles), 5.0e-8 with
    the one-launch kernel (the default at this size), and with the persistent flow 6.6e-7 while
    its L^{-1} rows were finalized through the coupling D_i R'' - H_i X(i-1,c), 3.8e-5 since they
    are D_i R''' (round 5): the line search's end points move with rounding-level differences
    of the objective, and the fp64 oracle's own driver stops 3.7e-5 off.  So the endpoint is held
    to the noise floor (5e-5) on the flow and step schedules and to 1e-6 on the one-launch kernel;
    the tight check is the GPU objective along the first L-BFGS evaluations against the oracle
    (1e-9)."""
    from conftest import forrester_demo_data
    X, Y = forrester_demo_data()
    tiny = flow == "tiny"
    eng.set_flow(bool(flow) and not tiny, any_size=True)
    eng.set_tiny(tiny)
    try:
        m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(), M.SquaredExponential())
        # every point the L-BFGS driver evaluates, with the device's value and gradient there
        visits, inner = [], m.log_marginal_likelihood_and_grad

        def recorded():
            lml, g = inner()
            visits.append((m._theta_map().theta(), lml, np.array(g)))
            return lml, g
        m.log_marginal_likelihood_and_grad = recorded
        m.optimize(max_iters=1000, learning_rate=0.01, use_adam=False, unfix_noise_after=500, verbose=False)
    finally:
        eng.set_flow(True)
        eng.set_tiny(True)   # the library default
    # the device objective is the oracle's at every point the optimizer visited, within what fp64
    # rounding of K itself moves the LML there.  The line search also visits nearly
    # singular K (noise at its 1e-6 floor, long lengthscales), where any fp64 Cholesky differs from
    # another by far more than 1e-11; the reference for "rounding level" at a point is the spread
    # of the oracle's own LML under symmetric relative perturbations of K of size n 2^-52 (four
    # draws): the backward error of an n x n Cholesky, |dK| <= gamma_{n+1} |L||L^T|.  So the
    # endpoint's spread between schedules is the line search's sensitivity, not a different
    # objective.
    rng = np.random.default_rng(0)
    worst, well, dg, nwell = 0.0, 0.0, 0.0, 0
    N, P = Y.shape
    for th, lml, g in visits:
        p = O.MFParams(th[0], th[1:2], th[2], th[3:4], np.full((1, 1), th[4]), th[5])
        lo, go = O.gpr_lml_and_grad(X, Y, p)
        K = O.mf_K(X, None, p)
        K[np.diag_indices_from(K)] += p.noise
        spread = 0.0
        for _ in range(4):
            U = rng.uniform(-1, 1, K.shape)
            Kp = K * (1.0 + N * 2.0 ** -52 * (U + U.T) / 2)
            Lp = np.linalg.cholesky(Kp)
            Ap = np.linalg.solve(Lp, Y)
            lp = -0.5 * np.sum(Ap * Ap) - P * np.sum(np.log(np.diag(Lp))) - 0.5 * N * P * np.log(2 * np.pi)
            spread = max(spread, abs(lp - lo))
        d = abs(lml - lo)
        worst = max(worst, d / max(spread, 1e-12 * abs(lo)))
        if spread < 1e-12 * abs(lo):   # well-conditioned points: value and gradient tight
            nwell += 1
            well = max(well, d / abs(lo))
            gov = np.concatenate([[go["vL"]], go["lL"], [go["vD"]], go["lD"], [go["rho0"]], [go["noise"]]])
            dg = max(dg, np.abs(g - gov).max() / max(np.abs(gov).max(), 1e-300))
    print(f"  {len(visits)} evaluations: |device - oracle| <= {worst:.2f} x the oracle's rounding spread; "
          f"at the {nwell} well-conditioned points value {well:.1e}, gradient {dg:.1e}")
    assert len(visits) > 20 and nwell >= 5
    assert worst < 50.0 and well < 1e-11 and dg < 1e-7
    rho = float(m.kernel.rho.numpy()[0, 0])
    print(f"L-BFGS Forrester ({'tiny' if tiny else ('flow' if flow else 'steps')}) rho {rho:.9f} vs recorded {kats['forrester_lbfgs']['rho']} "
          f"(rel {abs(rho - kats['forrester_lbfgs']['rho']) / kats['forrester_lbfgs']['rho']:.1e}), "
          f"noise {float(m.likelihood.variance.numpy()):.9e}")
    bound = 1e-6 if tiny else 5e-5
    assert abs(rho - kats["forrester_lbfgs"]["rho"]) < bound * kats["forrester_lbfgs"]["rho"]
    # the noise ends at its constraint's lower bound 1e-6 (GPflow's variance_lower_bound) plus
    # softplus of wherever the line search left u: the same stopping noise (8.8e-6 on the flow)
    assert float(m.likelihood.variance.numpy()) == pytest.approx(kats["forrester_lbfgs"]["noise"],
                                                                  rel=1e-6 if tiny else 5e-5)
    _, trace = O.lbfgs_train(X, Y, O.MFParams.initial(1, 1), max_iters=1000, return_trace=True)
    np.testing.assert_allclose(m.loss_history[:8], trace[:8], rtol=1e-9)


@pytest.mark.parametrize("n_lf,n_hf,p,D", [(50, 3, 49, 5), (20, 5, 1, 1), (24, 8, 32, 3), (40, 24, 64, 16),
                                           (60, 4, 33, 7), (1, 1, 1, 2)])
def test_tiny_matches_step_sequence(n_lf, n_hf, p, D, eng):
    """k_gpr_tiny (the whole LML value + gradient in one workgroup, n, p <= 64) against the
    four-launch step sequence and the oracle: T = 1 and 2 tiles, one and two column tiles of Y,
    D = 1 .. 16, n = 64 and p = 64 at the edges, a fractional-fidelity row (an exact-mask zero row
    of K, linear.py:67-70)."""
    rng = np.random.default_rng(n_lf * 7 + p)
    X = np.vstack([np.hstack([rng.random((n_lf, D)), np.zeros((n_lf, 1))]),
                   np.hstack([rng.random((n_hf, D)), np.ones((n_hf, 1))])])
    if n_lf + n_hf > 3:
        X[1, -1] = 0.9999999999999999
    Y = np.sin(X[:, :D] @ rng.standard_normal((D, p)) * 3.0)
    m = _model(X, Y, _params(D, p, seed=9))
    vals = []
    for tiny in (True, False):
        eng.set_tiny(tiny)
        vals.append(m.log_marginal_likelihood_and_grad())
        vals.append((float(m.log_marginal_likelihood()), None))
    eng.set_tiny(True)   # the library default
    assert abs(vals[0][0] - vals[2][0]) < 1e-12 * abs(vals[2][0])
    assert vals[0][0] == vals[1][0]                           # value-only call: the same kernel
    np.testing.assert_allclose(vals[0][1], vals[2][1], rtol=0, atol=1e-10 * np.abs(vals[2][1]).max())
    lo, go = O.gpr_lml_and_grad(X, Y, _oracle_params(m))
    gov = np.concatenate([[go["vL"]], go["lL"], [go["vD"]], go["lD"], [go["rho0"]], [go["noise"]]])
    assert abs(vals[0][0] - lo) < 1e-11 * abs(lo)
    np.testing.assert_allclose(vals[0][1], gov, rtol=0, atol=1e-8 * np.abs(gov).max())


@pytest.mark.parametrize("n_lf,n_hf,p,D,ns", [(50, 3, 49, 5, 10), (24, 8, 32, 3, 1), (40, 24, 64, 16, 64),
                                              (20, 5, 1, 1, 33)])
def test_tiny_predict_matches_step_sequence(n_lf, n_hf, p, D, ns, eng):
    """predict_f through k_gpr_tiny<true> (n, p, n* <= 64: one launch) against the seven-launch
    sequence and the oracle: T = 1 / 2, one / two column tiles of Y and of X*, D up to 16, n = p =
    n* = 64 at the edge, a fractional-fidelity test row (its K entries and K_diag are zero)."""
    rng = np.random.default_rng(n_lf * 5 + ns)
    X = np.vstack([np.hstack([rng.random((n_lf, D)), np.zeros((n_lf, 1))]),
                   np.hstack([rng.random((n_hf, D)), np.ones((n_hf, 1))])])
    Y = np.sin(X[:, :D] @ rng.standard_normal((D, p)) * 3.0)
    Xs = np.hstack([rng.random((ns, D)), (np.arange(ns) % 2)[:, None].astype(float)])
    if ns > 2:
        Xs[2, -1] = 0.5
    m = _model(X, Y, _params(D, p, seed=4))
    out = []
    for tiny in (True, False):
        eng.set_tiny(tiny)
        mean, var = m.predict_f(Xs)
        out.append((mean.numpy(), var.numpy()))
    eng.set_tiny(True)   # the library default
    np.testing.assert_allclose(out[0][0], out[1][0], rtol=0, atol=1e-10 * max(1.0, np.abs(out[1][0]).max()))
    np.testing.assert_allclose(out[0][1], out[1][1], rtol=0, atol=1e-10 * max(1.0, np.abs(out[1][1]).max()))
    mo, vo = O.gpr_predict_f(X, Y, Xs, _oracle_params(m))
    np.testing.assert_allclose(out[0][0], mo, rtol=0, atol=1e-9 * max(1.0, np.abs(mo).max()))
    np.testing.assert_allclose(out[0][1], vo, rtol=0, atol=1e-9 * max(1.0, np.abs(vo).max()))


def test_tiny_adam_matches_step_sequence(hbs, eng):
    """The HBS Adam step (mfgp_gpr_adam_step, graph-captured) through k_gpr_tiny and through the
    step sequence: 200 steps, the same loss history to rounding (the dynamics are smooth there)."""
    hs = []
    for tiny in (True, False):
        eng.set_tiny(tiny)   # empties the session pool: no graph captured under the other schedule is replayed
        m = M.MultiFidelityGPModel(hbs["X"], hbs["Y"], M.SquaredExponential(lengthscales=np.ones(5)),
                                   M.SquaredExponential(lengthscales=np.ones(5)))
        m.optimize(max_iters=200, learning_rate=0.1, verbose=False)
        hs.append(np.array(m.loss_history))
    eng.set_tiny(True)   # the library default
    err = np.abs(hs[0] - hs[1]) / np.abs(hs[1])
    print(f"tiny vs steps, 200 HBS Adam steps: max rel {err.max():.1e}")
    assert err.max() < 1e-10


def test_large_synthetic_properties(eng):
    """N = 4096 (T = 128 tiles): additivity of the shared-Gram LML over output
    columns, and agreement of the full value with the fp64 oracle."""
    rng = np.random.default_rng(20251015)
    nl, nh, D, P = 3584, 512, 10, 8
    X = np.vstack([np.hstack([rng.random((nl, D)), np.zeros((nl, 1))]),
                   np.hstack([rng.random((nh, D)), np.ones((nh, 1))])])
    Y = rng.standard_normal((nl + nh, P))
    p = O.MFParams(1.0, np.full(D, 1.0), 1.0, np.full(D, 1.0), np.ones((P, 1)), 1e-2)
    m = _model(X, Y, p)
    full = float(m.log_marginal_likelihood())
    parts = 0.0
    for i in range(0, P, 2):
        q = p.copy()
        q.rho = np.ones((2, 1))
        parts += float(_model(X, Y[:, i:i + 2], q).log_marginal_likelihood())
    assert abs(full - parts) < 1e-9 * abs(full)
    assert abs(full - O.gpr_lml(X, Y, _oracle_params(m))) < 1e-9 * abs(full)


@pytest.mark.parametrize("n_lf,n_hf,p", [(3584, 512, 64)])
def test_synthetic_scaleup_lml_vs_torch(n_lf, n_hf, p):
    """Synthetic scale-up recipe at N = 4096: LML and gradient-free LML
    of the HIP path vs. torch.linalg (fp64, on the GPU) on the same Gram built in torch
    (property check at a size the CPU oracle would take minutes on)."""
    from multi_fidelity_gpflow_amd.data import synthetic_multifidelity
    X, Y, _, _ = synthetic_multifidelity(n_lf, n_hf, 10, p, 16, seed=7)
    m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.full(10, 0.7)),
                               M.SquaredExponential(lengthscales=np.full(10, 0.9), variance=0.3))
    m.likelihood.variance.assign(1e-2)
    lml = float(m.log_marginal_likelihood())
    dev = torch.device("cuda")
    Xd, Yd = torch.tensor(X, device=dev), torch.tensor(Y, device=dev)

    def rbf(A, B, v, l):
        a, b = A / l, B / l
        return v * torch.exp(-0.5 * (-2 * a @ b.T + (a * a).sum(1)[:, None] + (b * b).sum(1)[None]))
    f = Xd[:, -1]
    s = (f == 0).double() + (f == 1).double()   # rho = 1
    h = (f == 1).double()
    K = (s[:, None] * s[None]) * rbf(Xd[:, :-1], Xd[:, :-1], 1.0, 0.7) \
        + (h[:, None] * h[None]) * rbf(Xd[:, :-1], Xd[:, :-1], 0.3, 0.9)
    K += 1e-2 * torch.eye(K.shape[0], device=dev, dtype=torch.float64)
    L = torch.linalg.cholesky(K)
    Z = torch.linalg.solve_triangular(L, Yd, upper=False)
    ref = float(-0.5 * (Z * Z).sum() - Yd.shape[1] * torch.log(torch.diagonal(L)).sum()
                - 0.5 * Yd.numel() * np.log(2 * np.pi))
    assert abs(lml - ref) < 1e-9 * abs(ref), (lml, ref)


def test_shared_theta_trainer_matches_adam_session(hbs):
    """distributed.SharedThetaTrainer's device path (LML+grad, all-reduce, packed Adam) on one
    rank reproduces MultiFidelityGPModel.optimize(use_adam=True)'s trajectory."""
    from multi_fidelity_gpflow_amd.distributed import SharedThetaTrainer
    X, Y = hbs["X"], hbs["Y"]
    mk = lambda: M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(5)),
                                        M.SquaredExponential(lengthscales=np.ones(5)))
    a = mk()
    a.optimize(max_iters=30, learning_rate=0.1, use_adam=True, verbose=False)
    b = mk()
    tr = SharedThetaTrainer(b, 0.1, 30)
    tr.run(30)
    tr.finish()
    np.testing.assert_allclose(b.loss_history, a.loss_history, rtol=1e-11)
    np.testing.assert_allclose(b.kernel.rho.numpy()[0], a.kernel.rho.numpy()[0], rtol=1e-11)
