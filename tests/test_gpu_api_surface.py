"""GPflow API surface beyond the LML hot loop, on the HIP path (round-2 additions).

* ``predict_f(full_cov=True)`` — GPflow base_conditional's
  full-covariance branch (Knn − AᵀA, tiled to [P, N*, N*]) for the linear and graph models,
  against oracle/mfgp_oracle.py and oracle/graph_oracle.py: 1e-9 abs (fp64).
* ``SeparateIndependent.K`` / ``K_diag`` (singlebin_svgp.py:47) stack per-bin device Grams.
* The persistent Cholesky's timeout path raises ``FlowTimeoutError`` (not a numerical
  ``CholeskyError``), and the next call on the same workspace is correct again.
* Training sessions own their workspaces: two interleaved sessions reproduce their solo
  trajectories bit for bit; a prepared (pre-captured) run replays the same steps.
"""
import numpy as np
import pytest
import torch

import multi_fidelity_gpflow_amd as M
from multi_fidelity_gpflow_amd._lib import FlowTimeoutError
from multi_fidelity_gpflow_amd.engine import Engine
from oracle import graph_oracle as GO
from oracle import mfgp_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = Engine.get()
    yield e
    e.set_flow(True)
    e.set_flow_timeout_us(50000)


def _model(d, theta_seed=None):
    D = d["X"].shape[1] - 1
    m = M.MultiFidelityGPModel(d["X"], d["Y"], M.SquaredExponential(lengthscales=np.ones(D)),
                               M.SquaredExponential(lengthscales=np.ones(D)))
    if theta_seed is not None:
        rng = np.random.default_rng(theta_seed)
        m.kernel.kernel_L.lengthscales.assign(0.5 + rng.random(D))
        m.kernel.kernel_delta.lengthscales.assign(0.5 + rng.random(D))
        m.kernel.kernel_L.variance.assign(0.5 + rng.random())
        m.kernel.kernel_delta.variance.assign(0.1 + rng.random())
        m.kernel.rho.assign(np.full((d["Y"].shape[1], 1), 0.5 + rng.random()))
    return m


def _oracle_params(m, D, P):
    k = m.kernel
    return O.MFParams(float(k.kernel_L.variance.numpy()), np.broadcast_to(k.kernel_L.lengthscales.numpy(), (D,)).copy(),
                      float(k.kernel_delta.variance.numpy()),
                      np.broadcast_to(k.kernel_delta.lengthscales.numpy(), (D,)).copy(),
                      np.array(k.rho.numpy()), float(m.likelihood.variance.numpy()))


@pytest.mark.parametrize("which", ["hbs", "goku"])
def test_predict_full_cov(which, hbs, goku, eng):
    d = hbs if which == "hbs" else goku
    D, P = d["X"].shape[1] - 1, d["Y"].shape[1]
    m = _model(d, theta_seed=11)
    Xs = d["Xtest"]
    mean, cov = m.predict_f(Xs, full_cov=True)
    mo, co = O.gpr_predict_f_full_cov(d["X"], d["Y"], Xs, _oracle_params(m, D, P))
    assert tuple(cov.shape) == (P, Xs.shape[0], Xs.shape[0])
    np.testing.assert_allclose(mean.numpy(), mo, rtol=0, atol=1e-9)
    np.testing.assert_allclose(cov.numpy(), co, rtol=0, atol=1e-9)
    # the diagonal is the full_cov=False variance
    _, var = m.predict_f(Xs)
    np.testing.assert_allclose(np.diagonal(cov.numpy()[0]), var.numpy()[:, 0], rtol=0, atol=1e-12)
    _, yvar = m.predict_y(Xs)
    np.testing.assert_allclose(yvar.numpy() - var.numpy(), 1e-3, rtol=1e-9)
    with pytest.raises(NotImplementedError):   # GPflow 2.9 GPModel.predict_y
        m.predict_y(Xs, full_cov=True)


def test_graph_predict_full_cov(eng):
    rng = np.random.default_rng(3)
    D, P = 3, 4
    Xs_, Ys_ = [], []
    w = rng.standard_normal((D, P))
    for s, n in enumerate((40, 30, 12)):
        x = rng.uniform(0, 1, (n, D))
        Xs_.append(np.hstack([x, np.full((n, 1), float(s))]))
        Ys_.append(np.sin(3 * x @ w) * (1 + 0.3 * s))
    X, Y = np.vstack(Xs_), np.vstack(Ys_)
    kLs = [M.SquaredExponential(lengthscales=np.full(D, 0.8), variance=1.2) for _ in range(2)]
    kd = M.SquaredExponential(lengthscales=np.full(D, 0.6), variance=0.3)
    mod = M.GraphMultiFidelityGPModel(X, Y, kLs, kd)
    Xt = np.hstack([rng.uniform(0, 1, (9, D)), np.full((9, 1), 2.0)])
    mean, cov = mod.predict_f(Xt, full_cov=True)
    k = mod.kernel
    ks = k.kernel_Ls + [k.kernel_delta]
    f64 = dict(dtype=torch.float64)
    prm = dict(v=torch.tensor([float(kk.variance.numpy()) for kk in ks], **f64),
               l=torch.tensor(np.stack([kk.lengthscale_vector(D) for kk in ks]), **f64),
               rho=torch.tensor(k.rho.numpy()[:, 0], **f64), rhoLF=torch.tensor(k.rho_LF.numpy(), **f64))
    mo, co = GO.predict_f_full_cov(torch.tensor(X), torch.tensor(Y), torch.tensor(Xt), prm, 1e-3)
    np.testing.assert_allclose(mean.numpy(), mo.numpy(), rtol=0, atol=1e-9)
    np.testing.assert_allclose(cov.numpy()[2], co.numpy(), rtol=0, atol=1e-9)


def test_separate_independent_K(hbs, eng):
    kern = [M.LinearMultiFidelityKernel(M.SquaredExponential(lengthscales=np.full(5, 0.5 + 0.2 * i)),
                                        M.SquaredExponential(lengthscales=np.ones(5)), 1) for i in range(3)]
    si = M.kernels.SeparateIndependent(kern)
    X = hbs["X"]
    K = si.K(X)
    Kd = si.K_diag(X)
    assert tuple(K.shape) == (3, X.shape[0], X.shape[0]) and tuple(Kd.shape) == (X.shape[0], 3)
    for i, k in enumerate(kern):
        np.testing.assert_array_equal(K.numpy()[i], k.K(X).numpy())
        np.testing.assert_array_equal(Kd.numpy()[:, i], k.K_diag(X).numpy())


def test_flow_timeout_is_not_a_cholesky_error(goku, eng):
    """mfgp_set_flow_timeout_us(0): any hand-off that polls 8 times gives up -> the launch drains
    with info = MFGP_FLOW_TIMEOUT -> FlowTimeoutError; the next call (default bound) is correct."""
    eng.set_flow(True)
    if not eng.flow():
        pytest.skip("persistent Cholesky not available on this device")
    m = _model(goku)
    ref = m.log_marginal_likelihood_and_grad()
    eng.set_flow_timeout_us(0)
    try:
        with pytest.raises(FlowTimeoutError):
            m.log_marginal_likelihood_and_grad()
    finally:
        eng.set_flow_timeout_us(50000)
    again = m.log_marginal_likelihood_and_grad()
    assert again[0] == ref[0]
    np.testing.assert_array_equal(again[1], ref[1])


def test_interleaved_sessions_own_their_workspaces(hbs, goku, eng):
    """Two live Adam sessions (different sizes) interleaved on one engine reproduce their solo
    trajectories exactly: neither writes the other's workspace."""
    solo = []
    for d in (hbs, goku):
        m = _model(d)
        m.optimize(max_iters=60, learning_rate=0.1, verbose=False)
        solo.append(np.array(m.loss_history))
    ma, mb = _model(hbs), _model(goku)
    sa, sb = ma.adam_session(0.1, 60), mb.adam_session(0.1, 60)
    for _ in range(6):
        sa.run(10)
        sb.run(10)
    sa.finish()
    sb.finish()
    np.testing.assert_array_equal(np.array(ma.loss_history), solo[0])
    np.testing.assert_array_equal(np.array(mb.loss_history), solo[1])


def test_prepared_run_matches(hbs, eng):
    m1, m2 = _model(hbs), _model(hbs)
    s1 = m1.adam_session(0.1, 80, graph_chunk=50)
    s1.run(5)
    s1.prepare(75)    # captures the 50-step and 25-step graphs, runs nothing
    s1.run(75)
    s1.finish()
    m2.optimize(max_iters=80, learning_rate=0.1, verbose=False, graph=False)
    np.testing.assert_array_equal(np.array(m1.loss_history), np.array(m2.loss_history))


def test_eager_lml_during_async_session_is_fenced(goku, eng):
    """An eager log_marginal_likelihood() issued while an AdamSession's graph replays are still in
    flight on the session's stream: the library's device-wide flow fence orders the eager flow
    after them (no co-resident flows, no FlowTimeoutError) and the value is exact."""
    eng.set_flow(True)
    m, other = _model(goku), _model(goku)
    ref = other.log_marginal_likelihood_and_grad()
    solo = _model(goku)
    solo.optimize(max_iters=150, learning_rate=0.1, verbose=False)
    sess = m.adam_session(0.1, 150, graph_chunk=50)
    sess.prepare(150)
    sess.run(150)                       # ~40 ms of replays queued on the session's stream
    got = other.log_marginal_likelihood_and_grad()   # default stream, eager, while they run
    sess.finish()
    assert got[0] == ref[0]
    np.testing.assert_array_equal(got[1], ref[1])
    np.testing.assert_array_equal(np.array(m.loss_history), np.array(solo.loss_history))


def test_eager_flows_on_two_streams_are_fenced(goku, eng):
    """Two eager value+grad calls enqueued back to back on two non-blocking streams (two flows
    that would otherwise interleave their workgroups) both return the exact value."""
    eng.set_flow(True)
    m = _model(goku)
    ref = m.log_marginal_likelihood_and_grad()
    eng_, X, Y = m._device_data()
    theta = torch.tensor(m._theta_map().theta(), dtype=torch.float64, device=eng.device)
    s1, s2 = torch.cuda.Stream(eng.device), torch.cuda.Stream(eng.device)
    for s in (s1, s2):
        s.wait_stream(torch.cuda.current_stream(eng.device))
    outs = []
    for _ in range(3):
        for s in (s1, s2):
            with torch.cuda.stream(s):
                ws = eng.private_workspace(eng.gpr_workspace_bytes(X.shape[0], Y.shape[1], X.shape[1] - 1))
                outs.append(eng.gpr_lml(X, Y, theta, want_grad=True, ws=ws))
    torch.cuda.synchronize()
    for out, info in outs:
        assert int(info.item()) == 0
        o = out.cpu().numpy()
        assert o[0] == ref[0]
        np.testing.assert_array_equal(o[1:], ref[1])


def test_session_graph_lifetime_is_deterministic(hbs, eng):
    """A session and its hipGraphs are freed by reference counting when dropped (no session <->
    runner cycle left for a cyclic collection to reap mid-capture), and a forced collection inside
    another session's capture is harmless."""
    import gc
    import weakref
    m = _model(hbs)
    sa = m.adam_session(0.1, 60, graph_chunk=20)
    sa.run(40)
    sa.sync()
    ref_a = weakref.ref(sa)
    was = gc.isenabled()
    gc.disable()
    try:
        del sa
        assert ref_a() is None, "session kept alive by a reference cycle"
    finally:
        if was:
            gc.enable()
    m2, m3 = _model(hbs), _model(hbs)
    sb = m2.adam_session(0.1, 60, graph_chunk=20)
    step = sb._step

    def step_with_collect():
        gc.collect()
        step()
    sb.runner = M.models._StepRunner(step_with_collect, 20)   # collects inside the capture
    sb.run(60)
    sb.finish()
    m3.optimize(max_iters=60, learning_rate=0.1, verbose=False, graph=False)
    np.testing.assert_array_equal(np.array(m2.loss_history), np.array(m3.loss_history))


@pytest.mark.parametrize("flow", [True, False])
def test_gpr_independent_of_workspace_contents(goku, eng, flow):
    """Every workspace byte the GPR LML / gradient / predict read is written first in the same
    call: with the shared workspaces pre-filled with NaN bytes (0xFF) the results are bitwise the
    clean ones, for the persistent-flow and the launch-per-step Cholesky."""
    eng.set_flow(flow)
    try:
        m = _model(goku, theta_seed=5)
        eng._ws.clear()
        ref = m.log_marginal_likelihood_and_grad()
        mref, vref = m.predict_f(goku["Xtest"])
        eng._ws.clear()
        n, p, d = goku["X"].shape[0], goku["Y"].shape[1], goku["X"].shape[1] - 1
        for key, nbytes in (("gpr", eng.gpr_workspace_bytes(n, p, d)), ("pred", 256 << 20)):
            eng._ws[key] = torch.full((int(nbytes),), 255, dtype=torch.uint8, device=eng.device)
        got = m.log_marginal_likelihood_and_grad()
        mg, vg = m.predict_f(goku["Xtest"])
    finally:
        eng.set_flow(True)
        eng._ws.clear()
    assert got[0] == ref[0]
    np.testing.assert_array_equal(got[1], ref[1])
    np.testing.assert_array_equal(mg.numpy(), mref.numpy())
    np.testing.assert_array_equal(vg.numpy(), vref.numpy())


def test_flow_size_threshold(eng):
    """mfgp_set_flow(1) (the default) takes the persistent flow only for factorizations of 8 or more
    32-tiles (smaller ones are faster as step launches, tools/flow_threshold.py); mode 3 takes it at
    every size.  Observed through the workspace size, which holds the flow's publication area only
    when the flow runs."""
    try:
        sizes = {}
        for mode, kw in (("steps", dict(enable=False)), ("auto", dict(enable=True)),
                         ("any", dict(enable=True, any_size=True))):
            eng.set_flow(**kw)
            sizes[mode] = (eng.gpr_workspace_bytes(53, 49, 5), eng.gpr_workspace_bytes(1164, 64, 10))
        assert eng.flow()
    finally:
        eng.set_flow(True)
    small, large = 0, 1
    assert sizes["auto"][small] == sizes["steps"][small] < sizes["any"][small]   # HBS: T = 2
    assert sizes["auto"][large] == sizes["any"][large] > sizes["steps"][large]   # Goku: T = 37


def test_session_pool_reuses_graphs_exactly(hbs, eng):
    """A finished AdamSession's buffers and captured graphs are reused by the next fresh model of
    the same shape (models._pool): no recapture, and the trajectories are bitwise those of eager
    (graph=False) runs -- the reused graphs read only the new model's data and state."""
    from multi_fidelity_gpflow_amd import models as MM
    ref = _model(hbs)
    ref.optimize(max_iters=100, learning_rate=0.1, verbose=False, graph=False)
    m1 = _model(hbs)
    m1.optimize(max_iters=100, learning_rate=0.1, verbose=False)
    key = [k for k in MM._pool if k[3] == tuple(hbs["X"].shape) and k[6] == 100 and k[7] == 50]
    assert key, "the finished session was not pooled"
    core = MM._pool[key[0]]
    g_before = dict(core.graphs)
    m2 = _model(hbs)
    m2.kernel.kernel_L.variance.assign(1.3)     # a different initial state through the same graphs
    ref2 = _model(hbs)
    ref2.kernel.kernel_L.variance.assign(1.3)
    ref2.optimize(max_iters=100, learning_rate=0.1, verbose=False, graph=False)
    sess = m2.adam_session(0.1, 100)
    assert sess._core is core and all(sess.runner.graphs[k] is g for k, g in g_before.items())
    sess.run(100)
    sess.finish()
    np.testing.assert_array_equal(np.array(m1.loss_history), np.array(ref.loss_history))
    np.testing.assert_array_equal(np.array(m2.loss_history), np.array(ref2.loss_history))
    np.testing.assert_array_equal(m2.kernel.rho.numpy(), ref2.kernel.rho.numpy())


def test_session_pool_keys_on_handle_mode(hbs, eng):
    """a pooled session's graphs were captured under the handle's settings (tile, flow,
    one-launch path, k_grad chunk); changing any of them empties the pool, so the next session of
    the same shape captures afresh under the new schedule.  A finished session drops its aliases
    of the pooled buffers; the pool is capped (LRU) by entries and bytes."""
    from multi_fidelity_gpflow_amd import models as MM
    MM.clear_session_pool()
    m1 = _model(hbs)
    s1 = m1.adam_session(0.1, 60)
    s1.run(60)
    s1.finish()
    assert s1.st is None and s1.hist is None and s1.out is None and s1.X is None
    assert len(MM._pool) == 1
    mode0 = eng.mode()
    eng.set_tiny(not bool(mode0[2]))
    try:
        assert len(MM._pool) == 0 and eng.mode() != mode0
        m2 = _model(hbs)
        s2 = m2.adam_session(0.1, 60)
        assert s2._key[1] == eng.mode()
        s2.run(60)
        s2.finish()
    finally:
        eng.set_tiny(bool(mode0[2]))
    assert len(MM._pool) == 0
    np.testing.assert_allclose(m2.loss_history, m1.loss_history, rtol=1e-10)
    # LRU cap by entry count
    old = MM._POOL_MAX_ENTRIES
    MM._POOL_MAX_ENTRIES = 2
    try:
        for it in (40, 41, 42):
            m = _model(hbs)
            s = m.adam_session(0.1, it)
            s.run(it)
            s.finish()
        assert [k[6] for k in MM._pool] == [41, 42]
    finally:
        MM._POOL_MAX_ENTRIES = old
        MM.clear_session_pool()
