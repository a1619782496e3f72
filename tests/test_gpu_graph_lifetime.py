"""Graph lifetime orders: a session's captured hipGraphs are destroyed while graphs
captured LATER by another session stay live and are replayed next.  Round 5's fp32 knob sweep
crashed in hipGraphLaunch on such an order; these run it on the product paths once each and check
the replayed results against eager runs:
  * fp32 with the one-panel lookahead (side-stream fork / join inside the graphs);
  * single-bin SVGP training (the gradient's side-stream fork / join);
  * a pooled fp64 Adam core evicted by the session pool's LRU cap after later sessions captured."""
import numpy as np
import pytest
import torch

import multi_fidelity_gpflow_amd as M
from multi_fidelity_gpflow_amd.engine import Engine

pytestmark = pytest.mark.gpu


def _f32_model(n_lf=3584, n_hf=512, p=64):
    from multi_fidelity_gpflow_amd.data import synthetic_multifidelity
    X, Y, _, _ = synthetic_multifidelity(n_lf=n_lf, n_hf=n_hf, p=p)
    d = X.shape[1] - 1
    return M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(d)),
                                  M.SquaredExponential(lengthscales=np.ones(d)), dtype="float32")


def _hist(sess, n):
    sess.sync()
    return sess.hist[:n].cpu().numpy().copy()


def test_f32_lookahead_release_earlier_graphs_then_replay():
    eng = Engine.get()
    eng.set_f32_lookahead(True)
    m = _f32_model()
    ref = m.adam_session(0.1, 6, graph=False)
    ref.run(6)
    h_ref = _hist(ref, 6)
    ref.close()
    del ref
    for _ in range(3):
        a = m.adam_session(0.1, 6, graph=True, graph_chunk=2)
        a.run(2)
        a.prepare(4)                  # capture A
        a.run(4)
        b = m.adam_session(0.1, 6, graph=True, graph_chunk=2)
        b.run(2)
        b.prepare(4)                  # capture B
        a.close()                     # release A's graphs (captured earlier)
        del a
        b.run(4)                      # replay B
        np.testing.assert_array_equal(_hist(b, 6), h_ref)
        b.close()
        del b


def test_f32_release_after_next_session_warmup():
    """The order that crashed (tools/graph_lifetime_probe.py small_graphs_after): the
    next session is created and runs its eager fp32 lookahead step on a new stream, THEN the
    previous session's graphs are released, then the next session captures and replays.  Without
    the graph retirement the fifth session's first replay segfaulted in hipGraphLaunch, every run."""
    from multi_fidelity_gpflow_amd import models as MM
    eng = Engine.get()
    eng.set_f32_lookahead(True)
    m = _f32_model()
    ref = m.adam_session(0.1, 6, graph=False)
    ref.run(6)
    h_ref = _hist(ref, 6)
    ref.close()
    del ref
    n0 = len(MM._retired_graphs)
    prev = None
    for _ in range(7):
        sess = m.adam_session(0.1, 6, graph=True, graph_chunk=2)
        sess.run(2)                   # eager, on the new session's stream
        if prev is not None:
            prev.close()              # release the previous session's graphs now
            prev = None
        sess.prepare(4)
        sess.run(4)
        np.testing.assert_array_equal(_hist(sess, 6), h_ref)
        prev = sess
    prev.close()
    assert len(MM._retired_graphs) >= n0 + 7


def test_svgp_release_earlier_graphs_then_replay(hbs):
    from multi_fidelity_gpflow_amd.svgp import _SVGPTrainer
    X, Y = hbs["X"], hbs["Y"]
    d = X.shape[1] - 1

    def model():
        sv = M.SingleBinSVGP(X, Y, M.SquaredExponential(lengthscales=np.ones(d)),
                             M.SquaredExponential(lengthscales=np.ones(d)), Y.shape[1], Z=np.zeros((50, d + 1)))
        sv.inducing_variable = M.Parameter(np.ascontiguousarray(X[:50]))
        return sv

    ref = _SVGPTrainer(model(), (X, Y), 8, 0.1, graph=False)
    ref.run(8)
    ref.sync()
    h_ref = ref.loss_hist.cpu().numpy().copy()
    for _ in range(3):
        a = _SVGPTrainer(model(), (X, Y), 8, 0.1, graph=True, graph_chunk=4)
        a.run(8)                      # capture + replay A
        b = _SVGPTrainer(model(), (X, Y), 8, 0.1, graph=True, graph_chunk=4)
        with torch.cuda.stream(b.stream):
            b.runner.prepare(8)       # capture B
        a.close()                     # release A's graphs
        del a
        b.run(8)                      # replay B
        b.sync()
        np.testing.assert_array_equal(b.loss_hist.cpu().numpy(), h_ref)
        b.close()
        del b


def test_pool_eviction_after_later_capture(hbs):
    from multi_fidelity_gpflow_amd import models as MM
    MM.clear_session_pool()
    X, Y = hbs["X"], hbs["Y"]
    d = X.shape[1] - 1

    def model():
        return M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(d)),
                                      M.SquaredExponential(lengthscales=np.ones(d)))

    ref = model()
    ref.optimize(max_iters=44, learning_rate=0.1, verbose=False, graph=False)
    old = MM._POOL_MAX_ENTRIES
    MM._POOL_MAX_ENTRIES = 1
    try:
        for it in (40, 41, 42, 43, 44):
            # session `it` captures while the pool still holds the core of `it - 1`; its finish()
            # evicts that older core (its graphs destroyed) after this later capture
            m = model()
            s = m.adam_session(0.1, it, graph_chunk=20)
            s.prepare(it)
            s.run(it)
            s.finish()
        m = model()
        s = m.adam_session(0.1, 44, graph_chunk=20)   # the pooled core of 44: replay only
        s.run(44)
        s.finish()
    finally:
        MM._POOL_MAX_ENTRIES = old
        MM.clear_session_pool()
    np.testing.assert_array_equal(np.array(m.loss_history), np.array(ref.loss_history))
