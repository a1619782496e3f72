"""RCCL runs the multi-GPU code paths: a world-size-1 "nccl" process group on the
one GPU of the box (legal with one rank per device; not a scaling claim).

A child process (tests/_dist_ws1_worker.py) drives broadcast_arrays, gather_bin_blocks, 30
SharedThetaTrainer steps and 8 SharedInducingTrainer steps through the process group.  Under nccl
both trainers replay their steps from hipGraphs with the RCCL all-reduce captured inside; under gloo
they run eagerly.  The two backends must agree bit for bit, and the shared-theta trajectory must be
the single-process AdamSession's (linear.py:200-214) and the shared-inducing one the single-process
SVGP trainer's (singlebin_svgp.py:64-97)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import HBS_DIR, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(backend, tmp_path):
    out = str(tmp_path / f"{backend}.npz")
    env = dict(os.environ)
    env.setdefault("NCCL_SOCKET_IFNAME", "lo")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "_dist_ws1_worker.py"), backend,
                        str(_free_port()), out], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"{backend} worker failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    return dict(np.load(out))


@pytest.fixture(scope="module")
def runs(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("ws1")
    return {b: _run(b, tmp) for b in ("nccl", "gloo")}


def test_rccl_collectives_and_graph_capture(runs):
    nc, gl = runs["nccl"], runs["gloo"]
    assert nc["bcast_ok"] and nc["gather_ok"] and gl["bcast_ok"] and gl["gather_ok"]
    assert int(nc["theta_graph"]) > 0 and int(nc["svgp_graph"]) > 0      # RCCL: captured steps
    assert int(gl["theta_graph"]) == 0 and int(gl["svgp_graph"]) == 0    # gloo: eager
    for k in ("theta_hist", "theta_rho", "theta_lL", "svgp_hist", "svgp_Z", "svgp_noise"):
        np.testing.assert_array_equal(nc[k], gl[k], err_msg=k)


def test_shared_trainers_match_single_process(runs):
    import multi_fidelity_gpflow_amd as M
    from multi_fidelity_gpflow_amd.data import PowerSpecs, multifidelity_training_set
    from multi_fidelity_gpflow_amd.svgp import _SVGPTrainer
    r = runs["nccl"]
    ps = PowerSpecs()
    ps.read_from_txt(HBS_DIR)
    X, Y, _, _ = multifidelity_training_set(ps)
    d = X.shape[1] - 1
    m = M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(d)),
                               M.SquaredExponential(lengthscales=np.ones(d)))
    m.optimize(max_iters=30, learning_rate=0.1, use_adam=True, verbose=False)
    np.testing.assert_allclose(r["theta_hist"], np.array(m.loss_history), rtol=1e-11)
    np.testing.assert_allclose(r["theta_rho"][0], m.kernel.rho.numpy().reshape(-1)[0], rtol=1e-11)
    np.testing.assert_allclose(r["theta_lL"], m.kernel.kernel_L.lengthscales.numpy(), rtol=1e-11)
    sv = M.SingleBinSVGP(X, Y, M.SquaredExponential(lengthscales=np.ones(d)),
                         M.SquaredExponential(lengthscales=np.ones(d)), Y.shape[1], Z=np.zeros((50, d + 1)))
    sv.inducing_variable = M.Parameter(np.asarray(r["Z0"]))
    tr = _SVGPTrainer(sv, (X, Y), 8, 0.1, graph=False)
    tr.run(8)
    tr.finish()
    np.testing.assert_allclose(r["svgp_hist"], np.array(sv.loss_history), rtol=1e-11)
    np.testing.assert_allclose(r["svgp_Z"], sv.inducing_variable.numpy(), rtol=0, atol=1e-9)
