"""Two processes drive the HIP path through a real process group.

world_size 2, gloo, both ranks on the one GPU of the box (MFGP_FLOW=0: two persistent flows of
two processes cannot both be resident; the library's fence is per process).  No injected hooks:
  * SharedThetaTrainer (SURVEY §8(e) shared-theta mode): each rank evaluates its HBS bin block with
    mfgp_gpr_lml, one all-reduce of 1 + G doubles, the packed Adam step -- against the
    single-process AdamSession trajectory (MultiFidelityGPModel.optimize, linear.py:200-214);
  * SharedInducingTrainer (single-bin SVGP, Z and the noise shared): mfgp_svgp_elbo_grad per rank,
    one all-reduce of [ELBO, KL, VE | flag | dE/dZ | dE/dnoise], mfgp_adam_packed_ex -- against the
    single-process _SVGPTrainer over all bins (singlebin_svgp.py:64-97).
Bounds: 1e-11 relative in the loss, 1e-6 in Z."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import HBS_DIR, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["MFGP_FLOW"] = "0"
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _hbs():
    from multi_fidelity_gpflow_amd.data import PowerSpecs, multifidelity_training_set
    ps = PowerSpecs()
    ps.read_from_txt(HBS_DIR)
    X, Y, _, _ = multifidelity_training_set(ps)
    return X, Y


def _kern(d):
    import multi_fidelity_gpflow_amd as M
    return M.SquaredExponential(lengthscales=np.ones(d))


def _theta_worker(rank, world, port, out_path, steps):
    dist = _init(rank, world, port)
    import multi_fidelity_gpflow_amd as M
    from multi_fidelity_gpflow_amd.distributed import SharedThetaTrainer, bin_block
    X, Y = _hbs()
    d = X.shape[1] - 1
    b0, b1 = bin_block(Y.shape[1], rank, world)
    model = M.MultiFidelityGPModel(X, np.ascontiguousarray(Y[:, b0:b1]), _kern(d), _kern(d))
    tr = SharedThetaTrainer(model, 0.1, steps)
    tr.run(steps)
    tr.finish()
    if rank == 0:
        np.savez(out_path, hist=np.array(model.loss_history), rho=model.kernel.rho.numpy()[0],
                 lL=model.kernel.kernel_L.lengthscales.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _svgp_worker(rank, world, port, out_path, steps):
    dist = _init(rank, world, port)
    import multi_fidelity_gpflow_amd as M
    from multi_fidelity_gpflow_amd.distributed import SharedInducingTrainer, bin_block, broadcast_inducing
    X, Y = _hbs()
    d = X.shape[1] - 1
    b0, b1 = bin_block(Y.shape[1], rank, world)
    Yr = np.ascontiguousarray(Y[:, b0:b1])
    model = broadcast_inducing(M.SingleBinSVGP(X, Yr, _kern(d), _kern(d), Yr.shape[1], Z=np.zeros((50, d + 1))),
                               rank, world, torch.device("cuda", 0))
    Z0 = model.inducing_variable.numpy().copy()
    tr = SharedInducingTrainer(model, (X, Yr), steps, 0.1)
    tr.run(steps)
    tr.finish()
    if rank == 0:
        np.savez(out_path, hist=np.array(model.loss_history), Z=model.inducing_variable.numpy(), Z0=Z0,
                 noise=float(model.likelihood.variance.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_process_shared_theta_matches_adam_session(tmp_path):
    import multi_fidelity_gpflow_amd as M
    steps = 30
    out = str(tmp_path / "theta.npz")
    mp.spawn(_theta_worker, args=(2, _free_port(), out, steps), nprocs=2, join=True)
    r = np.load(out)
    X, Y = _hbs()
    d = X.shape[1] - 1
    m = M.MultiFidelityGPModel(X, Y, _kern(d), _kern(d))
    m.optimize(max_iters=steps, learning_rate=0.1, use_adam=True, verbose=False)
    np.testing.assert_allclose(r["hist"], np.array(m.loss_history), rtol=1e-11)
    np.testing.assert_allclose(r["rho"], m.kernel.rho.numpy()[0], rtol=1e-11)
    np.testing.assert_allclose(r["lL"], m.kernel.kernel_L.lengthscales.numpy(), rtol=1e-11)


def test_two_process_shared_inducing_matches_single_process(tmp_path):
    import multi_fidelity_gpflow_amd as M
    from multi_fidelity_gpflow_amd.params import Parameter
    from multi_fidelity_gpflow_amd.svgp import _SVGPTrainer
    steps = 8
    out = str(tmp_path / "svgp.npz")
    mp.spawn(_svgp_worker, args=(2, _free_port(), out, steps), nprocs=2, join=True)
    r = np.load(out)
    X, Y = _hbs()
    d = X.shape[1] - 1
    m = M.SingleBinSVGP(X, Y, _kern(d), _kern(d), Y.shape[1], Z=np.zeros((50, d + 1)))
    m.inducing_variable = Parameter(np.asarray(r["Z0"]))   # the ranks' (rank 0's) KMeans centres
    tr = _SVGPTrainer(m, (X, Y), steps, 0.1, graph=False)
    tr.run(steps)
    tr.finish()
    np.testing.assert_allclose(r["hist"], np.array(m.loss_history), rtol=1e-11)
    np.testing.assert_allclose(r["Z"], m.inducing_variable.numpy(), rtol=0, atol=1e-6)
    assert abs(r["noise"] - float(m.likelihood.variance.numpy())) < 1e-10 * abs(r["noise"])
