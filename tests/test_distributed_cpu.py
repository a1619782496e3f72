"""world_size-2 gloo rehearsal of the bin-sharded path (CPU, oracle as the per-rank compute).

Checks the pieces bench.py runs over RCCL: the single packed broadcast of the
inputs from rank 0, the contiguous bin blocks, and the gather of per-rank
results.  With a shared theta the multi-bin LML is additive over output columns,
so the per-block LMLs must sum to the full-data LML."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import HBS_DIR, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from multi_fidelity_gpflow_amd.distributed import bin_block, broadcast_arrays, gather_bin_blocks
    from oracle import mfgp_oracle as O
    arrays = None
    if rank == 0:
        d = O.load_powerspecs(HBS_DIR)
        arrays = [d["X"], d["Y"], d["Xtest"]]
    X, Y, Xt = broadcast_arrays(arrays, rank, world, torch.device("cpu"))
    P = Y.shape[1]
    b0, b1 = bin_block(P, rank, world)
    p = O.MFParams.initial(X.shape[1] - 1, b1 - b0)
    lml = torch.tensor([O.gpr_lml(X, Y[:, b0:b1], p)], dtype=torch.float64)
    parts = [torch.zeros_like(lml) for _ in range(world)]
    dist.all_gather(parts, lml)
    mean, _ = O.gpr_predict_f(X, Y[:, b0:b1], Xt, p)
    full = gather_bin_blocks(torch.tensor(mean), P, rank, world)
    if rank == 0:
        np.savez(out_path, lml=np.array([float(t) for t in parts]), mean=full.numpy(), X=X, Y=Y)
    dist.destroy_process_group()


def test_two_rank_bin_sharding(tmp_path, hbs):
    from oracle import mfgp_oracle as O
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = np.load(out)
    np.testing.assert_array_equal(r["X"], hbs["X"])
    np.testing.assert_array_equal(r["Y"], hbs["Y"])
    full = O.gpr_lml(hbs["X"], hbs["Y"], O.MFParams.initial(5, 49))
    assert abs(r["lml"].sum() - full) < 1e-9 * abs(full)
    mean_full, _ = O.gpr_predict_f(hbs["X"], hbs["Y"], hbs["Xtest"], O.MFParams.initial(5, 49))
    np.testing.assert_allclose(r["mean"], mean_full, rtol=0, atol=1e-10)


def _theta_flat(lml, g):
    return np.concatenate([[lml, g["vL"]], g["lL"], [g["vD"]], g["lD"], [g["rho0"], g["noise"]]])


def _shared_worker(rank, world, port, out_path, steps):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from multi_fidelity_gpflow_amd.distributed import SharedThetaTrainer, bin_block
    from oracle import mfgp_oracle as O
    d = O.load_powerspecs(HBS_DIR)
    X, Y = d["X"], d["Y"]
    D = X.shape[1] - 1
    b0, b1 = bin_block(Y.shape[1], rank, world)
    p0 = O.MFParams.initial(D, Y.shape[1])
    st = {"u": O.pack_unconstrained(p0), "opt": O.AdamTF210(lr=0.1), "hist": []}

    def lml_grad():   # the block's LML and dLML/dtheta at the shared theta (oracle compute)
        lml, g = O.gpr_lml_and_grad(X, Y[:, b0:b1], O.unpack_unconstrained(st["u"], p0))
        return torch.tensor(_theta_flat(lml, g), dtype=torch.float64)

    def adam(out):    # identical on every rank: Keras Adam on the summed gradient
        o = out.numpy()
        st["hist"].append(-o[0])
        g = {"vL": -o[1], "lL": -o[2:2 + D], "vD": -o[2 + D], "lD": -o[3 + D:3 + 2 * D], "rho0": -o[3 + 2 * D]}
        st["u"] = st["opt"].step(st["u"], O.grad_unconstrained(st["u"], g))

    class _TM:   # theta map stub (the device state is not used with injected hooks)
        entries = list(range(2 * D + 4))
        noise_index = 2 * D + 3

        def u(self):
            return np.zeros(2 * D + 4)

        def trainable(self):
            return np.ones(2 * D + 4, bool)

        def tie(self):
            return np.arange(2 * D + 4)

    class _Model:
        def _theta_map(self):
            return _TM()

    tr = SharedThetaTrainer(_Model(), 0.1, steps, lml_grad=lml_grad, adam=adam)
    tr.run(steps)
    if rank == 0:
        np.save(out_path, np.array(st["hist"]))
    dist.destroy_process_group()


def _single_model_hist(d, steps):
    from oracle import mfgp_oracle as O
    p0 = O.MFParams.initial(5, 49)
    u = O.pack_unconstrained(p0)
    opt = O.AdamTF210(lr=0.1)
    hist = []
    for _ in range(steps):
        lml, g = O.gpr_lml_and_grad(d["X"], d["Y"], O.unpack_unconstrained(u, p0))
        hist.append(-lml)
        u = opt.step(u, O.grad_unconstrained(u, {k: -np.asarray(v) for k, v in g.items()}))
    return np.array(hist)


def test_two_rank_shared_theta_matches_single_model(tmp_path):
    """Shared-theta mode (SharedThetaTrainer): 2 ranks x half of the 49 HBS bins, one
    all-reduce per iteration, reproduce the single-model Adam trajectory (oracle compute)."""
    from oracle import mfgp_oracle as O
    steps = 3
    out = str(tmp_path / "h.npy")
    mp.spawn(_shared_worker, args=(2, _free_port(), out, steps), nprocs=2, join=True)
    hist = np.load(out)
    np.testing.assert_allclose(hist, _single_model_hist(O.load_powerspecs(HBS_DIR), steps), rtol=1e-10)


def _svgp_worker(rank, world, port, out_path, steps, Z):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import math
    from multi_fidelity_gpflow_amd.distributed import SharedInducingTrainer, bin_block
    from oracle import mfgp_oracle as O
    from oracle.svgp_oracle import SingleBinTrainer
    d = O.load_powerspecs(HBS_DIR)
    X, Y = d["X"], d["Y"]
    b0, b1 = bin_block(Y.shape[1], rank, world)
    tr = SingleBinTrainer(X, Y[:, b0:b1], Z, lr=0.1, max_iters=2000)   # this rank's bins (oracle compute)
    names = list(tr.vars)
    st = {"g": None, "hist": []}
    loss_t = torch.zeros(1, dtype=torch.float64)
    gZ = torch.zeros(tr.vars["Z"].numel(), dtype=torch.float64)
    gn = torch.zeros(1, dtype=torch.float64)

    def grad():   # local objective and gradient; the shared parts into the reduction views
        loss = tr.neg_elbo()
        g = torch.autograd.grad(loss, [tr.vars[k] for k in names])
        st["g"] = dict(zip(names, g))
        loss_t.copy_(loss.detach().reshape(1))
        gZ.copy_(st["g"]["Z"].reshape(-1))
        gn.copy_(st["g"]["noise"].reshape(1))
        return 0.0

    def adam(failed):   # the oracle's Keras Adam with the reduced Z / noise gradients
        assert float(failed) == 0.0
        st["hist"].append(float(loss_t.item()))
        g = dict(st["g"], Z=gZ.reshape(tr.vars["Z"].shape), noise=gn.reshape(()))
        lr = tr.sched(tr.t)
        tr.t += 1
        alpha = lr * math.sqrt(1.0 - tr.b2 ** tr.t) / (1.0 - tr.b1 ** tr.t)
        with torch.no_grad():
            for k in names:
                tr.m[k] += (g[k] - tr.m[k]) * (1.0 - tr.b1)
                tr.v[k] += (g[k] * g[k] - tr.v[k]) * (1.0 - tr.b2)
                tr.vars[k] -= (tr.m[k] * alpha) / (torch.sqrt(tr.v[k]) + tr.eps)

    sh = SharedInducingTrainer(max_iters=steps, grad=grad, shared=[loss_t, gZ, gn], adam=adam)
    sh.run(steps)
    if rank == 0:
        np.savez(out_path, hist=np.array(st["hist"]), Z=tr.vars["Z"].detach().numpy(),
                 noise=float(tr.vars["noise"].detach()))
    dist.destroy_process_group()


def test_two_rank_singlebin_svgp_shared_inducing(tmp_path, hbs):
    """SURVEY §8(e) single-bin SVGP mode (SharedInducingTrainer): 2 ranks x half of the 49 HBS bins,
    Z and the noise shared and trained, one all-reduce of [objective | flag | dZ | dnoise] per
    iteration, reproduce the single-process SingleBinSVGP trajectory (oracle compute) to 1e-11."""
    from sklearn.cluster import KMeans
    from oracle.svgp_oracle import SingleBinTrainer
    steps = 6
    Z = KMeans(n_clusters=50, random_state=42).fit(hbs["X"]).cluster_centers_
    out = str(tmp_path / "s.npz")
    mp.spawn(_svgp_worker, args=(2, _free_port(), out, steps, Z), nprocs=2, join=True)
    r = np.load(out)
    ref = SingleBinTrainer(hbs["X"], hbs["Y"], Z, lr=0.1, max_iters=2000)
    hist = np.array([ref.step() for _ in range(steps)])
    np.testing.assert_allclose(r["hist"], hist, rtol=1e-11)
    np.testing.assert_allclose(r["Z"], ref.vars["Z"].detach().numpy(), rtol=1e-11, atol=1e-13)
    assert abs(r["noise"] - float(ref.vars["noise"].detach())) < 1e-11 * abs(float(ref.vars["noise"].detach()))
