"""Child process of tests/test_gpu_rccl.py: one rank (world size 1) on the one GPU drives the
multi-GPU code paths of distributed.py through a real process group of the backend named on the
command line ("nccl" = RCCL, or "gloo"), and saves what they produced.

  python tests/_dist_ws1_worker.py BACKEND PORT OUT.npz

Under nccl the two trainers replay their steps from hipGraphs with the all-reduce captured inside
them; under gloo they run eagerly.  The test compares the two backends bit for bit."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBS_DIR = os.path.join(ROOT, "tests", "golden", "data", "50_LR_3_HR")


def main():
    backend, port, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=0, world_size=1)
    import multi_fidelity_gpflow_amd as M
    from multi_fidelity_gpflow_amd.data import PowerSpecs, multifidelity_training_set
    from multi_fidelity_gpflow_amd.distributed import (SharedInducingTrainer, SharedThetaTrainer, broadcast_arrays,
                                                      gather_bin_blocks)
    ps = PowerSpecs()
    ps.read_from_txt(HBS_DIR)
    X, Y, Xt, _ = multifidelity_training_set(ps)
    d = X.shape[1] - 1
    res = {}
    # one packed broadcast of the inputs, one all-gather of a [n, p] block
    Xb, Yb = broadcast_arrays([X, Y], 0, 1, dev)
    res["bcast_ok"] = np.array(np.array_equal(Xb, X) and np.array_equal(Yb, Y))
    blk = torch.tensor(Y, dtype=torch.float64, device=dev)
    res["gather_ok"] = np.array(bool(torch.equal(gather_bin_blocks(blk, Y.shape[1], 0, 1), blk)))

    def kern():
        return M.SquaredExponential(lengthscales=np.ones(d))

    # shared-theta trainer: 30 Adam steps (first eager, then graphs of 10 under nccl)
    model = M.MultiFidelityGPModel(X, Y, kern(), kern())
    tr = SharedThetaTrainer(model, 0.1, 30, graph_chunk=10)
    res["theta_graph"] = np.array(tr.graph_chunk)
    tr.run(30)
    tr.finish()
    res["theta_hist"] = np.array(model.loss_history)
    res["theta_rho"] = model.kernel.rho.numpy().reshape(-1)
    res["theta_lL"] = model.kernel.kernel_L.lengthscales.numpy()
    # shared-inducing trainer: 8 single-bin SVGP steps (first eager, then graphs of 4 under nccl)
    sv = M.SingleBinSVGP(X, Y, kern(), kern(), Y.shape[1], Z=np.zeros((50, d + 1)))
    # Z pinned to the first 50 training inputs (the host KMeans may differ in the last ulp between
    # processes, and the two backends' runs are compared bit for bit)
    sv.inducing_variable = M.Parameter(np.ascontiguousarray(X[:50]))
    res["Z0"] = sv.inducing_variable.numpy().copy()
    sh = SharedInducingTrainer(sv, (X, Y), 8, 0.1, graph_chunk=4)
    res["svgp_graph"] = np.array(sh.graph_chunk)
    sh.run(8)
    sh.finish()
    res["svgp_hist"] = np.array(sv.loss_history)
    res["svgp_Z"] = sv.inducing_variable.numpy()
    res["svgp_noise"] = np.array(float(sv.likelihood.variance.numpy()))
    np.savez(out, **res)
    dist.barrier()
    dist.destroy_process_group()
    print(f"{backend}: ok", flush=True)


if __name__ == "__main__":
    main()
