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
