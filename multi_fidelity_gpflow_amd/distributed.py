"""Multi-GPU sharding of the multi-bin emulator over output k-bins.

One process per GPU.  The P output bins are split into contiguous blocks, one per
rank.  Two modes:
  * per-shard theta (default, bench.py): every rank trains an independent multi-bin
    model on its block — the reference's shared Gram makes a bin only an extra
    right-hand side, so this is the "embarrassing" mode.  Collectives happen only at
    the edges: ONE broadcast of the packed inputs from rank 0 before training and one
    gather of the posterior blocks after it; nothing inside the training loop.
  * shared theta (SharedThetaTrainer): one model, the reference's trajectory; one
    all-reduce of 1 + G doubles per iteration.
Backend "nccl" is RCCL over xGMI on ROCm; "gloo" is used for CPU tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def bin_block(p: int, rank: int, world: int):
    """Contiguous [b0, b1) block of the p bins owned by `rank`."""
    edges = np.linspace(0, p, world + 1).round().astype(int)
    return int(edges[rank]), int(edges[rank + 1])


def broadcast_arrays(arrays, rank: int, world: int, device):
    """Rank 0 passes a list of float64 arrays; every rank gets copies.  One
    broadcast of the shape header and ONE broadcast of the packed payload."""
    if rank == 0:
        shapes = [np.shape(a) for a in arrays]
        hdr = [len(shapes)] + [len(s) for s in shapes] + [d for s in shapes for d in s]
        hdr_t = torch.tensor([len(hdr)] + hdr, dtype=torch.int64, device=device)
    else:
        hdr_t = torch.zeros(64, dtype=torch.int64, device=device)
    if rank == 0:
        pad = torch.zeros(64, dtype=torch.int64, device=device)
        pad[:hdr_t.numel()] = hdr_t
        hdr_t = pad
    if world > 1:
        dist.broadcast(hdr_t, 0)
    h = hdr_t.tolist()
    k = h[1]
    ndims = h[2:2 + k]
    dims = h[2 + k:2 + k + sum(ndims)]
    shapes, o = [], 0
    for nd in ndims:
        shapes.append(tuple(dims[o:o + nd]))
        o += nd
    size = sum(int(np.prod(s)) for s in shapes)
    if rank == 0:
        buf = torch.tensor(np.concatenate([np.asarray(a, dtype=np.float64).ravel() for a in arrays]),
                           dtype=torch.float64, device=device)
    else:
        buf = torch.empty(size, dtype=torch.float64, device=device)
    if world > 1:
        dist.broadcast(buf, 0)
    flat = buf.cpu().numpy()
    out, o = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(flat[o:o + n].reshape(s))
        o += n
    return out


def gather_bin_blocks(block: torch.Tensor, p: int, rank: int, world: int) -> torch.Tensor:
    """All-gather [n, p_r] column blocks into the full [n, p] array (bins in order)."""
    if world == 1:
        return block
    widths = [bin_block(p, r, world)[1] - bin_block(p, r, world)[0] for r in range(world)]
    wmax = max(widths)
    padded = torch.zeros((block.shape[0], wmax), dtype=block.dtype, device=block.device)
    padded[:, :block.shape[1]] = block
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded)
    return torch.cat([parts[r][:, :widths[r]] for r in range(world)], dim=1)


class SharedThetaTrainer:
    """Reference-parity multi-GPU training of ONE multi-bin model (SURVEY §8(e) shared-theta
    mode).  Every rank holds the full X and its contiguous bin block of Y; per Adam
    iteration it evaluates the block's LML and dLML/dtheta (the shared Gram / Cholesky is
    replicated, the bins' solves are split), ONE all-reduce sums the 1 + G values over
    ranks (the multi-bin LML is additive over output columns), and every rank applies the
    same Keras-Adam step, so theta stays identical everywhere and the trajectory is the
    single-model one of MultiFidelityGPModel.optimize(use_adam=True) (linear.py:200-214).

    Device path: mfgp_gpr_lml(want_grad) -> dist.all_reduce (RCCL over xGMI) ->
    mfgp_adam_packed.  The three hooks can be replaced (CPU rehearsal with gloo)."""

    def __init__(self, model, lr, max_iters, lml_grad=None, allreduce=None, adam=None):
        from .engine import Engine
        self.model = model
        self.max_iters = max(int(max_iters), 1)
        tm = model._theta_map()
        self.tm = tm
        G = len(tm.entries)
        u = tm.u()
        trainable = tm.trainable().astype(np.uint8)
        transform = np.ones(G, np.uint8)
        transform[tm.noise_index] = 2
        tie = tm.tie()
        span = np.ones(G, np.uint8)
        for q in range(G):
            lead = int(np.argmax(tie == tie[q]))
            if lead != q:
                span[q] = 0
                span[lead] += 1
        self.done = 0
        self.hist = []
        if lml_grad is None:   # MI355X path
            eng, X, Y = model._device_data()
            dev = eng.device
            f64 = dict(dtype=torch.float64, device=dev)
            self.eng, self.X, self.Y = eng, X, Y
            self.theta = torch.tensor(tm.theta(), **f64)
            self.u = torch.tensor(u, **f64)
            self.m = torch.zeros(G, **f64)
            self.v = torch.zeros(G, **f64)
            self.trainable = torch.tensor(trainable, device=dev)
            self.transform = torch.tensor(transform, device=dev)
            self.span = torch.tensor(span, device=dev)
            self.step_t = torch.zeros((1,), dtype=torch.int32, device=dev)
            self.lr = torch.full((self.max_iters,), float(np.float32(lr)), **f64)
            self.hist_t = torch.zeros((self.max_iters,), **f64)
            self.out = torch.zeros((1 + G,), **f64)
            self.info = torch.zeros((1,), dtype=torch.int32, device=dev)
            self.b1, self.b2 = float(np.float32(0.9)), float(np.float32(0.999))

            def _lml_grad():
                out, info = eng.gpr_lml(self.X, self.Y, self.theta, want_grad=True)
                self.out.copy_(out)
                self.info.copy_(info)
                return self.out

            self.bad = torch.zeros((1,), dtype=torch.int32, device=dev)

            def _adam(out):
                # the reduced LML is NaN on every rank when any rank's evaluation failed (its
                # finalize writes NaN): all ranks then skip the update and keep the step counter
                self.bad.copy_(torch.isnan(out[:1]))
                eng.adam_packed(self.u, self.theta, out[1:], self.m, self.v, self.trainable, self.transform,
                                self.span, self.step_t, self.lr, self.b1, self.b2, 1e-7, out, 1.0, self.hist_t,
                                None, info=self.bad)
            self.lml_grad, self.adam = _lml_grad, _adam
        else:
            self.lml_grad, self.adam = lml_grad, adam
        self.allreduce = allreduce or (lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM)
                                       if dist.is_available() and dist.is_initialized() else None)

    def step(self):
        out = self.lml_grad()
        self.allreduce(out)
        self.adam(out)
        self.done += 1

    def run(self, n):
        if self.done + n > self.max_iters:
            raise ValueError("SharedThetaTrainer: more iterations than max_iters")
        for _ in range(n):
            self.step()

    def finish(self):
        """Write theta back into the model (device path) and its loss_history."""
        from ._lib import MFGP_FLOW_TIMEOUT, MFGPError, info_error
        from .models import CholeskyError
        if not hasattr(self, "u"):
            return
        torch.cuda.synchronize()
        self.tm.set_u(self.u.cpu().numpy())
        h = self.hist_t[:self.done].cpu().numpy()
        self.model.loss_history = [np.float64(v) for v in h]
        v = int(self.info.item())
        steps = int(self.step_t.item())
        if v == MFGP_FLOW_TIMEOUT:
            raise info_error(v, "shared-theta optimize")
        if v == 0 and steps != self.done and np.all(np.isfinite(h)):
            raise MFGPError(f"shared-theta optimize: {self.done - steps} of {self.done} steps failed on some rank "
                            f"and were retried; the trajectory is incomplete")
        if v != 0 or not np.all(np.isfinite(h)):
            raise CholeskyError("shared-theta optimize: Cholesky failed")
