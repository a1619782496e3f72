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


def _group() -> bool:
    return dist.is_available() and dist.is_initialized()


def broadcast_arrays(arrays, rank: int, world: int, device):
    """Rank 0 passes a list of float64 arrays; every rank gets copies.  One
    broadcast of the shape header and ONE broadcast of the packed payload (whenever a process
    group exists, world size 1 included)."""
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
    if world > 1 or _group():
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
    if world > 1 or _group():
        dist.broadcast(buf, 0)
    flat = buf.cpu().numpy()
    out, o = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(flat[o:o + n].reshape(s))
        o += n
    return out


def gather_bin_blocks(block: torch.Tensor, p: int, rank: int, world: int) -> torch.Tensor:
    """All-gather [n, p_r] column blocks into the full [n, p] array (bins in order; with no process
    group the block is the whole array)."""
    if world == 1 and not _group():
        return block
    widths = [bin_block(p, r, world)[1] - bin_block(p, r, world)[0] for r in range(world)]
    wmax = max(widths)
    padded = torch.zeros((block.shape[0], wmax), dtype=block.dtype, device=block.device)
    padded[:, :block.shape[1]] = block
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded)
    return torch.cat([parts[r][:, :widths[r]] for r in range(world)], dim=1)


def _graph_default() -> bool:
    """Whether a trainer replays its steps (collective included) from hipGraphs: with RCCL ("nccl",
    whose collectives are stream-ordered and capturable) or with no process group (the all-reduce
    is then a no-op); gloo collectives synchronise on the host, so a gloo trainer runs eagerly."""
    if not (dist.is_available() and dist.is_initialized()):
        return True
    return dist.get_backend() == "nccl"


class SharedThetaTrainer:
    """Reference-parity multi-GPU training of ONE multi-bin model (SURVEY §8(e) shared-theta
    mode).  Every rank holds the full X and its contiguous bin block of Y; per Adam
    iteration it evaluates the block's LML and dLML/dtheta (the shared Gram / Cholesky is
    replicated, the bins' solves are split), ONE all-reduce sums the 1 + G values over
    ranks (the multi-bin LML is additive over output columns), and every rank applies the
    same Keras-Adam step, so theta stays identical everywhere and the trajectory is the
    single-model one of MultiFidelityGPModel.optimize(use_adam=True) (linear.py:200-214).

    Device path: mfgp_gpr_lml(want_grad) -> dist.all_reduce (RCCL over xGMI) ->
    mfgp_adam_packed, on the trainer's stream, with a private workspace that only its own steps
    write (so every step may skip the flow's set-up launch, mfgp_set_resident).  Under RCCL (or
    with no process group) the steps are replayed from hipGraphs of `graph_chunk` steps, the
    all-reduce captured inside them (`graph`: None = that default; gloo runs eagerly).  The three
    hooks can be replaced (CPU rehearsal with gloo)."""

    def __init__(self, model, lr, max_iters, lml_grad=None, allreduce=None, adam=None, graph=None,
                 graph_chunk=50):
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
        self.stream = None
        self.allreduce = allreduce or (lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM)
                                       if dist.is_available() and dist.is_initialized() else None)
        if lml_grad is None:   # MI355X path
            eng, X, Y = model._device_data()
            dev = eng.device
            f64 = dict(dtype=torch.float64, device=dev)
            self.eng = eng
            self.stream = torch.cuda.Stream(dev)
            self.stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(self.stream):
                # every buffer a captured step points at is the trainer's own (the
                # workspace too -- the engine's shared one may be written by other calls between
                # steps, and a resident step would then skip a set-up it needs)
                self.X, self.Y = X.clone(), Y.clone()
                n, p, d = X.shape[0], Y.shape[1], X.shape[1] - 1
                self.ws = eng.private_workspace(eng.gpr_workspace_bytes(n, p, d))
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
                self.bad = torch.zeros((1,), dtype=torch.int32, device=dev)
            self.b1, self.b2 = float(np.float32(0.9)), float(np.float32(0.999))

            def _lml_grad():
                # every step is a value+grad call of the same problem on the private workspace,
                # which leaves it set up for the next (mfgp_set_resident)
                with eng.resident():
                    eng.gpr_lml(self.X, self.Y, self.theta, want_grad=True, ws=self.ws, out=self.out, info=self.info)
                return self.out

            def _adam(out):
                # the reduced LML is NaN on every rank when any rank's evaluation failed (its
                # finalize writes NaN): all ranks then skip the update and keep the step counter
                torch.ne(out[:1], out[:1], out=self._isnan)   # NaN test, no allocation
                self.bad.copy_(self._isnan)
                eng.adam_packed(self.u, self.theta, out[1:], self.m, self.v, self.trainable, self.transform,
                                self.span, self.step_t, self.lr, self.b1, self.b2, 1e-7, out, 1.0, self.hist_t,
                                None, info=self.bad)
            self._isnan = torch.zeros((1,), dtype=torch.bool, device=dev)
            self.lml_grad, self.adam = _lml_grad, _adam
            if graph is None:
                graph = _graph_default()
            self.graph_chunk = int(graph_chunk) if graph else 0
            self._warm = False
        else:
            self.lml_grad, self.adam = lml_grad, adam
            self.graph_chunk = 0
            self._warm = True
        from .models import _StepRunner
        self.runner = _StepRunner(self._one, self.graph_chunk)

    def _one(self):
        out = self.lml_grad()
        self.allreduce(out)
        self.adam(out)

    def step(self):
        self.run(1)

    def _ctx(self):
        import contextlib
        if self.stream is None:
            return contextlib.nullcontext()
        st = contextlib.ExitStack()
        st.enter_context(torch.cuda.stream(self.stream))
        st.enter_context(self.eng.ordered(self.stream))
        return st

    def run(self, n):
        if self.done + n > self.max_iters:
            raise ValueError("SharedThetaTrainer: more iterations than max_iters")
        if n <= 0:
            return
        with self._ctx():
            if not self._warm:
                # the first step runs eagerly: the communicator, the workspace set-up and the
                # kernels' launch attributes exist before any capture
                self._one()
                self.done += 1
                n -= 1
                self._warm = True
            self.runner.run(n)
        self.done += n

    def prepare(self, n):
        """Capture the graphs a later run(n) replays (nothing executes; after the first step)."""
        if self.stream is not None and self._warm:
            with torch.cuda.stream(self.stream):
                self.runner.prepare(n)

    def sync(self):
        if self.stream is not None:
            self.stream.synchronize()

    def close(self):
        self.runner.close()

    def finish(self):
        """Write theta back into the model (device path) and its loss_history."""
        from ._lib import MFGP_FLOW_TIMEOUT, MFGPError, info_error
        from .models import CholeskyError
        if not hasattr(self, "u"):
            return
        self.sync()
        self.close()
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


class SharedInducingTrainer:
    """SURVEY §8(e) sharding of ONE SingleBinSVGP (singlebin_svgp.py:39-62): every per-bin quantity
    (kernel theta_l, q_mu[:, l], q_sqrt[l]) lives on the rank that owns bin l, while the inducing
    inputs Z and the Gaussian noise are shared, trainable parameters of the one model.  The
    objective is additive over bins (SeparateIndependent: ELBO = sum_l VE_l * scale - KL_l), so per
    Adam iteration each rank evaluates its bins' ELBO and gradient, ONE all-reduce sums
    [ELBO, KL, VE | failed-evaluation flag | dE/dZ (M (D+1)) | dE/dnoise] over the ranks, and every
    rank applies the same Keras-Adam step: Z and the noise stay identical everywhere and the
    trajectory is the single-process one (singlebin_svgp.py:64-97).

    Device path (model = this rank's SingleBinSVGP of its bin block, Z identical on every rank,
    e.g. broadcast_inducing): mfgp_svgp_elbo_grad -> pack -> dist.all_reduce (RCCL over xGMI) ->
    unpack -> mfgp_adam_packed_ex gated on the reduced flag (a failed evaluation on any rank skips
    the step everywhere), on the trainer's stream.  Under RCCL (or with no process group) the steps
    are replayed from hipGraphs of `graph_chunk` steps with the all-reduce captured inside them
    (`graph`: None = that default; gloo, whose collectives synchronise on the host, runs eagerly).
    Hooks (CPU rehearsal with gloo): grad() fills the tensors in `shared` (and returns the local
    failure flag), adam(failed) applies the step."""

    def __init__(self, model=None, data=None, max_iters=1, initial_lr=0.1, grad=None, shared=None, adam=None,
                 allreduce=None, graph=None, graph_chunk=50):
        self.tr = None
        if grad is None:   # MI355X path
            from .svgp import _SVGPTrainer
            tr = _SVGPTrainer(model, data, max_iters, initial_lr, graph=False)
            self.tr = tr
            self.gate = torch.zeros((1,), dtype=torch.int32, device=tr.eng.device)
            shared = [tr.out, tr.view(tr.g, "Z").reshape(-1), tr.view(tr.g, "noise").reshape(-1)]

            self._failed = torch.zeros((1,), dtype=torch.float64, device=tr.eng.device)

            def _grad():
                tr._grad()
                torch.amax(tr.info, dim=0, keepdim=True, out=self._imax)
                self._failed.copy_(self._imax != 0)
                return self._failed
            self._imax = torch.zeros((1,), dtype=torch.int32, device=tr.eng.device)

            def _adam(failed):
                self.gate.copy_(failed.reshape(1) > 0)
                tr.eng.adam_packed(tr.u, tr.c, tr.g, tr.mo, tr.vo, tr.trainable, tr.transform, tr.span, tr.step_t,
                                   tr.lr, tr.b1, tr.b2, 1e-7, tr.out, tr.klm, tr.loss_hist, tr.kl_hist,
                                   info=self.gate)
            grad, adam = _grad, _adam
            self.stream = tr.stream
        else:
            self.stream = None
        self.grad_fn, self.adam_fn, self.shared = grad, adam, list(shared)
        self.sizes = [t.numel() for t in self.shared]
        t0 = self.shared[0]
        self.buf = torch.zeros(sum(self.sizes) + 1, dtype=torch.float64, device=t0.device)
        self.allreduce = allreduce or (lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM)
                                       if dist.is_available() and dist.is_initialized() else None)
        self.done = 0
        self.max_iters = max(int(max_iters), 1)
        if self.tr is not None and graph is None:
            graph = _graph_default()
        self.graph_chunk = int(graph_chunk) if (graph and self.tr is not None) else 0
        self._warm = self.graph_chunk == 0
        from .models import _StepRunner
        self.runner = _StepRunner(self._one, self.graph_chunk)

    def _ctx(self):
        import contextlib
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def pack(self):
        """Local evaluation, then its shared part into the reduction buffer."""
        failed = self.grad_fn()
        o = 0
        for t, n in zip(self.shared, self.sizes):
            self.buf[o:o + n].copy_(t.reshape(-1))
            o += n
        self.buf[o:o + 1].copy_(torch.as_tensor(failed, dtype=torch.float64, device=self.buf.device).reshape(1))

    def unpack_step(self):
        """Reduced values back into the gradient / output views, then the Adam step."""
        o = 0
        for t, n in zip(self.shared, self.sizes):
            t.copy_(self.buf[o:o + n].reshape(t.shape))
            o += n
        self.adam_fn(self.buf[o:o + 1])

    def _one(self):
        self.pack()
        self.allreduce(self.buf)
        self.unpack_step()

    def step(self):
        self.run(1)

    def run(self, n):
        if self.done + n > self.max_iters:
            raise ValueError("SharedInducingTrainer: more iterations than max_iters")
        if n <= 0:
            return
        with self._ctx():
            if not self._warm:
                # the first step runs eagerly (communicator and workspace exist before any capture)
                self._one()
                self._count(1)
                n -= 1
                self._warm = True
            self.runner.run(n)
        self._count(n)

    def _count(self, n):
        self.done += n
        if self.tr is not None:   # the device trainer's own count (its finish() reads that many losses)
            self.tr.done = self.done

    def prepare(self, n):
        """Capture the graphs a later run(n) replays (nothing executes; after the first step)."""
        if self._warm and self.graph_chunk:
            with self._ctx():
                self.runner.prepare(n)

    def set_trainable(self, name, flag):
        self.tr.set_trainable(name, flag)

    def optimize(self, unfix_noise_after=None):
        """singlebin_svgp.py:64-97 loop (the noise becomes trainable after iteration
        unfix_noise_after), then the parameters and loss_history back into the model."""
        while self.done < self.max_iters:
            stop = self.max_iters
            noise_fixed = not self.tr.model.likelihood.variance.trainable
            if noise_fixed and unfix_noise_after is not None and self.done <= unfix_noise_after < self.max_iters:
                stop = unfix_noise_after + 1
            self.run(stop - self.done)
            if noise_fixed and unfix_noise_after is not None and self.done == unfix_noise_after + 1:
                self.set_trainable("noise", True)
        self.finish()

    def sync(self):
        if self.tr is not None:
            self.tr.sync()

    def finish(self):
        self.runner.close()
        if self.tr is not None:
            self.tr.finish()


def broadcast_inducing(model, rank: int, world: int, device):
    """Make the model's inducing inputs identical on every rank (rank 0's KMeans centres: the
    host KMeans can differ in the last ulp between processes)."""
    from .params import Parameter
    Z = broadcast_arrays([model.inducing_variable.numpy()] if rank == 0 else None, rank, world, device)[0]
    model.inducing_variable = Parameter(np.ascontiguousarray(Z, dtype=np.float64))
    return model
