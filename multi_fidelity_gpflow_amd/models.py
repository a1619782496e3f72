"""MultiFidelityGPModel — drop-in for mfgpflow.linear.MultiFidelityGPModel.

Reference: mfgpflow/linear.py:138-234 (constructor, optimize) plus the GPflow 2.9
GPR methods it inherits (log_marginal_likelihood, training_loss, predict_f,
predict_y).  Every evaluation runs on the GPU through libmfgp.so:

  log_marginal_likelihood  -> mfgp_gpr_lml           (K1 gram, K2 tile Cholesky, K3, K4)
  optimize(use_adam=True)  -> mfgp_gpr_adam_step     (value + analytic grad + Keras Adam on
                                                      device, captured in a hipGraph)
  optimize(use_adam=False) -> scipy L-BFGS-B on the host, value+grad on the device
  predict_f                -> mfgp_gpr_predict       (K1, K2, K6)

Behavioural quirks of the reference that are reproduced:
  * one Gram / Cholesky shared by all P outputs; only rho[0] is used;
  * the likelihood noise starts at 1e-3, fixed; ``unfix_noise_after`` has no
    effect in the Adam path (the reference's tf.function traced the variable list
    before set_trainable), but the L-BFGS path does train it in its second pass;
  * ``loss_history`` records the pre-step loss (-LML) of every iteration.
"""
from __future__ import annotations

import atexit
import threading
import weakref
from collections import OrderedDict

import numpy as np
import torch

from ._lib import MFGP_FLOW_TIMEOUT, MFGPError, info_error
from .engine import AdamState, Engine, resolve_dtype, theta_size, to_dev
from .kernels import LinearMultiFidelityKernel
from .params import Module, Parameter, as_result, positive, set_trainable


class CholeskyError(MFGPError):
    """Analogue of TF's InvalidArgumentError('Cholesky decomposition was not successful')."""


class Gaussian(Module):
    """gpflow.likelihoods.Gaussian: variance >= 1e-6 via Shift(1e-6) o Softplus."""

    DEFAULT_VARIANCE_LOWER_BOUND = 1e-6

    def __init__(self, variance=1.0, variance_lower_bound=DEFAULT_VARIANCE_LOWER_BOUND):
        self.variance = Parameter(variance, transform=positive(lower=variance_lower_bound))


class _ThetaMap:
    """Maps the model's Parameters onto the device theta vector
    [vL, lL(d), vD, lD(d), rho0, noise] of include/mfgp.h."""

    def __init__(self, model: "MultiFidelityGPModel", d: int):
        k = model.kernel
        self.d = d
        self.entries = []   # (Parameter, index tuple or None)
        self.entries.append((k.kernel_L.variance, None))
        for i in range(d):
            self.entries.append((k.kernel_L.lengthscales, None if k.kernel_L.lengthscales.shape == () else (i,)))
        self.entries.append((k.kernel_delta.variance, None))
        for i in range(d):
            self.entries.append((k.kernel_delta.lengthscales,
                                 None if k.kernel_delta.lengthscales.shape == () else (i,)))
        self.entries.append((k.rho, (0, 0)))
        self.entries.append((model.likelihood.variance, None))
        assert len(self.entries) == theta_size(d)
        self.noise_index = theta_size(d) - 1

    def _gather(self, which: str) -> np.ndarray:
        # each Parameter's (constrained or unconstrained) array once, however many entries it owns
        arrs, out = {}, []
        for p, idx in self.entries:
            arr = arrs.get(id(p))
            if arr is None:
                arr = arrs[id(p)] = p.numpy() if which == "c" else p.unconstrained_variable
            out.append(float(arr if idx is None else arr[idx]))
        return np.array(out)

    def theta(self) -> np.ndarray:
        return self._gather("c")

    def u(self) -> np.ndarray:
        return self._gather("u")

    def trainable(self) -> np.ndarray:
        return np.array([p.trainable for p, _ in self.entries], dtype=bool)

    def tie(self) -> np.ndarray:
        ids, out = {}, []
        for p, i in self.entries:
            key = (id(p), i)
            out.append(ids.setdefault(key, len(ids)))
        return np.array(out, dtype=np.int32)

    def set_u(self, u: np.ndarray):
        # one assignment per Parameter (entries in order: a later entry of the same index wins)
        new = {}
        for (p, idx), val in zip(self.entries, u):
            if idx is None:
                new[id(p)] = (p, np.full(p.shape, val))
            else:
                arr = new[id(p)][1] if id(p) in new else p.unconstrained_variable.copy()
                arr[idx] = val
                new[id(p)] = (p, arr)
        for p, arr in new.values():
            p.unconstrained_variable = arr


class MultiFidelityGPModel(Module):
    """GPR with the linear multi-fidelity kernel and a shared Gram over P outputs.

    ``dtype`` (this engine's addition; the reference forces fp64, linear.py:63-64): ``None`` /
    ``"float64"`` runs the fp64 path; ``"float32"`` keeps X, Y on the device in fp32 and runs
    the fp32 path (include/mfgp.h ``*_ex`` with MFGP_F32: the BASELINE "Synth" config).  The
    parameters, the LML, its gradient and the Adam state stay fp64 either way."""

    def __init__(self, X, Y, kernel_L, kernel_delta, dtype=None):
        Xh = np.asarray(X.cpu().numpy() if isinstance(X, torch.Tensor) else X, dtype=np.float64)
        Yh = np.asarray(Y.cpu().numpy() if isinstance(Y, torch.Tensor) else Y, dtype=np.float64)
        if Yh.ndim == 1:
            Yh = Yh[:, None]
        num_output_dims = Yh.shape[1]
        self.kernel = LinearMultiFidelityKernel(kernel_L, kernel_delta, num_output_dims)
        self.likelihood = Gaussian(variance=1e-3)
        set_trainable(self.likelihood.variance, False)
        self.num_output_dims = num_output_dims
        self.mean_function = None
        self._Xh, self._Yh = Xh, Yh
        self.dtype = resolve_dtype(dtype)
        self._dev = None
        self.loss_history = []

    # ------------------------------------------------------------ data
    @property
    def data(self):
        return self._Xh, self._Yh

    def _device_data(self):
        eng = Engine.get()
        if self._dev is None or self._dev[0].device != eng.device:
            # X and Y as two views of one device buffer, filled by ONE pinned host-to-device copy
            npdt = np.float32 if self.dtype == torch.float32 else np.float64
            nx, ny = self._Xh.size, self._Yh.size
            hb = torch.empty((nx + ny,), dtype=self.dtype, pin_memory=True)
            hn = hb.numpy()
            hn[:nx] = self._Xh.astype(npdt, copy=False).ravel()
            hn[nx:] = self._Yh.astype(npdt, copy=False).ravel()
            db = hb.to(eng.device, non_blocking=True)
            self._dev = (db[:nx].view(self._Xh.shape), db[nx:].view(self._Yh.shape))
        return eng, self._dev[0], self._dev[1]

    def _device_inputs(self, eng, Xnew):
        """theta (fp64) and the new inputs (the model's dtype) on the device; on fp64 in ONE pinned
        host-to-device copy"""
        th = self._theta_map().theta()
        if self.dtype != torch.float64 or isinstance(Xnew, torch.Tensor):
            return (torch.tensor(th, dtype=torch.float64, device=eng.device), to_dev(Xnew, eng.device, self.dtype))
        xh = np.asarray(Xnew, dtype=np.float64)
        hb = torch.empty((th.size + xh.size,), dtype=torch.float64, pin_memory=True)
        hn = hb.numpy()
        hn[:th.size] = th
        hn[th.size:] = xh.ravel()
        db = hb.to(eng.device, non_blocking=True)
        return db[:th.size], db[th.size:].view(xh.shape)

    @property
    def input_dim(self) -> int:
        return self._Xh.shape[1] - 1

    def _theta_map(self) -> _ThetaMap:
        return _ThetaMap(self, self.input_dim)

    @staticmethod
    def _raise_info(info: torch.Tensor, what: str):
        err = info_error(int(info.reshape(-1)[0].item()), what)
        if err is not None:
            raise err

    # ------------------------------------------------------------ GPR surface
    def log_marginal_likelihood(self):
        """GPR log marginal likelihood.  On the float32 path the value-only call takes one fp64
        refinement step (mfgp_set_f32_refine), while log_marginal_likelihood_and_grad() and the
        training steps return the unrefined fp32 value: at the Synth size the two differ by
        ~8e-4 relative (the refined one is ~5e-5 from fp64).  On float64 they agree to rounding."""
        eng, X, Y = self._device_data()
        theta = torch.tensor(self._theta_map().theta(), dtype=torch.float64, device=eng.device)
        out, info = eng.gpr_lml(X, Y, theta, want_grad=False)
        self._raise_info(info, "log_marginal_likelihood")
        return as_result(out[0].clone())

    def maximum_log_likelihood_objective(self):
        return self.log_marginal_likelihood()

    def training_loss(self):
        return as_result(-self.log_marginal_likelihood())

    def log_marginal_likelihood_and_grad(self):
        """(LML, dLML/dtheta) with theta in the include/mfgp.h layout (numpy)."""
        eng, X, Y = self._device_data()
        theta = torch.tensor(self._theta_map().theta(), dtype=torch.float64, device=eng.device)
        out, info = eng.gpr_lml(X, Y, theta, want_grad=True)
        self._raise_info(info, "log_marginal_likelihood")
        o = out.cpu().numpy()
        return float(o[0]), o[1:]

    def predict_f(self, Xnew, full_cov: bool = False, full_output_cov: bool = False):
        """GPflow GPR.predict_f (mirror at linear.py:237-286): mean [N*, P]; var [N*, P]
        (full_cov=False) or [P, N*, N*] (full_cov=True, base_conditional's tiled Knn - AᵀA)."""
        if full_output_cov:
            raise NotImplementedError("predict_f(full_output_cov=True): GPR has no output covariance to return")
        eng, X, Y = self._device_data()
        theta, Xs = self._device_inputs(eng, Xnew)
        if full_cov:
            mean, _, cov, info = eng.gpr_predict_cov(0, X, Y, Xs, theta)
            self._raise_info(info, "predict_f")
            return as_result(mean), as_result(cov[None].expand(Y.shape[1], -1, -1).contiguous())
        mean, var, info = eng.gpr_predict(X, Y, Xs, theta)
        self._raise_info(info, "predict_f")
        return as_result(mean), as_result(var[:, None].expand(-1, Y.shape[1]).contiguous())

    def predict_y(self, Xnew, full_cov: bool = False, full_output_cov: bool = False):
        """GPflow GPModel.predict_y: predict_f plus the Gaussian noise variance."""
        if full_cov or full_output_cov:
            # GPflow 2.9 GPModel.predict_y (gpflow issue 1461): only the marginal form is supported
            raise NotImplementedError("The predict_y method currently supports only the argument values "
                                      "full_cov=False and full_output_cov=False")
        mean, var = self.predict_f(Xnew)
        return mean, as_result(var + float(self.likelihood.variance.numpy()))

    # ------------------------------------------------------------ training
    def optimize(self, max_iters=1000, learning_rate=0.01, use_adam=True, unfix_noise_after=500, verbose=True,
                 graph=True, graph_chunk=50):
        """mfgpflow/linear.py:190-234."""
        self.loss_history = []
        if use_adam:
            if verbose:
                print("Optimizing with Adam...")
            self._optimize_adam(max_iters, learning_rate, unfix_noise_after, verbose, graph, graph_chunk)
        else:
            if verbose:
                print("Optimizing with L-BFGS (Scipy)...")
            self._optimize_lbfgs(max_iters)

    def adam_session(self, learning_rate: float, max_iters: int, graph: bool = True, graph_chunk: int = 50):
        """Device-resident Adam training state (used by optimize() and bench.py)."""
        return AdamSession(self, learning_rate, max_iters, graph, graph_chunk)

    def _optimize_adam(self, max_iters, lr, unfix_noise_after, verbose, graph, chunk):
        sess = self.adam_session(lr, max_iters, graph, chunk)
        report = list(range(0, max_iters, 100)) if verbose else []
        done = 0
        for r in report + [max_iters - 1]:
            if r < done:
                continue
            sess.run(r + 1 - done)
            done = r + 1
            if verbose and r in report:
                sess.sync()
                if r == unfix_noise_after:
                    # reference prints this; the traced tf.function never sees the noise (Appendix C-2)
                    print(f"🔹 Unfixing noise at iteration {r}")
                print(f"🔹 Iteration {r}: Loss = {-sess.loss_at(r)}")
        sess.finish()

    def _optimize_lbfgs(self, max_iters):
        """gpflow.optimizers.Scipy().minimize twice: noise fixed, then trainable
        (linear.py:230-234).  GPflow semantics: the optimisation vector is the
        concatenation of the trainable Parameters' UNCONSTRAINED values in
        tf.Module attribute order (kernel_L.lengthscales, kernel_L.variance,
        kernel_delta.lengthscales, kernel_delta.variance, rho (all P entries),
        likelihood.variance); value + gradient come from the device, L-BFGS-B
        (scipy, jac=True) runs on the host."""
        from scipy.optimize import minimize

        for phase in (0, 1):
            if phase == 1:
                set_trainable(self.likelihood.variance, True)
            tm = self._theta_map()
            params = [p for _, p in self.parameters_with_names() if p.trainable]
            sizes = [int(np.prod(p.shape)) if p.shape else 1 for p in params]

            def pack():
                return np.concatenate([np.asarray(p.unconstrained_variable, dtype=np.float64).ravel() for p in params])

            def unpack(x):
                o = 0
                for p, n in zip(params, sizes):
                    p.unconstrained_variable = x[o:o + n].reshape(p.shape)
                    o += n

            def fg(x):
                unpack(x)
                lml, g = self.log_marginal_likelihood_and_grad()
                grads = {id(p): np.zeros(p.shape) for p in params}
                for (p, idx), gq in zip(tm.entries, g):
                    if id(p) not in grads:
                        continue
                    if idx is None:
                        grads[id(p)] = grads[id(p)] + gq
                    else:
                        grads[id(p)][idx] += gq
                # TF SoftplusGrad: upstream / (exp(-u) + 1), applied to the loss (-LML) gradient
                gu = np.concatenate([(-grads[id(p)] / (np.exp(-p.unconstrained_variable) + 1.0)).ravel()
                                     for p in params])
                self.loss_history.append(np.float64(-lml))
                return -lml, gu

            res = minimize(fg, pack(), jac=True, method="L-BFGS-B", options={"maxiter": max_iters})
            unpack(res.x)


# ---------------------------------------------------------------- session pool
# A fresh AdamSession of a shape seen before reuses the device buffers AND the captured step
# graphs of a finished one: its model's data and initial state are copied into the buffers the
# graphs point at, so no capture, no allocation and no warm-up evaluation are repeated.  The
# reference's multi-bin test (tests/test_ho2021_multibin.py:20-43) builds a fresh model per run;
# at HBS size the capture of the 50-step graph was a third of the 100-step protocol.
#
# Retention: only sessions whose private workspace is at most _POOL_MAX_WS_BYTES are pooled, one
# idle core per key (device, dtype, shapes, lr, max_iters, graph chunk and the handle's execution
# settings, Engine.mode()), at most _POOL_MAX_ENTRIES cores and _POOL_MAX_BYTES of their device
# buffers in all; beyond that the least recently used core is evicted (its graphs destroyed and its
# buffers freed -- eviction runs in finish(), outside any capture).  Changing the handle's settings
# (Engine.set_tile / set_flow / set_tiny) empties the pool, as does clear_session_pool() and
# interpreter exit (before the HIP runtime goes away).
_POOL_MAX_WS_BYTES = 96 << 20
_POOL_MAX_ENTRIES = 8
_POOL_MAX_BYTES = 512 << 20
_pool: "OrderedDict" = OrderedDict()   # key -> idle _AdamCore, least recently used first
_pool_lock = threading.Lock()


def _release(cores):
    for c in cores:
        c.release()


def clear_session_pool():
    """Destroy every pooled training session core (captured graphs and device buffers).  Must not
    run while a stream capture is in progress on the device."""
    with _pool_lock:
        cores = list(_pool.values())
        _pool.clear()
    _release(cores)


_pool_clear = clear_session_pool   # earlier name, kept for the tests and tools that use it


def _pool_put(key, core):
    """Pool an idle core (False if its key already holds one); evicts LRU cores over the caps."""
    evicted = []
    with _pool_lock:
        if key in _pool:
            return False
        _pool[key] = core
        total = sum(c.nbytes for c in _pool.values())
        while len(_pool) > _POOL_MAX_ENTRIES or (total > _POOL_MAX_BYTES and len(_pool) > 1):
            _, old = _pool.popitem(last=False)
            total -= old.nbytes
            evicted.append(old)
    _release(evicted)
    return True


def _pool_take(key):
    with _pool_lock:
        return _pool.pop(key, None)


atexit.register(lambda: release_retired_graphs())
atexit.register(clear_session_pool)
Engine._mode_listeners.append(lambda eng: clear_session_pool())


# ---------------------------------------------------------------- retired step graphs
# The captured step graphs of a closed, released or dropped session are not destroyed before the
# interpreter exits; they are kept here (no buffers: a graph holds no reference to the tensors it
# was captured on).  Reason: in the HIP runtime this image ships (libamdhip64 of
# ROCm 7.0.2, GPU_MAX_HW_QUEUES = 4), instantiating a graph with parallel branches (the fp32
# lookahead's and the SVGP gradient's fork / join) acquires hardware queues for its internal branch
# streams, shared by reference count with user streams; destroying such a graph exec after a later
# user stream came to share one of those queues made the next hipGraphLaunch on it segfault
# (tools/graph_lifetime_probe.py small_graphs_after: the fifth session's first replay, every run,
# with AMD_LOG_LEVEL=3 showing the exec's releaseQueue on the queue the new session's stream
# holds; never with the graphs kept).  A retired graph costs its exec's host nodes and kernel
# arguments (a few hundred KB at the Synth size); release_retired_graphs() frees them when the
# caller knows that no captured graph will be launched again in the process.
_retired_graphs: list = []


def _retire_graphs(graphs: dict):
    if graphs:
        _retired_graphs.extend(graphs.values())
        graphs.clear()


def release_retired_graphs():
    """Destroy the retired step graphs now (see above: only when no captured graph is launched in
    this process afterwards).  Returns how many were destroyed."""
    n = len(_retired_graphs)
    if n and torch.cuda.is_available():
        torch.cuda.synchronize()
    _retired_graphs.clear()
    return n


class _AdamCore:
    """Every buffer an AdamSession's recorded graphs point at (session-owned copies of X and Y,
    the Adam state, loss history, output, info, private workspace), its stream and its graphs."""

    def __init__(self, eng: Engine, X: torch.Tensor, Y: torch.Tensor, tm: "_ThetaMap", lr: float,
                 max_iters: int):
        self.eng = eng
        self.stream = torch.cuda.Stream(eng.device)
        self.stream.wait_stream(torch.cuda.current_stream(eng.device))
        self.graphs = {}
        with torch.cuda.stream(self.stream):
            self.X = torch.empty_like(X)
            self.Y = torch.empty_like(Y)
            self.st = AdamState(eng.device, tm.u(), tm.trainable(), tm.tie(), lr)
            G = self.st.u.numel()
            # the whole per-model state as typed views of ONE byte buffer -- u | m | v (f64), tie
            # (i32), step | info (i32), trainable (u8) -- written by ONE pinned host-to-device copy
            # per load (u, tie, trainable from the model, zero moments and counters); the results
            # come back in ONE device-to-host copy (fewer launches and synchronising transfers on
            # the HBS protocol)
            b = 8 * max_iters   # the loss history first: finish() reads hist | u | ... | si as one range
            self._off = o = {"hist": 0, "u": b, "m": b + 8 * G, "v": b + 16 * G, "tie": b + 24 * G,
                             "si": b + 28 * G, "tr": b + 28 * G + 8, "end": b + 29 * G + 8}
            self.d_in = torch.zeros((o["end"],), dtype=torch.uint8, device=eng.device)
            self.h_in = torch.zeros((o["end"],), dtype=torch.uint8, pin_memory=True)
            self.st.u = self.d_in[o["u"]:o["m"]].view(torch.float64)
            self.st.m = self.d_in[o["m"]:o["v"]].view(torch.float64)
            self.st.v = self.d_in[o["v"]:o["tie"]].view(torch.float64)
            self.st.tie = self.d_in[o["tie"]:o["si"]].view(torch.int32)
            self.si = self.d_in[o["si"]:o["tr"]].view(torch.int32)
            self.st.step = self.si[0:1]
            self.info = self.si[1:2]
            self.st.trainable = self.d_in[o["tr"]:o["end"]]
            self.hist = self.d_in[o["hist"]:o["u"]].view(torch.float64)
            self.h_out = torch.empty((o["tr"],), dtype=torch.uint8, pin_memory=True)
            self.out = torch.empty((1 + theta_size(tm.d),), dtype=torch.float64, device=eng.device)
            n, p, d = X.shape[0], Y.shape[1], tm.d
            self.ws_bytes = eng.gpr_workspace_bytes(n, p, d, X.dtype)
            self.ws = eng.private_workspace(self.ws_bytes)
        self.nbytes = self.ws_bytes + 2 * o["end"] + X.numel() * X.element_size() + Y.numel() * Y.element_size()
        self.warm = False

    def __del__(self):
        _retire_graphs(getattr(self, "graphs", None))

    def release(self):
        """Retire the captured graphs and drop every buffer (an evicted or cleared pool entry)."""
        _retire_graphs(self.graphs)
        self.X = self.Y = self.st = self.ws = self.d_in = self.h_in = self.h_out = None
        self.hist = self.si = self.info = self.out = None

    def load(self, X: torch.Tensor, Y: torch.Tensor, tm: "_ThetaMap"):
        """A model's data and initial state into the buffers (on the core's stream)."""
        st = self.st
        o = self._off
        self.X.copy_(X)
        self.Y.copy_(Y)
        h = self.h_in.numpy()   # the previous load's copy from it completed before that session finished
        h[o["u"]:o["m"]].view(np.float64)[:] = tm.u()
        h[o["m"]:o["tie"]] = 0                                  # moments
        h[o["tie"]:o["si"]].view(np.int32)[:] = tm.tie()
        h[o["si"]:o["tr"]] = 0                                  # step, info
        h[o["tr"]:o["end"]] = np.asarray(tm.trainable()).astype(np.uint8)
        self.d_in.copy_(self.h_in, non_blocking=True)
        self.eng.theta_from_u(st.u, st.theta, tm.noise_index)
        if not self.warm:
            # one eager evaluation before any capture: builds the schedule tables and sets every
            # step kernel's launch attributes; value + gradient, as the step (on the fp32 path a
            # value-only call would also run the fp64 refinement, which the step never does)
            self.eng.gpr_lml(self.X, self.Y, st.theta, want_grad=True, ws=self.ws)
            self.warm = True


def _pool_key(eng, X, Y, lr, max_iters, chunk):
    return (eng.index, eng.mode(), X.dtype, tuple(X.shape), tuple(Y.shape), float(np.float32(lr)), int(max_iters),
            int(chunk))


class AdamSession:
    """Runs MultiFidelityGPModel Adam iterations on the device.

    State (unconstrained u, moments, step counter, loss history) lives in HBM; each
    iteration is ONE mfgp_gpr_adam_step call (≈T+6 kernel launches), replayed from
    hipGraphs of `graph_chunk` iterations on a dedicated stream.  The host only
    syncs when asked (progress prints, finish).  finish() hands the buffers and graphs to the
    session pool, so the next session of the same shape replays them without a capture."""

    def __init__(self, model: "MultiFidelityGPModel", lr: float, max_iters: int, graph: bool, chunk: int):
        self.model = model
        self.eng, Xm, Ym = model._device_data()
        self.tm = model._theta_map()
        self.max_iters = max(int(max_iters), 1)
        chunk = chunk if graph else 0
        self._key = _pool_key(self.eng, Xm, Ym, lr, self.max_iters, chunk)
        core = _pool_take(self._key) if chunk else None
        if core is None:
            core = _AdamCore(self.eng, Xm, Ym, self.tm, lr, self.max_iters)
        self._core = core
        self.stream, self.st, self.hist, self.out = core.stream, core.st, core.hist, core.out
        self.info, self.ws, self.X, self.Y = core.info, core.ws, core.X, core.Y
        # every buffer the recorded graphs point at is owned by the core (no shared grow-only
        # workspace under a graph); loading is ordered on its stream after the caller's work
        core.stream.wait_stream(torch.cuda.current_stream(self.eng.device))
        with torch.cuda.stream(self.stream), self.eng.ordered(self.stream):
            core.load(Xm, Ym, self.tm)
        self.done = 0
        self.runner = _StepRunner(self._step, chunk, graphs=core.graphs)

    def _step(self):
        # the session's private workspace is written by its own steps only (and its warm-up, a
        # value+grad call): each step leaves it set up for the next (mfgp_set_resident)
        with self.eng.resident():
            self.eng.gpr_adam_step(self.X, self.Y, self.st, self.hist, self.out, self.info, ws=self.ws)

    def run(self, n: int):
        if self._core is None:
            raise MFGPError("AdamSession: the session is finished")
        if self.done + n > self.max_iters:
            raise ValueError("AdamSession: more iterations than max_iters")
        if self.eng.mode() != self._key[1]:
            # the session's graphs and workspace belong to the settings it started under; a step
            # captured now would run another schedule on them
            raise MFGPError("AdamSession: the engine's tile / flow / tiny settings changed during the session")
        with torch.cuda.stream(self.stream), self.eng.ordered(self.stream):
            self.runner.run(n)
        self.done += n

    def prepare(self, n: int):
        """Capture the step graphs a later run(n) replays (nothing executes)."""
        with torch.cuda.stream(self.stream):
            self.runner.prepare(n)

    def sync(self):
        self.stream.synchronize()

    def loss_at(self, i: int) -> float:
        self.sync()
        return float(self.hist[i].item())

    def close(self):
        """Release the recorded step graphs now (a later run re-captures)."""
        self.runner.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _retire(self):
        """Hand the core (buffers + graphs) to the pool, or release the graphs now.  Either way
        this finished session drops its aliases of the core's buffers: a pooled core is reloaded
        and overwritten by the next session of its shape."""
        core, self._core = self._core, None
        if core is None:
            return
        self.st = self.hist = self.out = self.info = self.ws = self.X = self.Y = None
        if self.runner.chunk and self.runner.graphs and core.ws_bytes <= _POOL_MAX_WS_BYTES:
            # this finished session must never touch the pooled graphs again (a close() from it
            # could destroy them while their next user captures)
            runner, self.runner = self.runner, _StepRunner(self._step, 0)
            if _pool_put(self._key, core):
                return
            runner.close()
            return
        self.close()

    def finish(self):
        n, G, core = self.done, self.st.u.numel(), self._core
        if core is None:
            raise MFGPError("AdamSession: the session is finished")
        o = core._off
        with torch.cuda.stream(self.stream):   # loss history, u, step and info: one byte range, one copy
            core.h_out.copy_(core.d_in[:o["tr"]], non_blocking=True)
        self.sync()
        res = core.h_out.numpy()
        h = res[o["hist"]:o["u"]].view(np.float64)[:n].copy()
        self.model.loss_history = [np.float64(v) for v in h]
        self.tm.set_u(res[o["u"]:o["m"]].view(np.float64).copy())
        si = res[o["si"]:o["tr"]].view(np.int32)
        steps, v = int(si[0]), int(si[1])
        self._retire()
        if v == 0 and steps != self.done and np.all(np.isfinite(h)):
            # a failed step leaves the step counter behind and the next one retries it, so a
            # failure followed by good steps shows only here (trailing loss entries never written)
            raise MFGPError(f"optimize: {self.done - steps} of {self.done} steps failed (Cholesky or flow "
                            f"hand-off) and were retried; the trajectory is incomplete")
        if v != 0 or not np.all(np.isfinite(h)):
            bad = int(np.argmax(~np.isfinite(h))) if not np.all(np.isfinite(h)) else len(h) - 1
            self.model.loss_history = self.model.loss_history[:bad + 1]
            if v == MFGP_FLOW_TIMEOUT:
                raise info_error(v, f"optimize (by iteration {bad})")
            raise CholeskyError(f"optimize: Cholesky failed at iteration {bad}")


class _StepRunner:
    """Runs a step function n times: eagerly, or replaying a hipGraph of `chunk`
    captured steps (torch.cuda.CUDAGraph is the HIP graph API on ROCm).

    Graph lifetime is deterministic: the runner holds its session's step method weakly (no
    session <-> runner reference cycle), so a session and its hipGraphExecs are freed by
    reference counting the moment the last reference goes, or at close() -- never by a cyclic
    collection that could run in the middle of another session's capture (destroying a graph
    while a stream captures is illegal and aborts the process)."""

    def __init__(self, step, chunk: int, graphs: dict = None):
        self._step = weakref.WeakMethod(step) if hasattr(step, "__self__") else (lambda f=step: f)
        self.chunk = chunk
        self._owns = graphs is None
        self.graphs = {} if graphs is None else graphs

    def step(self):
        fn = self._step()
        if fn is None:
            raise MFGPError("the training session of this step runner was released")
        fn()

    def close(self):
        """Release the captured graphs now (retired until exit, see release_retired_graphs)."""
        _retire_graphs(self.graphs)

    def __del__(self):
        # a dropped runner's own graphs are retired too, not destroyed by reference counting (a
        # session's graphs belong to its _AdamCore, which retires them itself)
        if getattr(self, "_owns", False):
            _retire_graphs(self.graphs)

    def _graph(self, n):
        g = self.graphs.get(n)
        if g is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    self.step()
            self.graphs[n] = g
        return g

    def prepare(self, n: int):
        """Capture (without running) every graph that run(n) will replay, so a later
        run(n) is replay-only (bench.py captures before its timed region)."""
        if self.chunk <= 0 or n < 4:
            return
        full, rem = divmod(n, self.chunk)
        if full:
            self._graph(self.chunk)
        if rem >= 4:
            self._graph(rem)

    def run(self, n: int):
        if self.chunk <= 0 or n < 4:
            for _ in range(n):
                self.step()
            return
        full, rem = divmod(n, self.chunk)
        for _ in range(full):
            self._graph(self.chunk).replay()
        if rem:
            if rem < 4:
                for _ in range(rem):
                    self.step()
            else:
                self._graph(rem).replay()
