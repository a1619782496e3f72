"""Graph-structured multi-fidelity GPR (mfgpflow/graph.py:118-188) on the MI355X engine.

``GraphMultiFidelityGPModel(X, Y, kernel_Ls, kernel_delta)`` — GPR with the
``GraphMultiFidelityKernel`` (m LF sources, learnable LF-LF correlations rho_LF
under a Sigmoid), a Gaussian likelihood of variance 1e-3 that starts non-trainable,
and ``optimize`` by Adam or two-pass L-BFGS like the linear model.

The log-marginal-likelihood, its gradient over every theta entry and predict_f run in
libmfgp.so (mfgp_gmf_gpr_lml / mfgp_gmf_gpr_predict: the tiled Gram + Cholesky path of
the linear model with the graph Gram entry).  Adam iterations are device-resident: one
gradient call plus one mfgp_adam_packed step (Softplus / Sigmoid transforms, tied
isotropic lengthscales) per iteration, replayed from hipGraphs.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import Engine, to_dev
from .kernels import GraphMultiFidelityKernel
from ._lib import MFGP_FLOW_TIMEOUT, MFGPError, info_error
from .models import CholeskyError, Gaussian, _StepRunner
from .params import Module, Sigmoid, Softplus, as_result, set_trainable


def _code(prm) -> int:
    t = prm.transform
    if t is None:
        return 0
    if isinstance(t, Sigmoid):
        return 3
    if isinstance(t, Softplus):
        return 2 if float(t.lower or 0.0) == 1e-6 else 1
    raise NotImplementedError(f"transform {t!r}")


class GraphMultiFidelityGPModel(Module):
    """mfgpflow/graph.py:118-188."""

    def __init__(self, X, Y, kernel_Ls, kernel_delta):
        Xh = np.asarray(X.cpu().numpy() if isinstance(X, torch.Tensor) else X, dtype=np.float64)
        Yh = np.asarray(Y.cpu().numpy() if isinstance(Y, torch.Tensor) else Y, dtype=np.float64)
        if Yh.ndim == 1:
            Yh = Yh[:, None]
        self.num_LF = len(kernel_Ls)
        self.num_output_dims = Yh.shape[1]
        self.kernel = GraphMultiFidelityKernel(kernel_Ls, kernel_delta, self.num_LF, self.num_output_dims)
        self.likelihood = Gaussian(variance=1e-3)
        set_trainable(self.likelihood.variance, False)
        self.data = (Xh, Yh)
        self.loss_history = []
        self._dev = None

    # ------------------------------------------------------------ device state
    def _device_data(self):
        eng = Engine.get()
        if self._dev is None or self._dev[0] is not eng:
            self._dev = (eng, to_dev(self.data[0], eng.device), to_dev(self.data[1], eng.device))
        return self._dev

    def _entries(self):
        d = self.data[0].shape[1] - 1
        return self.kernel.theta_entries(d) + [(self.likelihood.variance, None)]

    def _theta(self):
        vals = []
        for prm, idx in self._entries():
            v = prm.numpy()
            vals.append(float(v if idx is None else np.asarray(v)[idx]))
        return np.array(vals)

    @staticmethod
    def _raise_info(info, what):
        err = info_error(int(info.reshape(-1)[0].item()), what)
        if err is not None:
            raise err

    # ------------------------------------------------------------ GPR surface
    def log_marginal_likelihood(self):
        eng, X, Y = self._device_data()
        th = torch.tensor(self._theta(), dtype=torch.float64, device=eng.device)
        out, info = eng.gmf_lml(self.num_LF, X, Y, th, want_grad=False)
        self._raise_info(info, "log_marginal_likelihood")
        return as_result(out[0].clone())

    def training_loss(self):
        return as_result(-self.log_marginal_likelihood())

    def log_marginal_likelihood_and_grad(self):
        """(LML, dLML/dtheta) over the graph theta layout (include/mfgp.h), numpy."""
        eng, X, Y = self._device_data()
        th = torch.tensor(self._theta(), dtype=torch.float64, device=eng.device)
        out, info = eng.gmf_lml(self.num_LF, X, Y, th, want_grad=True)
        self._raise_info(info, "log_marginal_likelihood")
        o = out.cpu().numpy()
        return float(o[0]), o[1:]

    def predict_f(self, Xnew, full_cov: bool = False, full_output_cov: bool = False):
        """GPR.predict_f(full_cov=False).  (The reference's K(X, Xnew) adds tf.eye(len(X)) and
        fails unless len(Xnew) == len(X); the engine computes K(X, Xnew) without it.)"""
        if full_output_cov:
            raise NotImplementedError("predict_f(full_output_cov=True): GPR has no output covariance to return")
        eng, X, Y = self._device_data()
        Xs = to_dev(Xnew, eng.device)
        th = torch.tensor(self._theta(), dtype=torch.float64, device=eng.device)
        if full_cov:   # [P, N*, N*]; K(X*, X*) carries the kernel's 1e-6 jitter (graph.py:96)
            mean, _, cov, info = eng.gpr_predict_cov(self.num_LF, X, Y, Xs, th)
            self._raise_info(info, "predict_f")
            return as_result(mean), as_result(cov[None].expand(Y.shape[1], -1, -1).contiguous())
        mean, var, info = eng.gmf_predict(self.num_LF, X, Y, Xs, th)
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
    def optimize(self, max_iters=1000, learning_rate=0.01, use_adam=True, unfix_noise_after=500, verbose=False,
                 graph=True, graph_chunk=50):
        """graph.py:143-188.  Adam: the noise keeps its flag (set_trainable inside the python
        loop after tf.function tracing does not reach the traced step, as for the linear
        model); L-BFGS-B: noise fixed, then trainable."""
        self.loss_history = []
        if use_adam:
            sess = _GraphAdamSession(self, learning_rate, max_iters, graph, graph_chunk)
            sess.run(max_iters)
            sess.finish()
        else:
            self._optimize_lbfgs(max_iters)

    def _unique_params(self):
        seen, out = set(), []
        for prm, _ in self._entries():
            if id(prm) not in seen:
                seen.add(id(prm))
                out.append(prm)
        return out

    def _optimize_lbfgs(self, max_iters):
        from scipy.optimize import minimize
        for phase in (0, 1):
            if phase == 1:
                set_trainable(self.likelihood.variance, True)
            params = [p for p in self._unique_params() if p.trainable]
            sizes = [int(np.prod(p.shape)) if p.shape else 1 for p in params]
            ents = self._entries()

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
                for (p, idx), gq in zip(ents, g):
                    if id(p) not in grads:
                        continue
                    if idx is None:
                        grads[id(p)] = grads[id(p)] + gq
                    else:
                        grads[id(p)][idx] += gq
                gu = np.concatenate([(-grads[id(p)] * p.transform.dforward(p.unconstrained_variable)).ravel()
                                     if p.transform else (-grads[id(p)]).ravel() for p in params])
                self.loss_history.append(np.float64(-lml))
                return -lml, gu

            res = minimize(fg, pack(), jac=True, method="L-BFGS-B", options={"maxiter": max_iters})
            unpack(res.x)


class _GraphAdamSession:
    """Keras Adam (constant lr) on the graph theta vector, device-resident: per iteration
    one mfgp_gmf_gpr_lml(want_grad) + one mfgp_adam_packed (Softplus / Sigmoid transforms,
    tied isotropic lengthscales), replayed from hipGraphs on a dedicated stream."""

    def __init__(self, model: GraphMultiFidelityGPModel, lr, max_iters, graph, chunk):
        self.model = model
        self.eng, self.X, self.Y = model._device_data()
        dev = self.eng.device
        ents = model._entries()
        G = len(ents)
        c = np.zeros(G); u = np.zeros(G); tr = np.zeros(G, np.uint8); tf = np.zeros(G, np.uint8)
        span = np.ones(G, np.uint8)
        first = {}
        for q, (prm, idx) in enumerate(ents):
            cv, uv = prm.numpy(), prm.unconstrained_variable
            c[q] = float(cv if idx is None else np.asarray(cv)[idx])
            u[q] = float(uv if idx is None else np.asarray(uv)[idx])
            tr[q] = prm.trainable
            tf[q] = _code(prm)
            key = (id(prm), idx)
            if key in first:
                span[q] = 0
                span[first[key]] += 1
            else:
                first[key] = q
        # rho_LF's diagonal is never used by K (graph.py:62): its gradient is 0 and Adam
        # leaves it; rho[:, 1:] is not in theta at all (only column 0 is used).
        self.ents = ents
        self.max_iters = max(int(max_iters), 1)
        self.stream = torch.cuda.Stream(dev)
        f64 = dict(dtype=torch.float64, device=dev)
        with torch.cuda.stream(self.stream), self.eng.ordered(self.stream):
            self.theta = torch.tensor(c, **f64)
            self.u = torch.tensor(u, **f64)
            self.mo = torch.zeros(G, **f64)
            self.vo = torch.zeros(G, **f64)
            self.trainable = torch.tensor(tr, device=dev)
            self.transform = torch.tensor(tf, device=dev)
            self.span = torch.tensor(span, device=dev)
            self.step = torch.zeros((1,), dtype=torch.int32, device=dev)
            self.lr = torch.full((self.max_iters,), float(np.float32(lr)), **f64)
            self.hist = torch.zeros((self.max_iters,), **f64)
            self.out = torch.zeros((1 + G,), **f64)
            self.info = torch.zeros((1,), dtype=torch.int32, device=dev)
            n, p, d = self.X.shape[0], self.Y.shape[1], self.X.shape[1] - 1
            self.ws = self.eng.private_workspace(self.eng.gmf_workspace_bytes(self.model.num_LF, n, p, d))
            self._lml()   # builds the schedule tables outside capture
        self.b1, self.b2 = float(np.float32(0.9)), float(np.float32(0.999))
        self.done = 0
        self.runner = _StepRunner(self._step, chunk if graph else 0)

    def _lml(self):
        self.eng.gmf_lml(self.model.num_LF, self.X, self.Y, self.theta, want_grad=True, out=self.out, info=self.info,
                         ws=self.ws)

    def _step(self):
        self._lml()
        self.eng.adam_packed(self.u, self.theta, self.out[1:], self.mo, self.vo, self.trainable, self.transform,
                             self.span, self.step, self.lr, self.b1, self.b2, 1e-7, self.out, 1.0, self.hist, None,
                             info=self.info)

    def run(self, n):
        if self.done + n > self.max_iters:
            raise ValueError("optimize: more iterations than max_iters")
        with torch.cuda.stream(self.stream), self.eng.ordered(self.stream):
            self.runner.run(n)
        self.done += n

    def close(self):
        """Release the recorded step graphs now (a later run re-captures)."""
        self.runner.close()

    def finish(self):
        self.stream.synchronize()
        self.close()
        u = self.u.cpu().numpy()
        for (prm, idx), uq in zip(self.ents, u):
            if idx is None:
                prm.unconstrained_variable = np.full(prm.shape, uq)
            else:
                arr = np.array(prm.unconstrained_variable, copy=True)
                arr[idx] = uq
                prm.unconstrained_variable = arr
        h = self.hist[:self.done].cpu().numpy()
        self.model.loss_history = [np.float64(v) for v in h]
        v = int(self.info.item())
        steps = int(self.step.item())
        if v == MFGP_FLOW_TIMEOUT:
            raise info_error(v, "optimize")
        if v == 0 and steps != self.done and np.all(np.isfinite(h)):
            raise MFGPError(f"optimize: {self.done - steps} of {self.done} steps failed and were retried; "
                            f"the trajectory is incomplete")
        if v != 0 or not np.all(np.isfinite(h)):
            raise CholeskyError("optimize: Cholesky failed")
