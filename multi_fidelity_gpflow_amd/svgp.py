"""Sparse variational multi-fidelity emulators (value path on the MI355X engine).

* ``LatentMFCoregionalizationSVGP`` — mfgpflow/linear_svgp.py:64-221: L latent
  LinearMultiFidelityKernels mixed by W (LinearCoregionalization), KMeans
  inducing points, whitened q(u).
* ``SingleBinSVGP`` — mfgpflow/singlebin_svgp.py:13-135: one LinearMultiFidelityKernel
  per output bin (SeparateIndependent), q_sqrt = 0.1 I.

``elbo``, ``prior_kl`` and ``predict_f`` run in libmfgp.so (mfgp_svgp_elbo /
mfgp_svgp_predict: batched K_uu factor, fused K_uf K_uu^{-1} products, mixing,
variational expectations, KL).  ``optimize`` runs the analytic ELBO
gradient (mfgp_svgp_elbo_grad) and a packed Keras-Adam step (mfgp_adam_packed) per
iteration, replayed from hipGraphs; all state stays in HBM (_SVGPTrainer).
"""
from __future__ import annotations

import copy
import pickle

import numpy as np
import torch

from .engine import Engine, theta_size, to_dev
from .kernels import LinearCoregionalization, LinearMultiFidelityKernel, SeparateIndependent
from ._lib import MFGPError
from .models import CholeskyError, Gaussian, _StepRunner
from .params import Module, Parameter, Softplus, as_result, parameter_dict, multiple_assign

DEFAULT_JITTER = 1e-6


def initialize_W(output_dim, num_latents, window_fraction=0.3, scale=0.5):
    """Structured diagonal W (P x L) — linear_svgp.py:17-48."""
    W = np.zeros((output_dim, num_latents))
    window = max(int(output_dim * window_fraction), 2)
    stride = max(output_dim // (num_latents - 1), 1) if num_latents > 1 else 1
    for j in range(num_latents):
        center = min(int(j * stride), output_dim - 1)
        for i in range(output_dim):
            dist = abs(i - center)
            if dist < window / 2:
                W[i, j] = np.exp(-0.1 * dist)
    return W * scale


def initialize_W_pca(Y, output_dim, num_latents, perturb=0.01, seed=None):
    """PCA-based W — linear_svgp.py:50-62."""
    from sklearn.decomposition import PCA
    pca = PCA(n_components=num_latents)
    pca.fit(Y)
    W = pca.components_.T
    W = W / np.linalg.norm(W, axis=0)
    rng = np.random if seed is None else np.random.RandomState(seed)
    return W + perturb * rng.randn(*W.shape)


def kmeans_inducing(X, num_inducing, random_state=42):
    """KMeans(n_clusters, random_state=42).fit(X).cluster_centers_ (host, one-time init)."""
    from sklearn.cluster import KMeans
    return KMeans(n_clusters=num_inducing, random_state=random_state).fit(X).cluster_centers_


class _SVGPBase(Module):
    """Shared state: kernel (multi-output), Z, q_mu [M, L], q_sqrt [L, M, M], likelihood."""

    def _setup(self, Z, q_mu, q_sqrt, likelihood, num_data):
        self.inducing_variable = Parameter(np.asarray(Z, dtype=np.float64))
        self.q_mu = Parameter(np.asarray(q_mu, dtype=np.float64))
        self.q_sqrt = Parameter(np.asarray(q_sqrt, dtype=np.float64))
        self.likelihood = likelihood
        self.num_data = num_data
        self.loss_history = []

    @property
    def num_latent_gps(self) -> int:
        return self.q_mu.shape[1]

    def _W(self):
        return None

    def _dev_state(self):
        eng = Engine.get()
        D = self.inducing_variable.shape[1] - 1
        Z = to_dev(self.inducing_variable.numpy(), eng.device)
        thetas = self.kernel.latent_thetas(D, eng.device)
        q_mu = to_dev(self.q_mu.numpy(), eng.device)
        q_sqrt = to_dev(np.tril(self.q_sqrt.numpy()), eng.device)
        W = self._W()
        W = None if W is None else to_dev(W, eng.device)
        return eng, Z, thetas, q_mu, q_sqrt, W

    def _elbo_parts(self, data):
        X, Y = data
        eng, Z, thetas, q_mu, q_sqrt, W = self._dev_state()
        Xd, Yd = to_dev(X, eng.device), to_dev(Y, eng.device)
        scale = (self.num_data / Xd.shape[0]) if self.num_data else 1.0
        out, g_mu, g_var, info = eng.svgp_elbo(Xd, Yd, Z, thetas, q_mu, q_sqrt, W,
                                               float(self.likelihood.variance.numpy()), scale, DEFAULT_JITTER)
        if int(info.max().item()) != 0:
            raise CholeskyError("elbo: Cholesky of K_uu was not successful")
        return out

    def elbo(self, data):
        """GPflow SVGP.elbo: sum of variational expectations (x num_data / N) - KL."""
        return as_result(self._elbo_parts(data)[0].clone())

    def training_loss(self, data):
        return as_result(-self.elbo(data))

    def prior_kl(self):
        """gauss_kl(q_mu, q_sqrt) with the whitened N(0, I) prior."""
        L = np.tril(self.q_sqrt.numpy())
        q = self.q_mu.numpy()
        M, Lat = q.shape
        d = np.diagonal(L, axis1=-2, axis2=-1)
        return 0.5 * (np.sum(q * q) - M * Lat + np.sum(L * L) - np.sum(np.log(d * d)))

    def predict_f(self, Xnew, full_cov=False, full_output_cov=False):
        """GPflow SVGP.predict_f (IndependentPosteriorMultiOutput + mix_latent_gp): mean [N*, P];
        var [N*, P], or with full_cov [P, N*, N*], with full_output_cov [N*, P, P], with both
        [N*, P, N*, P] (linear_svgp.py:64 / singlebin_svgp.py:13 inherit it)."""
        eng, Z, thetas, q_mu, q_sqrt, W = self._dev_state()
        Xs = to_dev(Xnew, eng.device)
        if full_cov or full_output_cov:
            mode = 3 if (full_cov and full_output_cov) else (1 if full_cov else 2)
            f_mu, f_cov, info = eng.svgp_predict_cov(mode, Xs, Z, thetas, q_mu, q_sqrt, W, self.num_outputs,
                                                     DEFAULT_JITTER)
            if int(info.max().item()) != 0:
                raise CholeskyError("predict_f: Cholesky of K_uu was not successful")
            return as_result(f_mu), as_result(f_cov)
        f_mu, f_var, _, _, info = eng.svgp_predict(Xs, Z, thetas, q_mu, q_sqrt, W, self.num_outputs, DEFAULT_JITTER)
        if int(info.max().item()) != 0:
            raise CholeskyError("predict_f: Cholesky of K_uu was not successful")
        return as_result(f_mu), as_result(f_var)

    def predict_y(self, Xnew, full_cov=False, full_output_cov=False):
        """GPflow GPModel.predict_y: predict_f plus the Gaussian noise variance."""
        if full_cov or full_output_cov:
            # GPflow 2.9 GPModel.predict_y (gpflow issue 1461): only the marginal form is supported
            raise NotImplementedError("The predict_y method currently supports only the argument values "
                                      "full_cov=False and full_output_cov=False")
        mean, var = self.predict_f(Xnew)
        return mean, as_result(var + float(self.likelihood.variance.numpy()))

    def elbo_and_grad(self, data, kl_multiplier=1.0):
        """(ELBO, dict of d(VE*scale - kl_multiplier*KL)/d(constrained parameter)) on the device:
        keys 'Z', 'theta' [L, 2d+4] (theta_vector layout), 'q_mu', 'q_sqrt' (lower), 'W', 'noise'."""
        tr = _SVGPTrainer(self, data, max_iters=1, initial_lr=0.0, kl_multiplier=kl_multiplier, graph=False)
        e = tr.elbo_now()
        g = {k: v.cpu().numpy().copy() for k, v in tr.grad_views().items()}
        return e, g

    def _optimize(self, data, max_iters, initial_lr, unfix_noise_after, kl_multiplier, reset_history, graph,
                  graph_chunk, verbose, every, start=0):
        """Iterations start..max_iters-1 with a fresh Adam over CosineDecay(initial_lr, max_iters)
        whose step counter starts at 0 (the reference builds both inside optimize)."""
        n = max_iters - start
        if n <= 0:
            return None
        tr = _SVGPTrainer(self, data, n, initial_lr, kl_multiplier, graph=graph, graph_chunk=graph_chunk,
                          decay_steps=max_iters)
        noise_fixed = not self.likelihood.variance.trainable
        done = 0
        while done < n:
            stop = n
            if noise_fixed and unfix_noise_after is not None and done <= unfix_noise_after < n:
                stop = unfix_noise_after + 1
            if verbose:
                stop = min(stop, done + every)
            tr.run(stop - done)
            done = stop
            if noise_fixed and unfix_noise_after is not None and done == unfix_noise_after + 1:
                tr.set_trainable("noise", True)
                noise_fixed = False
            if verbose:
                print(f"Iteration {start + done - 1}: loss = {tr.loss_at(done - 1)}", flush=True)
        tr.finish(reset_history)
        return tr

    def save_model(self, filename):
        """parameter_dict pickled (linear_svgp.py:206-212) — our own file format."""
        with open(filename, "wb") as f:
            pickle.dump(parameter_dict(self), f)



def cosine_decay_schedule(initial_lr, decay_steps, n):
    """tf.keras.optimizers.schedules.CosineDecay (TF 2.10, alpha = 0) for steps 0..n-1,
    evaluated in float32 like TF (the python-float initial lr is a float32 tensor)."""
    out = np.empty(max(int(n), 1), dtype=np.float64)
    lr0 = np.float32(initial_lr)
    ds = np.float32(max(int(decay_steps), 1))
    for t in range(out.size):
        frac = np.float32(min(t, decay_steps)) / ds
        cosd = np.float32(0.5) * (np.float32(1.0) + np.cos(np.float32(np.pi) * frac, dtype=np.float32))
        out[t] = float(np.float32(lr0 * cosd))
    return out


def _transform_code(p: Parameter) -> int:
    t = p.transform
    if t is None:
        return 0
    if isinstance(t, Softplus) and float(t.lower or 0.0) == 0.0:
        return 1
    if isinstance(t, Softplus) and float(t.lower or 0.0) == 1e-6:
        return 2
    raise NotImplementedError(f"transform {t!r} is not supported by the device Adam step")


class _SVGPTrainer:
    """Device state of one SVGP optimize() call.

    Every trainable quantity lives in ONE packed fp64 buffer of constrained values
    ``c`` (the model's Z / thetas / q_mu / q_sqrt / W / noise are views into it), with
    the unconstrained ``u``, Adam moments, per-entry trainable / transform / tie-span
    bytes, a packed gradient buffer of the same layout (written in place by
    mfgp_svgp_elbo_grad), the float32 CosineDecay schedule and the step counter.  One
    iteration = one gradient call + one mfgp_adam_packed call; iterations are replayed
    from hipGraphs on a dedicated stream."""

    def __init__(self, model, data, max_iters, initial_lr, kl_multiplier=1.0, graph=True, graph_chunk=50,
                 decay_steps=None):
        """max_iters: the iterations this trainer runs; decay_steps (default max_iters): the
        CosineDecay length, whose schedule starts at step 0 for this trainer's first iteration."""
        self.model = model
        self.eng = eng = Engine.get()
        dev = eng.device
        X, Y = data
        Xh = np.ascontiguousarray(np.asarray(X.cpu() if isinstance(X, torch.Tensor) else X, dtype=np.float64))
        Yh = np.ascontiguousarray(np.asarray(Y.cpu() if isinstance(Y, torch.Tensor) else Y, dtype=np.float64))
        if Yh.ndim == 1:
            Yh = Yh[:, None]
        self.klm = float(kl_multiplier)
        self.max_iters = max(int(max_iters), 1)
        Zp = model.inducing_variable
        m, dp1 = Zp.shape
        d = dp1 - 1
        self.d, self.m = d, m
        kernels = model.kernel.kernels
        L = len(kernels)
        G = theta_size(d)
        p = Yh.shape[1]
        self.L, self.G, self.p = L, G, p
        Wp = model.kernel.W if isinstance(model.kernel, LinearCoregionalization) else None
        # ---- packed layout: (name, shape, c, u, trainable, transform, span)
        segs = []
        segs.append(("Z", (m, dp1), Zp.numpy(), Zp.unconstrained_variable, np.full((m, dp1), Zp.trainable), 0, None))
        self._theta_refs = []
        tc = np.zeros((L, G)); tu = np.zeros((L, G)); tt = np.zeros((L, G), bool)
        tf = np.zeros((L, G), np.uint8); ts = np.ones((L, G), np.uint8)
        for l, k in enumerate(kernels):
            refs = [(k.kernel_L.variance, None)]
            refs += [(k.kernel_L.lengthscales, None if k.kernel_L.lengthscales.shape == () else (i,)) for i in range(d)]
            refs += [(k.kernel_delta.variance, None)]
            refs += [(k.kernel_delta.lengthscales, None if k.kernel_delta.lengthscales.shape == () else (i,))
                     for i in range(d)]
            refs += [(k.rho, (0, 0))]
            seen = {}
            for q, (prm, idx) in enumerate(refs):
                cv, uv = prm.numpy(), prm.unconstrained_variable
                tc[l, q] = float(cv if idx is None else cv[idx])
                tu[l, q] = float(uv if idx is None else uv[idx])
                tt[l, q] = prm.trainable
                tf[l, q] = _transform_code(prm)
                key = (id(prm), idx)
                if key in seen:   # tied entry (isotropic lengthscale): follower of the first
                    ts[l, q] = 0
                    ts[l, seen[key]] += 1
                else:
                    seen[key] = q
            tt[l, G - 1] = False   # noise slot of the theta layout is unused here
            self._theta_refs.append(refs)
        segs.append(("theta", (L, G), tc, tu, tt, tf, ts))
        qm = model.q_mu
        segs.append(("q_mu", (m, L), qm.numpy(), qm.unconstrained_variable, np.full((m, L), qm.trainable), 0, None))
        qs = model.q_sqrt
        # q_sqrt as packed lower triangles [L][M(M+1)/2] (row-major (i, j <= i) at i(i+1)/2 + j;
        # mfgp_set_svgp_qs_packed): GPflow's unconstrained variable has no upper half either, and
        # the packed Adam then moves half the bytes
        self._tril = np.tril_indices(m)
        ti, tj = self._tril
        segs.append(("q_sqrt", (L, ti.size), qs.numpy()[:, ti, tj], np.asarray(qs.unconstrained_variable)[:, ti, tj],
                     np.full((L, ti.size), qs.trainable), 0, None))
        if Wp is not None:
            segs.append(("W", (p, L), Wp.numpy(), Wp.unconstrained_variable, np.full((p, L), Wp.trainable), 0, None))
        nv = model.likelihood.variance
        segs.append(("noise", (1,), np.reshape(nv.numpy(), (1,)), np.reshape(nv.unconstrained_variable, (1,)),
                     np.full((1,), nv.trainable), _transform_code(nv), None))
        self.layout = {}
        off = 0
        cs, us, trs, tfs, sps = [], [], [], [], []
        for name, shape, cv, uv, tv, trf, spn in segs:
            size = int(np.prod(shape))
            self.layout[name] = (off, shape)
            off += size
            cs.append(np.asarray(cv, np.float64).reshape(-1))
            us.append(np.asarray(uv, np.float64).reshape(-1))
            trs.append(np.asarray(tv, bool).reshape(-1))
            tfs.append(np.asarray(trf if isinstance(trf, np.ndarray) else np.full(size, trf), np.uint8).reshape(-1))
            sps.append(np.asarray(spn if spn is not None else np.ones(size), np.uint8).reshape(-1))
        self.n = off
        self.stream = torch.cuda.Stream(dev)
        f64 = dict(dtype=torch.float64, device=dev)
        with torch.cuda.stream(self.stream):
            self.X = torch.tensor(Xh, **f64)
            self.Y = torch.tensor(Yh, **f64)
            self.c = torch.tensor(np.concatenate(cs), **f64)
            self.u = torch.tensor(np.concatenate(us), **f64)
            self.g = torch.zeros(self.n, **f64)
            self.mo = torch.zeros(self.n, **f64)
            self.vo = torch.zeros(self.n, **f64)
            self.trainable = torch.tensor(np.concatenate(trs).astype(np.uint8), device=dev)
            self.transform = torch.tensor(np.concatenate(tfs), device=dev)
            self.span = torch.tensor(np.concatenate(sps), device=dev)
            self.step_t = torch.zeros((1,), dtype=torch.int32, device=dev)
            decay = self.max_iters if decay_steps is None else int(decay_steps)
            self.lr = torch.tensor(cosine_decay_schedule(initial_lr, decay, self.max_iters), **f64)
            self.loss_hist = torch.zeros((self.max_iters,), **f64)
            self.kl_hist = torch.zeros((self.max_iters,), **f64)
            self.out = torch.zeros((3,), **f64)
            n = Xh.shape[0]
            self.g_mu = torch.empty((L, n), **f64)
            self.g_var = torch.empty((L, n), **f64)
            self.info = torch.zeros((L,), dtype=torch.int32, device=dev)
            # owned by the trainer for the life of its graphs (not the engine's shared buffer)
            self.ws = eng.private_workspace(eng.svgp_grad_workspace_bytes(n, m, L, p, d))
        self.scale = (model.num_data / n) if model.num_data else 1.0
        self.b1, self.b2 = float(np.float32(0.9)), float(np.float32(0.999))
        self.done = 0
        self.runner = _StepRunner(self._step, graph_chunk if graph else 0)
        if graph:   # size the workspace outside capture
            self.grad()

    def view(self, buf, name):
        off, shape = self.layout[name]
        return buf[off:off + int(np.prod(shape))].view(*shape)

    def grad_views(self):
        """Gradient views by parameter; q_sqrt's unpacked to [L, M, M] (lower part)."""
        g = {k: self.view(self.g, k) for k in self.layout}
        ti, tj = self._tril
        dense = torch.zeros((self.L, self.m, self.m), dtype=torch.float64, device=self.g.device)
        dense[:, torch.as_tensor(ti, device=dense.device), torch.as_tensor(tj, device=dense.device)] = g["q_sqrt"]
        g["q_sqrt"] = dense
        return g

    def grad(self):
        """One gradient evaluation at the current parameters, ordered on the trainer's stream."""
        with torch.cuda.stream(self.stream):
            self._grad()

    def _grad(self):
        c, g = self.c, self.g
        W = self.view(c, "W") if "W" in self.layout else None
        gW = self.view(g, "W") if "W" in self.layout else None
        self.eng.svgp_elbo_grad(self.X, self.Y, self.view(c, "Z"), self.view(c, "theta"), self.view(c, "q_mu"),
                                self.view(c, "q_sqrt"), W, self.view(c, "noise"), self.scale, self.klm,
                                DEFAULT_JITTER, self.out, self.g_mu, self.g_var, self.view(g, "Z"),
                                self.view(g, "theta"), self.view(g, "q_mu"), self.view(g, "q_sqrt"), gW,
                                self.view(g, "noise"), self.info, ws=self.ws, qs_packed=True)

    def _step(self):
        self._grad()
        self.eng.adam_packed(self.u, self.c, self.g, self.mo, self.vo, self.trainable, self.transform, self.span,
                             self.step_t, self.lr, self.b1, self.b2, 1e-7, self.out, self.klm, self.loss_hist,
                             self.kl_hist, info=self.info)

    def run(self, n):
        if self.done + n > self.max_iters:
            raise ValueError("SVGP optimize: more iterations than max_iters")
        with torch.cuda.stream(self.stream):
            self.runner.run(n)
        self.done += n

    def set_trainable(self, name, flag):
        off, shape = self.layout[name]
        with torch.cuda.stream(self.stream):
            self.trainable[off:off + int(np.prod(shape))] = int(bool(flag))
        if name == "noise":
            self.model.likelihood.variance.trainable = bool(flag)

    def sync(self):
        self.stream.synchronize()

    def elbo_now(self):
        """ELBO at the current parameters (one gradient evaluation, synchronised)."""
        self.grad()
        self.sync()
        return float(self.out[0].item())

    def loss_at(self, i):
        self.sync()
        return float(self.loss_hist[i].item())

    def close(self):
        """Release the recorded step graphs now (a later run re-captures)."""
        self.runner.close()

    def finish(self, reset_history=True):
        self.sync()
        self.close()
        model = self.model
        u = self.u.cpu().numpy()

        def seg(name):
            off, shape = self.layout[name]
            return u[off:off + int(np.prod(shape))].reshape(shape)

        model.inducing_variable.unconstrained_variable = seg("Z")
        model.q_mu.unconstrained_variable = seg("q_mu")
        qs = np.array(model.q_sqrt.unconstrained_variable)
        qs[:, self._tril[0], self._tril[1]] = seg("q_sqrt")
        model.q_sqrt.unconstrained_variable = qs
        if "W" in self.layout:
            model.kernel.W.unconstrained_variable = seg("W")
        model.likelihood.variance.unconstrained_variable = np.reshape(seg("noise"), model.likelihood.variance.shape)
        th = seg("theta")
        for l, refs in enumerate(self._theta_refs):
            for q, (prm, idx) in enumerate(refs):
                if idx is None:
                    prm.unconstrained_variable = np.full(prm.shape, th[l, q])
                else:
                    arr = prm.unconstrained_variable.copy()
                    arr[idx] = th[l, q]
                    prm.unconstrained_variable = arr
        h = self.loss_hist[:self.done].cpu().numpy()
        k = self.kl_hist[:self.done].cpu().numpy()
        if reset_history:
            model.loss_history = []
        model.loss_history.extend(np.float64(v) for v in h)
        if hasattr(model, "kl_history"):
            model.kl_history.extend(np.float64(v) for v in k)
        steps = int(self.step_t.item())
        if int(self.info.max().item()) != 0 or not np.all(np.isfinite(h)):
            raise CholeskyError("SVGP optimize: Cholesky of K_uu failed")
        if steps != self.done:
            raise MFGPError(f"SVGP optimize: {self.done - steps} of {self.done} steps failed (Cholesky of K_uu) "
                            f"and were retried; the trajectory is incomplete")


class LatentMFCoregionalizationSVGP(_SVGPBase):
    """mfgpflow/linear_svgp.py:64-151 constructor semantics."""

    def __init__(self, X, Y, kernel_L, kernel_delta, num_latents, num_inducing, num_outputs, use_rho=True,
                 heterosed=False, loss_type='gaussian', w_type='diagonal', window_fraction=0.4, scale=0.2):
        if heterosed:
            raise NotImplementedError("heteroscedastic likelihoods are out of scope (SURVEY §2)")
        self.num_outputs = num_outputs
        self.num_latents = num_latents
        self.loss_type = loss_type
        if w_type == 'pca':
            W = Parameter(initialize_W_pca(np.asarray(Y)[:, :num_outputs], num_outputs, num_latents))
        elif w_type == 'diagonal':
            W = Parameter(initialize_W(num_outputs, num_latents, window_fraction=window_fraction, scale=scale))
        elif w_type == 'fixed_independent':
            W = Parameter(np.eye(num_outputs, num_latents), trainable=False)
        else:
            raise ValueError(f"Unknown w_type: {w_type}. Choose from 'pca', 'diagonal', or 'fixed_independent'.")
        kernels = [LinearMultiFidelityKernel(copy.deepcopy(kernel_L), copy.deepcopy(kernel_delta), num_output_dims=1,
                                             use_rho=use_rho) for _ in range(num_latents)]
        self.kernel = LinearCoregionalization(kernels, W=W)
        Z = kmeans_inducing(np.asarray(X), num_inducing, 42)
        M = Z.shape[0]
        self._setup(Z, np.zeros((M, num_latents)), np.tile(np.eye(M)[None], (num_latents, 1, 1)),
                    Gaussian(variance=1.0), np.asarray(X).shape[0])
        self.kl_history = []

    def _W(self):
        return self.kernel.W.numpy()

    def optimize(self, data, max_iters=10000, initial_lr=0.005, unfix_noise_after=5000, kl_multiplier=1.0,
                 verbose=False, graph=True, graph_chunk=50):
        """linear_svgp.py:153-203: Adam + CosineDecay(initial_lr, max_iters) on
        -ELBO + (kl_multiplier - 1) KL; loss_history / kl_history are appended.  Like the
        reference it RESUMES: the loop is `for i in range(len(self.loss_history), max_iters)`
        (linear_svgp.py:194) with a fresh Adam and a fresh CosineDecay(initial_lr, max_iters) whose
        step counter starts at 0 each call (:169), so a second optimize(max_iters=N) after N steps
        runs none.  (The reference's noise-unfix branch compares loss_type with 'gausssian' and
        never fires: the noise keeps the trainable flag it has.)"""
        self._optimize(data, max_iters, initial_lr, None, kl_multiplier, False, graph, graph_chunk, verbose, 100,
                       start=len(self.loss_history))

    def save_model(self, filename="latent_mf_svgp.pkl"):
        """linear_svgp.py:206-212 (parameter_dict pickled)."""
        super().save_model(filename)

    @staticmethod
    def load_model(filename, *args):
        """linear_svgp.py:214-221: rebuild with the constructor arguments, then
        multiple_assign the saved parameter_dict."""
        with open(filename, "rb") as f:
            params = pickle.load(f)
        model = LatentMFCoregionalizationSVGP(*args)
        multiple_assign(model, params)
        return model


class SingleBinSVGP(_SVGPBase):
    """mfgpflow/singlebin_svgp.py:20-62 constructor semantics (Z values are ignored;
    KMeans is recomputed with Z.shape[0] clusters, singlebin_svgp.py:50-51)."""

    def __init__(self, X, Y, kernel_L, kernel_delta, num_outputs, Z, random_state=42):
        self.num_outputs = num_outputs
        kernels = [LinearMultiFidelityKernel(copy.deepcopy(kernel_L), copy.deepcopy(kernel_delta), num_output_dims=1)
                   for _ in range(num_outputs)]
        self.kernel = SeparateIndependent(kernels)
        Zi = kmeans_inducing(np.asarray(X), np.asarray(Z).shape[0], random_state)
        M = Zi.shape[0]
        self._setup(Zi, np.zeros((M, num_outputs)), np.repeat(np.eye(M)[None], num_outputs, axis=0) * 0.1,
                    Gaussian(), None)

    def optimize(self, data, max_iters=10000, initial_lr=0.01, unfix_noise_after=5000, verbose=False, graph=True,
                 graph_chunk=50):
        """singlebin_svgp.py:64-97: Adam + CosineDecay(initial_lr, max_iters) on -ELBO;
        loss_history restarts; the noise becomes trainable after iteration unfix_noise_after."""
        self._optimize(data, max_iters, initial_lr, unfix_noise_after, 1.0, True, graph, graph_chunk, verbose, 10)

    def save_model(self, filename="svgp_model.pkl"):
        """singlebin_svgp.py:99-110 (parameter_dict pickled)."""
        super().save_model(filename)

    @staticmethod
    def load_model(filename, X, Y, kernel_L, kernel_delta, num_outputs, Z):
        model = SingleBinSVGP(X, Y, kernel_L, kernel_delta, num_outputs, Z)
        with open(filename, "rb") as f:
            multiple_assign(model, pickle.load(f))
        return model
