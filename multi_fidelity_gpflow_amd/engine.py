"""Device engine: torch-ROCm buffers + calls into libmfgp.so (include/mfgp.h).

PyTorch only provides device memory, streams and graphs here; every FLOP of the
hot path runs in the hand-written HIP kernels of ``csrc/``.  There is no CPU
fallback — on a machine without a GPU every compute call raises.
"""
from __future__ import annotations

import contextlib
import ctypes as C

import numpy as np

import torch

from . import _lib
from ._lib import MFGPError, check, ptr


def theta_size(d: int) -> int:
    return 2 * d + 4


def default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise MFGPError("no GPU visible: the MI355X engine has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def to_dev(x, device: torch.device, dtype: torch.dtype = torch.float64) -> torch.Tensor:
    """`dtype` (default float64), contiguous, on `device` (numpy / list / torch accepted)."""
    if isinstance(x, torch.Tensor):
        t = x.detach()
    else:
        t = torch.as_tensor(np.asarray(x, dtype=np.float64))
    return t.to(device=device, dtype=dtype).contiguous()


def dtype_code(t: torch.Tensor) -> int:
    """include/mfgp.h dtype of a data tensor: MFGP_F32 for float32, MFGP_F64 for float64."""
    if t.dtype == torch.float32:
        return _lib.MFGP_F32
    if t.dtype == torch.float64:
        return _lib.MFGP_F64
    raise MFGPError(f"unsupported data dtype {t.dtype} (float64 or float32)")


def resolve_dtype(dtype) -> torch.dtype:
    """Model compute dtype: None / 'float64' / torch.float64 -> float64; 'float32' / torch.float32 -> float32."""
    if dtype is None or dtype in ("float64", "f64", torch.float64, np.float64):
        return torch.float64
    if dtype in ("float32", "f32", torch.float32, np.float32):
        return torch.float32
    raise MFGPError(f"unsupported compute dtype {dtype!r} (float64 or float32)")


class Engine:
    """One per device: owns the library handle binding and grow-only workspaces."""

    _engines: dict = {}

    def __init__(self, device: torch.device):
        self.device = device
        self.index = device.index if device.index is not None else torch.cuda.current_device()
        self._ws: dict = {}
        self.lib = _lib.load()

    @classmethod
    def get(cls, device=None) -> "Engine":
        device = torch.device(device) if device is not None else default_device()
        if device.type != "cuda":
            raise MFGPError(f"MI355X engine needs a GPU device, got {device}")
        key = device.index if device.index is not None else torch.cuda.current_device()
        eng = cls._engines.get(key)
        if eng is None:
            eng = cls(torch.device("cuda", key))
            cls._engines[key] = eng
        return eng

    # ------------------------------------------------------------ session ordering
    @contextlib.contextmanager
    def ordered(self, stream: torch.cuda.Stream):
        """Work enqueued on `stream` inside the block starts after the previous flow-bearing work
        on this device ended (whatever its stream, handle or host thread), and the block's end
        becomes the new last one: the library's device-wide flow fence (include/mfgp.h
        mfgp_flow_fence).  Two persistent k_chol_flow launches must never share the device: each
        needs every CU resident, and one that cannot get them stalls until its hand-off bound
        expires (a lost step).  The library fences every eager flow launch itself; this block is
        for graph replays, whose flows were captured unfenced.  Between WAIT and RECORD this host
        thread holds the fence: a flow launched from another host thread blocks (on the host) until
        the block ends.  No device synchronisation."""
        with torch.cuda.stream(stream):
            check(self.lib.mfgp_flow_fence(self.h, _lib.MFGP_FENCE_WAIT), "mfgp_flow_fence")
        try:
            yield
        finally:
            with torch.cuda.stream(stream):
                check(self.lib.mfgp_flow_fence(self.h, _lib.MFGP_FENCE_RECORD), "mfgp_flow_fence")

    # ------------------------------------------------------------ plumbing
    @property
    def h(self):
        return _lib.handle(self.index)

    def workspace(self, key: str, nbytes: int) -> torch.Tensor:
        buf = self._ws.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(int(nbytes), dtype=torch.uint8, device=self.device)
            self._ws[key] = buf
        return buf

    def _size(self, fn, *args) -> int:
        out = C.c_size_t(0)
        check(fn(self.h, *args, C.byref(out)), fn.__name__)
        return out.value

    # callables run after any change of the handle's execution settings (tile, flow, tiny): the
    # session pool (models.py) drops the cores whose captured graphs recorded the old settings
    _mode_listeners: list = []

    def _set_mode(self, fn, *args):
        before = self.mode()
        check(fn(self.h, *args), fn.__name__)
        if self.mode() != before:
            for cb in list(Engine._mode_listeners):
                cb(self)

    def mode(self) -> tuple:
        """The handle's execution settings that captured step graphs and workspace sizes depend
        on: (flow mode, tile size, one-launch small-problem path, k_grad chunk)."""
        h = self.h
        return (self.lib.mfgp_get_flow(h), self.lib.mfgp_get_tile(h), self.lib.mfgp_get_tiny(h),
                self.lib.mfgp_get_grad_chunk(h))

    def tile(self) -> int:
        return self.lib.mfgp_get_tile(self.h)

    def set_tile(self, nb: int):
        self._set_mode(self.lib.mfgp_set_tile, nb)

    def flow(self) -> bool:
        return self.lib.mfgp_get_flow(self.h) in (1, 3)

    FLOW_MIN_TILES = 8   # mfgp_capi.hip: below this many 32-tiles mode 1 runs the step launches

    def flow_runs(self, n: int) -> bool:
        """Whether an n-point fp64 factorization takes the persistent flow under the current mode."""
        mode = self.lib.mfgp_get_flow(self.h)
        return self.tile() == 32 and (mode == 3 or (mode == 1 and -(-n // 32) >= self.FLOW_MIN_TILES))

    def set_flow(self, enable: bool, any_size: bool = False):
        """Cholesky schedule of the LML path: persistent dataflow launch (True; for factorizations of
        8 or more 32-tiles unless any_size) or one launch per step (False)."""
        self._set_mode(self.lib.mfgp_set_flow, (3 if any_size else 1) if enable else 0)

    def set_tiny(self, enable: bool):
        """One-launch LML step for small problems (n, p <= 64, D <= 16; True, the default) or the
        step sequence of the general path (False)."""
        self._set_mode(self.lib.mfgp_set_tiny, 1 if enable else 0)

    @contextlib.contextmanager
    def resident(self):
        """Value+grad LML calls inside the block may skip the flow's set-up launch when the previous
        fp64 LML call on this thread's handle left their workspace set up for the same problem
        (include/mfgp.h mfgp_set_resident).  For training sessions, whose private workspace nothing
        else writes."""
        if not hasattr(self.lib, "mfgp_set_resident"):   # an older diagnostic build (MFGP_LIB_PATH)
            yield
            return
        check(self.lib.mfgp_set_resident(self.h, 1), "mfgp_set_resident")
        try:
            yield
        finally:
            check(self.lib.mfgp_set_resident(self.h, 0), "mfgp_set_resident")

    def set_flow_timeout_us(self, us: int):
        """Bound of every k_chol_flow hand-off wait (default 50000 us; 0: diagnostic abort path)."""
        check(self.lib.mfgp_set_flow_timeout_us(self.h, int(us)), "mfgp_set_flow_timeout_us")

    # ------------------------------------------------------------ kernels
    def rbf_gram(self, X1: torch.Tensor, X2: torch.Tensor, params: torch.Tensor) -> torch.Tensor:
        n1, d = X1.shape
        n2 = X2.shape[0]
        K = torch.empty((n1, n2), dtype=torch.float64, device=self.device)
        check(self.lib.mfgp_rbf_gram(self.h, n1, n2, d, ptr(X1), d, ptr(X2), X2.shape[1], ptr(params), ptr(K), n2),
              "mfgp_rbf_gram")
        return K

    def mf_gram(self, X1: torch.Tensor, X2: torch.Tensor, theta: torch.Tensor, diag_add: float = 0.0) -> torch.Tensor:
        """K(X1, X2) in X1's dtype (float64: mfgp_mf_gram; float32: mfgp_mf_gram_ex)."""
        n1, dp1 = X1.shape
        n2 = X2.shape[0]
        K = torch.empty((n1, n2), dtype=X1.dtype, device=self.device)
        check(self.lib.mfgp_mf_gram_ex(self.h, dtype_code(X1), n1, n2, dp1 - 1, ptr(X1), dp1, ptr(X2), X2.shape[1],
                                       ptr(theta), float(diag_add), ptr(K), n2), "mfgp_mf_gram_ex")
        return K

    def mf_kdiag(self, X: torch.Tensor, theta: torch.Tensor) -> torch.Tensor:
        n, dp1 = X.shape
        out = torch.empty((n,), dtype=torch.float64, device=self.device)
        check(self.lib.mfgp_mf_kdiag(self.h, n, dp1 - 1, ptr(X), dp1, ptr(theta), ptr(out)), "mfgp_mf_kdiag")
        return out

    def gpr_workspace_bytes(self, n: int, p: int, d: int, dtype: torch.dtype = torch.float64) -> int:
        return self._size(self.lib.mfgp_gpr_workspace_size_ex, dtype_code(torch.empty(0, dtype=dtype)), n, p, d)

    def set_f32_panel(self, tiles: int):
        """fp32 path: 128-wide tile columns per outer Cholesky panel (trailing-update K = 128 * tiles)."""
        check(self.lib.mfgp_set_f32_panel(self.h, int(tiles)), "mfgp_set_f32_panel")

    def set_f32_refine(self, steps):
        """fp32 path: fp64 iterative refinement of the value-only LML (one step) and the predictive
        mean (`steps` steps: True / 2 = the default two, 1, False / 0 = off); gradients and Adam
        steps are never refined.  mfgp_set_f32_refine."""
        steps = 2 if steps is True else 0 if steps is False else int(steps)
        check(self.lib.mfgp_set_f32_refine(self.h, steps), "mfgp_set_f32_refine")

    def set_f32_lookahead(self, enable: bool):
        """fp32 path: factor the next panel on a side stream beside the trailing update (default on)."""
        check(self.lib.mfgp_set_f32_lookahead(self.h, 1 if enable else 0), "mfgp_set_f32_lookahead")

    def set_f32_reserve(self, cus: int):
        """fp32 lookahead: CUs the trailing update leaves to the side stream (0: uncapped)."""
        check(self.lib.mfgp_set_f32_reserve(self.h, int(cus)), "mfgp_set_f32_reserve")

    def private_workspace(self, nbytes: int) -> torch.Tensor:
        """A workspace owned by its caller (a training session keeps it for the life of its
        recorded graphs; the shared grow-only buffers may be replaced under them)."""
        return torch.empty(int(nbytes), dtype=torch.uint8, device=self.device)

    def gpr_lml(self, X, Y, theta, want_grad=False, ws=None, out=None, info=None):
        n, dp1 = X.shape
        p = Y.shape[1]
        d = dp1 - 1
        nbytes = self.gpr_workspace_bytes(n, p, d, X.dtype)
        if ws is None:
            ws = self.workspace("gpr" if X.dtype == torch.float64 else "gpr32", nbytes)
        elif ws.numel() < nbytes:
            raise MFGPError("gpr_lml: private workspace too small")
        if Y.dtype != X.dtype:
            raise MFGPError("gpr_lml: X and Y must share a dtype")
        if out is None:
            out = torch.empty((1 + theta_size(d),), dtype=torch.float64, device=self.device)
        if info is None:
            info = torch.empty((1,), dtype=torch.int32, device=self.device)
        check(self.lib.mfgp_gpr_lml_ex(self.h, dtype_code(X), n, p, d, ptr(X), dp1, ptr(Y), p, ptr(theta),
                                       int(want_grad), ptr(ws), ws.numel(), ptr(out), ptr(info)), "mfgp_gpr_lml_ex")
        return out, info

    def gpr_adam_step(self, X, Y, st: "AdamState", loss_hist: torch.Tensor, out: torch.Tensor, info: torch.Tensor,
                      ws: torch.Tensor = None):
        n, dp1 = X.shape
        p = Y.shape[1]
        d = dp1 - 1
        nbytes = self.gpr_workspace_bytes(n, p, d, X.dtype)
        if ws is None:
            ws = self.workspace("gpr" if X.dtype == torch.float64 else "gpr32", nbytes)
        elif ws.numel() < nbytes:
            raise MFGPError("gpr_adam_step: private workspace too small")
        check(self.lib.mfgp_gpr_adam_step_ex(self.h, dtype_code(X), n, p, d, ptr(X), dp1, ptr(Y), p, ptr(st.theta),
                                             ptr(st.u), ptr(st.m), ptr(st.v), ptr(st.trainable), ptr(st.tie),
                                             ptr(st.step), st.lr, st.b1, st.b2, st.eps, ptr(loss_hist), ptr(ws),
                                             ws.numel(), ptr(out), ptr(info)), "mfgp_gpr_adam_step_ex")

    def theta_from_u(self, u: torch.Tensor, theta: torch.Tensor, noise_index: int):
        check(self.lib.mfgp_theta_from_u(self.h, ptr(u), ptr(theta), u.numel(), noise_index), "mfgp_theta_from_u")

    def gpr_predict(self, X, Y, Xs, theta):
        n, dp1 = X.shape
        p = Y.shape[1]
        d = dp1 - 1
        ns = Xs.shape[0]
        dt = dtype_code(X)
        nbytes = self._size(self.lib.mfgp_gpr_predict_workspace_size_ex, dt, n, p, d, ns)
        ws = self.workspace("pred" if X.dtype == torch.float64 else "pred32", nbytes)
        mean = torch.empty((ns, p), dtype=X.dtype, device=self.device)
        var = torch.empty((ns,), dtype=X.dtype, device=self.device)
        info = torch.empty((1,), dtype=torch.int32, device=self.device)
        check(self.lib.mfgp_gpr_predict_ex(self.h, dt, n, p, d, ns, ptr(X), dp1, ptr(Y), p, ptr(Xs), Xs.shape[1],
                                           ptr(theta), ptr(ws), ws.numel(), ptr(mean), p, ptr(var), ptr(info)),
              "mfgp_gpr_predict_ex")
        return mean, var, info

    def gpr_predict_cov(self, nlf, X, Y, Xs, theta):
        """predict_f(full_cov=True): mean [ns, p], var [ns], cov [ns, ns] in X's dtype (nlf 0: linear
        MF kernel; float32 only for nlf 0)."""
        n, dp1 = X.shape
        p = Y.shape[1]
        d = dp1 - 1
        ns = Xs.shape[0]
        dt = dtype_code(X)
        nbytes = self._size(self.lib.mfgp_gpr_predict_cov_workspace_size_ex, dt, nlf, n, p, d, ns)
        ws = self.workspace("pred_cov" if X.dtype == torch.float64 else "pred_cov32", nbytes)
        mean = torch.empty((ns, p), dtype=X.dtype, device=self.device)
        var = torch.empty((ns,), dtype=X.dtype, device=self.device)
        cov = torch.empty((ns, ns), dtype=X.dtype, device=self.device)
        info = torch.empty((1,), dtype=torch.int32, device=self.device)
        check(self.lib.mfgp_gpr_predict_cov_ex(self.h, dt, nlf, n, p, d, ns, ptr(X), dp1, ptr(Y), p, ptr(Xs),
                                               Xs.shape[1], ptr(theta), ptr(ws), ws.numel(), ptr(mean), p, ptr(var),
                                               ptr(cov), ns, ptr(info)), "mfgp_gpr_predict_cov_ex")
        return mean, var, cov, info

    # ---- GraphMultiFidelityKernel (graph.py) with nlf LF sources
    def gmf_gram(self, nlf, X1, X2, theta, diag_add=0.0):
        n1, dp1 = X1.shape
        n2 = X2.shape[0]
        K = torch.empty((n1, n2), dtype=torch.float64, device=self.device)
        check(self.lib.mfgp_gmf_gram(self.h, nlf, n1, n2, dp1 - 1, ptr(X1), dp1, ptr(X2), X2.shape[1], ptr(theta),
                                     float(diag_add), ptr(K), n2), "mfgp_gmf_gram")
        return K

    def gmf_kdiag(self, nlf, X, theta):
        n, dp1 = X.shape
        out = torch.empty((n,), dtype=torch.float64, device=self.device)
        check(self.lib.mfgp_gmf_kdiag(self.h, nlf, n, dp1 - 1, ptr(X), dp1, ptr(theta), ptr(out)), "mfgp_gmf_kdiag")
        return out

    def gmf_workspace_bytes(self, nlf, n, p, d) -> int:
        return self._size(self.lib.mfgp_gmf_gpr_workspace_size, nlf, n, p, d)

    def gmf_lml(self, nlf, X, Y, theta, want_grad=False, out=None, info=None, ws=None):
        n, dp1 = X.shape
        p = Y.shape[1]
        d = dp1 - 1
        nbytes = self.gmf_workspace_bytes(nlf, n, p, d)
        if ws is None:
            ws = self.workspace("gmf", nbytes)
        elif ws.numel() < nbytes:
            raise MFGPError("gmf_lml: private workspace too small")
        if out is None:
            out = torch.empty((1 + theta.numel(),), dtype=torch.float64, device=self.device)
        if info is None:
            info = torch.empty((1,), dtype=torch.int32, device=self.device)
        check(self.lib.mfgp_gmf_gpr_lml(self.h, nlf, n, p, d, ptr(X), dp1, ptr(Y), p, ptr(theta), int(want_grad),
                                        ptr(ws), ws.numel(), ptr(out), ptr(info)), "mfgp_gmf_gpr_lml")
        return out, info

    def gmf_predict(self, nlf, X, Y, Xs, theta):
        n, dp1 = X.shape
        p = Y.shape[1]
        d = dp1 - 1
        ns = Xs.shape[0]
        nbytes = self._size(self.lib.mfgp_gmf_gpr_predict_workspace_size, nlf, n, p, d, ns)
        ws = self.workspace("gmf_pred", nbytes)
        mean = torch.empty((ns, p), dtype=torch.float64, device=self.device)
        var = torch.empty((ns,), dtype=torch.float64, device=self.device)
        info = torch.empty((1,), dtype=torch.int32, device=self.device)
        check(self.lib.mfgp_gmf_gpr_predict(self.h, nlf, n, p, d, ns, ptr(X), dp1, ptr(Y), p, ptr(Xs), Xs.shape[1],
                                            ptr(theta), ptr(ws), ws.numel(), ptr(mean), p, ptr(var), ptr(info)),
              "mfgp_gmf_gpr_predict")
        return mean, var, info

    def potrf_inv(self, A: torch.Tensor):
        """A: [n, n] or [b, n, n] SPD -> (Linv, diag(L), info[b])."""
        batched = A.dim() == 3
        A3 = A if batched else A.unsqueeze(0)
        A3 = A3.contiguous()
        b, n, _ = A3.shape
        nbytes = self._size(self.lib.mfgp_potrf_inv_workspace_size, n, b)
        ws = self.workspace("potrf", nbytes)
        Linv = torch.empty_like(A3)
        ld = torch.empty((b, n), dtype=torch.float64, device=self.device)
        info = torch.empty((b,), dtype=torch.int32, device=self.device)
        check(self.lib.mfgp_potrf_inv(self.h, n, b, ptr(A3), n, n * n, ptr(ws), ws.numel(), ptr(Linv), n, n * n,
                                      ptr(ld), ptr(info)), "mfgp_potrf_inv")
        if not batched:
            return Linv[0], ld[0], info
        return Linv, ld, info

    def svgp_elbo(self, X, Y, Z, thetas, q_mu, q_sqrt, W, noise, scale, jitter=1e-6):
        n, dp1 = X.shape
        d = dp1 - 1
        p = Y.shape[1]
        m = Z.shape[0]
        L = thetas.shape[0]
        nbytes = self._size(self.lib.mfgp_svgp_workspace_size, n, m, L, p, d)
        ws = self.workspace("svgp", nbytes)
        out = torch.empty((3,), dtype=torch.float64, device=self.device)
        g_mu = torch.empty((L, n), dtype=torch.float64, device=self.device)
        g_var = torch.empty((L, n), dtype=torch.float64, device=self.device)
        info = torch.empty((L,), dtype=torch.int32, device=self.device)
        check(self.lib.mfgp_svgp_elbo(self.h, n, m, L, p, d, ptr(X), dp1, ptr(Y), p, ptr(Z), Z.shape[1],
                                      ptr(thetas), ptr(q_mu), ptr(q_sqrt), ptr(W), float(noise), float(scale),
                                      float(jitter), ptr(ws), ws.numel(), ptr(out), ptr(g_mu), ptr(g_var),
                                      ptr(info)), "mfgp_svgp_elbo")
        return out, g_mu, g_var, info

    def svgp_grad_workspace_bytes(self, n, m, L, p, d) -> int:
        return self._size(self.lib.mfgp_svgp_grad_workspace_size, n, m, L, p, d)

    def svgp_elbo_grad(self, X, Y, Z, thetas, q_mu, q_sqrt, W, noise, scale, kl_mult, jitter, out, g_mu, g_var,
                       gZ, gtheta, gq_mu, gq_sqrt, gW, gnoise, info, ws=None, qs_packed=False):
        """Gradient of VE*scale - kl_mult*KL w.r.t. the constrained SVGP parameters (all device
        tensors, written in place; noise is a device scalar).  qs_packed: q_sqrt and gq_sqrt are
        packed lower triangles [L, M(M+1)/2] (mfgp_set_svgp_qs_packed), else [L, M, M]."""
        n, dp1 = X.shape
        d = dp1 - 1
        p = Y.shape[1]
        m = Z.shape[0]
        L = thetas.shape[0]
        nbytes = self.svgp_grad_workspace_bytes(n, m, L, p, d)
        if ws is None:
            ws = self.workspace("svgp_grad", nbytes)
        elif ws.numel() < nbytes:
            raise MFGPError("svgp_elbo_grad: private workspace too small")
        h = self.h
        check(self.lib.mfgp_set_svgp_qs_packed(h, 1 if qs_packed else 0), "mfgp_set_svgp_qs_packed")
        try:
            check(self.lib.mfgp_svgp_elbo_grad(h, n, m, L, p, d, ptr(X), dp1, ptr(Y), Y.stride(0), ptr(Z), dp1,
                                               ptr(thetas), ptr(q_mu), ptr(q_sqrt), ptr(W), ptr(noise), float(scale),
                                               float(kl_mult), float(jitter), ptr(ws), ws.numel(), ptr(out),
                                               ptr(g_mu), ptr(g_var), ptr(gZ), ptr(gtheta), ptr(gq_mu), ptr(gq_sqrt),
                                               ptr(gW), ptr(gnoise), ptr(info)), "mfgp_svgp_elbo_grad")
        finally:
            check(self.lib.mfgp_set_svgp_qs_packed(h, 0), "mfgp_set_svgp_qs_packed")

    def adam_packed(self, u, c, g, m, v, trainable, transform, span, step, lr_sched, b1, b2, eps, out, kl_mult,
                    loss_hist, kl_hist, info=None):
        """One packed Keras-Adam step; with `info` (the evaluation's int32 info words) a failed
        evaluation leaves the parameters and the step counter unchanged (mfgp_adam_packed_ex)."""
        check(self.lib.mfgp_adam_packed_ex(self.h, u.numel(), ptr(u), ptr(c), ptr(g), ptr(m), ptr(v), ptr(trainable),
                                           ptr(transform), ptr(span), ptr(step), ptr(lr_sched), float(b1), float(b2),
                                           float(eps), ptr(out), float(kl_mult), ptr(loss_hist), ptr(kl_hist),
                                           ptr(info), 0 if info is None else info.numel()),
              "mfgp_adam_packed_ex")

    def svgp_predict(self, Xs, Z, thetas, q_mu, q_sqrt, W, p, jitter=1e-6):
        ns, dp1 = Xs.shape
        d = dp1 - 1
        m = Z.shape[0]
        L = thetas.shape[0]
        nbytes = self._size(self.lib.mfgp_svgp_workspace_size, ns, m, L, p, d)
        ws = self.workspace("svgp_pred", nbytes)
        g_mu = torch.empty((L, ns), dtype=torch.float64, device=self.device)
        g_var = torch.empty((L, ns), dtype=torch.float64, device=self.device)
        f_mu = torch.empty((ns, p), dtype=torch.float64, device=self.device)
        f_var = torch.empty((ns, p), dtype=torch.float64, device=self.device)
        info = torch.empty((L,), dtype=torch.int32, device=self.device)
        check(self.lib.mfgp_svgp_predict(self.h, ns, m, L, p, d, ptr(Xs), dp1, ptr(Z), Z.shape[1], ptr(thetas),
                                         ptr(q_mu), ptr(q_sqrt), ptr(W), float(jitter), ptr(ws), ws.numel(),
                                         ptr(g_mu), ptr(g_var), ptr(f_mu), ptr(f_var), ptr(info)),
              "mfgp_svgp_predict")
        return f_mu, f_var, g_mu, g_var, info

    def svgp_predict_cov(self, mode, Xs, Z, thetas, q_mu, q_sqrt, W, p, jitter=1e-6):
        """SVGP predict_f covariance forms (include/mfgp.h mfgp_svgp_predict_cov): mode 1 full_cov
        -> f_cov [p, ns, ns]; 2 full_output_cov -> [ns, p, p]; 3 both -> [ns, p, ns, p]."""
        ns, dp1 = Xs.shape
        d = dp1 - 1
        m = Z.shape[0]
        L = thetas.shape[0]
        nbytes = self._size(self.lib.mfgp_svgp_predict_cov_workspace_size, ns, m, L, p, d)
        ws = self.workspace("svgp_pred_cov", nbytes)
        f64 = dict(dtype=torch.float64, device=self.device)
        g_mu, g_var = torch.empty((L, ns), **f64), torch.empty((L, ns), **f64)
        f_mu, f_var = torch.empty((ns, p), **f64), torch.empty((ns, p), **f64)
        shape = {1: (p, ns, ns), 2: (ns, p, p), 3: (ns, p, ns, p)}[mode]
        f_cov = torch.empty(shape, **f64)
        info = torch.empty((L,), dtype=torch.int32, device=self.device)
        check(self.lib.mfgp_svgp_predict_cov(self.h, mode, ns, m, L, p, d, ptr(Xs), dp1, ptr(Z), Z.shape[1],
                                             ptr(thetas), ptr(q_mu), ptr(q_sqrt), ptr(W), float(jitter), ptr(ws),
                                             ws.numel(), ptr(g_mu), ptr(g_var), ptr(f_mu), ptr(f_var), ptr(f_cov),
                                             ptr(info)), "mfgp_svgp_predict_cov")
        return f_mu, f_cov, info

    def selftest_mfma(self) -> np.ndarray:
        out = torch.zeros((16, 16), dtype=torch.float64, device=self.device)
        check(self.lib.mfgp_selftest_mfma(self.h, ptr(out)), "mfgp_selftest_mfma")
        return out.cpu().numpy()


class AdamState:
    """Device-resident Keras-Adam state over the unconstrained theta vector."""

    def __init__(self, device, u: np.ndarray, trainable: np.ndarray, tie: np.ndarray, lr: float, b1=0.9, b2=0.999,
                 eps=1e-7):
        f32 = lambda x: float(np.float32(x))   # TF 2.10 OptimizerV2 hyper variables are float32
        self.u = torch.tensor(u, dtype=torch.float64, device=device)
        self.theta = torch.empty_like(self.u)
        self.m = torch.zeros_like(self.u)
        self.v = torch.zeros_like(self.u)
        self.trainable = torch.tensor(trainable.astype(np.uint8), device=device)
        self.tie = torch.tensor(tie.astype(np.int32), device=device)
        self.step = torch.zeros((1,), dtype=torch.int32, device=device)
        self.lr, self.b1, self.b2, self.eps = f32(lr), f32(b1), f32(b2), float(eps)


F32_PHASES = ["gram", "diag", "panel", "update_in", "update_out", "alpha", "grad", "finalize"]


def gpr_phase_times_ex(eng: Engine, X, Y, theta):
    """One value+grad evaluation with hipEvents around every launch (diagnostic).  Returns
    {phase: (ms, flops performed, launches)}: fp32 phases F32_PHASES; fp64 the five of gpr_phase_times."""
    n, dp1 = X.shape
    p = Y.shape[1]
    d = dp1 - 1
    nbytes = eng.gpr_workspace_bytes(n, p, d, X.dtype)
    ws = eng.workspace("gpr" if X.dtype == torch.float64 else "gpr32", nbytes)
    out = torch.empty((1 + theta_size(d),), dtype=torch.float64, device=eng.device)
    info = torch.empty((1,), dtype=torch.int32, device=eng.device)
    k = len(F32_PHASES)
    ms, fl, la = (C.c_float * k)(), (C.c_double * k)(), (C.c_int * k)()
    check(eng.lib.mfgp_gpr_phase_times_ex(eng.h, dtype_code(X), n, p, d, ptr(X), dp1, ptr(Y), p, ptr(theta), ptr(ws),
                                          ws.numel(), ptr(out), ptr(info), ms, fl, la, k), "mfgp_gpr_phase_times_ex")
    names = F32_PHASES if X.dtype == torch.float32 else ["pre", "gram", "chol_steps", "grad", "finalize"]
    return {nm: (float(ms[i]), float(fl[i]), int(la[i])) for i, nm in enumerate(names)}


def gpr_phase_times(eng: Engine, X, Y, theta):
    """Per-phase device times (ms) of one value+grad evaluation, measured with
    hipEvents on the launch stream: [pre, gram, chol_steps (+alpha), grad, finalize]."""
    n, dp1 = X.shape
    p = Y.shape[1]
    d = dp1 - 1
    nbytes = eng._size(eng.lib.mfgp_gpr_workspace_size, n, p, d)
    ws = eng.workspace("gpr", nbytes)
    out = torch.empty((1 + theta_size(d),), dtype=torch.float64, device=eng.device)
    info = torch.empty((1,), dtype=torch.int32, device=eng.device)
    ms = (C.c_float * 5)()
    check(eng.lib.mfgp_gpr_lml_phase_times(eng.h, n, p, d, ptr(X), dp1, ptr(Y), p, ptr(theta), ptr(ws), ws.numel(),
                                           ptr(out), ptr(info), ms), "mfgp_gpr_lml_phase_times")
    return [float(v) for v in ms]
