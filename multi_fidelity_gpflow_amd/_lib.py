"""ctypes binding of libmfgp.so — the C-ABI declared in include/mfgp.h.

The shared library is built in-tree (``multi_fidelity_gpflow_amd/libmfgp.so``)
by :func:`multi_fidelity_gpflow_amd.build.build_lib`.  There is no CPU
fallback: if the library or a GPU is missing, every compute entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmfgp.so")

_p = C.c_void_p
_i = C.c_int
_l = C.c_long
_d = C.c_double
_sz = C.c_size_t

# name -> argtypes (restype is int everywhere except noted)
SIGNATURES = {
    "mfgp_version": [],
    "mfgp_build_id": [],
    "mfgp_error_string": [_i],
    "mfgp_create": [_i, C.POINTER(_p)],
    "mfgp_destroy": [_p],
    "mfgp_set_stream": [_p, _p],
    "mfgp_set_tile": [_p, _i],
    "mfgp_get_tile": [_p],
    "mfgp_set_flow": [_p, _i],
    "mfgp_set_tiny": [_p, _i],
    "mfgp_get_tiny": [_p],
    "mfgp_set_resident": [_p, _i],
    "mfgp_get_grad_chunk": [_p],
    "mfgp_set_f32_refine": [_p, _i],
    "mfgp_get_flow": [_p],
    "mfgp_set_flow_timeout_us": [_p, C.c_longlong],
    "mfgp_flow_fence": [_p, _i],
    "mfgp_gpr_flow_trace": [_p, _i, _i, _i, C.POINTER(C.c_size_t), C.POINTER(_i)],
    "mfgp_rbf_gram": [_p, _i, _i, _i, _p, _i, _p, _i, _p, _p, _i],
    "mfgp_mf_gram": [_p, _i, _i, _i, _p, _i, _p, _i, _p, _d, _p, _i],
    "mfgp_mf_kdiag": [_p, _i, _i, _p, _i, _p, _p],
    "mfgp_gpr_workspace_size": [_p, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_gpr_lml": [_p, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _sz, _p, _p],
    "mfgp_gpr_adam_step": [_p, _i, _i, _i, _p, _i, _p, _i, _p, _p, _p, _p, _p, _p, _p, _d, _d, _d, _d, _p, _p,
                           _sz, _p, _p],
    "mfgp_gpr_lml_phase_times": [_p, _i, _i, _i, _p, _i, _p, _i, _p, _p, _sz, _p, _p, C.POINTER(C.c_float)],
    "mfgp_theta_from_u": [_p, _p, _p, _i, _i],
    "mfgp_gpr_predict_workspace_size": [_p, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_gpr_predict": [_p, _i, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _p, _sz, _p, _i, _p, _p],
    "mfgp_gpr_predict_cov_workspace_size": [_p, _i, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_gpr_predict_cov": [_p, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _p, _sz, _p, _i, _p, _p, _i, _p],
    "mfgp_potrf_inv_workspace_size": [_p, _i, _i, C.POINTER(_sz)],
    "mfgp_potrf_inv": [_p, _i, _i, _p, _i, _l, _p, _sz, _p, _i, _l, _p, _p],
    "mfgp_svgp_workspace_size": [_p, _i, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_svgp_elbo": [_p, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _p, _p, _p, _d, _d, _d, _p, _sz, _p,
                       _p, _p, _p],
    "mfgp_svgp_predict": [_p, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p, _p, _p, _p, _d, _p, _sz, _p, _p, _p, _p,
                          _p],
    "mfgp_svgp_predict_cov_workspace_size": [_p, _i, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_svgp_predict_cov": [_p, _i, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p, _p, _p, _p, _d, _p, _sz, _p, _p, _p,
                              _p, _p, _p],
    "mfgp_svgp_grad_workspace_size": [_p, _i, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_svgp_elbo_grad": [_p, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _p, _p, _p, _p, _d, _d, _d, _p,
                            _sz, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p],
    "mfgp_set_svgp_qs_packed": [_p, _i],
    "mfgp_adam_packed": [_p, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _d, _d, _d, _p, _d, _p, _p],
    "mfgp_adam_packed_ex": [_p, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _d, _d, _d, _p, _d, _p, _p, _p, _i],
    "mfgp_gmf_gram": [_p, _i, _i, _i, _i, _p, _i, _p, _i, _p, _d, _p, _i],
    "mfgp_gmf_kdiag": [_p, _i, _i, _i, _p, _i, _p, _p],
    "mfgp_gmf_gpr_workspace_size": [_p, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_gmf_gpr_lml": [_p, _i, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _sz, _p, _p],
    "mfgp_gmf_gpr_predict_workspace_size": [_p, _i, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_gmf_gpr_predict": [_p, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _p, _sz, _p, _i, _p, _p],
    "mfgp_selftest_mfma": [_p, _p],
    # dtype-generic forms (MFGP_F64 = 0, MFGP_F32 = 1)
    "mfgp_set_f32_panel": [_p, _i],
    "mfgp_set_f32_lookahead": [_p, _i],
    "mfgp_set_f32_reserve": [_p, _i],
    "mfgp_mf_gram_ex": [_p, _i, _i, _i, _i, _p, _i, _p, _i, _p, _d, _p, _i],
    "mfgp_gpr_workspace_size_ex": [_p, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_gpr_lml_ex": [_p, _i, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _sz, _p, _p],
    "mfgp_gpr_adam_step_ex": [_p, _i, _i, _i, _i, _p, _i, _p, _i, _p, _p, _p, _p, _p, _p, _p, _d, _d, _d, _d, _p,
                              _p, _sz, _p, _p],
    "mfgp_gpr_phase_times_ex": [_p, _i, _i, _i, _i, _p, _i, _p, _i, _p, _p, _sz, _p, _p, C.POINTER(C.c_float),
                                C.POINTER(_d), C.POINTER(_i), _i],
    "mfgp_gpr_predict_workspace_size_ex": [_p, _i, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_gpr_predict_ex": [_p, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _p, _sz, _p, _i, _p, _p],
    "mfgp_gpr_predict_cov_workspace_size_ex": [_p, _i, _i, _i, _i, _i, _i, C.POINTER(_sz)],
    "mfgp_gpr_predict_cov_ex": [_p, _i, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p, _i, _p, _p, _sz, _p, _i, _p, _p, _i,
                                _p],
}

MFGP_F64 = 0
MFGP_F32 = 1

_lib = None
_lock = threading.Lock()
_handles = {}


class MFGPError(RuntimeError):
    pass


MFGP_FLOW_TIMEOUT = -100   # include/mfgp.h: info written when a k_chol_flow hand-off stalled
MFGP_FENCE_WAIT = 0        # include/mfgp.h mfgp_flow_fence ops
MFGP_FENCE_RECORD = 1


class FlowTimeoutError(MFGPError):
    """The persistent Cholesky (k_chol_flow) gave up on a stalled hand-off (info = MFGP_FLOW_TIMEOUT):
    a scheduling failure (e.g. another kernel holding CUs, so not every workgroup was resident),
    not a numerical one.  Re-run with the launch-per-step schedule (``Engine.set_flow(False)`` or
    MFGP_FLOW=0)."""


def info_error(v: int, what: str):
    """The exception for a nonzero device info word (None for 0)."""
    if v == 0:
        return None
    if v == MFGP_FLOW_TIMEOUT:
        return FlowTimeoutError(f"{what}: the persistent Cholesky timed out waiting for a hand-off "
                                f"(info {v}); set MFGP_FLOW=0 / Engine.set_flow(False) to use the step schedule")
    from .models import CholeskyError
    return CholeskyError(f"{what}: Cholesky decomposition was not successful "
                         f"(non-positive pivot at row {v}); the input might not be valid.")


def load(path: str = None):
    """Load libmfgp.so (no compute; safe without a GPU).  MFGP_LIB_PATH points at an
    alternative in-tree build (diagnostic A/B of compile-time variants)."""
    global _lib
    path = path or os.environ.get("MFGP_LIB_PATH") or LIB_PATH
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise MFGPError(
                    f"libmfgp.so not found at {path}: build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
            lib = C.CDLL(path)
            variant = path != LIB_PATH   # an older diagnostic build may predate newer entry points
            for name, args in SIGNATURES.items():
                if variant and not hasattr(lib, name):
                    continue
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = C.c_char_p if name in ("mfgp_error_string", "mfgp_build_id") else C.c_int
            _lib = lib
    return _lib


def build_id() -> str:
    """The source hash the loaded library was built from (include/mfgp.h mfgp_build_id)."""
    lib = load()
    return lib.mfgp_build_id().decode() if hasattr(lib, "mfgp_build_id") else "unknown"


def check_provenance():
    """Raise unless the loaded libmfgp.so was built from the sources checked out beside it
    (build.source_hash() of csrc/ + include/mfgp.h).  Diagnostic builds (MFGP_LIB_PATH) pass."""
    from .build import source_hash
    path = os.environ.get("MFGP_LIB_PATH")
    if path and path != LIB_PATH:
        return
    want, got = source_hash(), build_id()
    if got != want:
        raise MFGPError(f"libmfgp.so was built from other sources (build id {got}, sources {want}): "
                        "rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")


def check(code: int, what: str):
    if code != 0:
        msg = load().mfgp_error_string(code).decode()
        raise MFGPError(f"{what} failed: {msg} ({code})")


def handle(device_index: int):
    """Per-(thread, device) library handle bound to torch's current stream."""
    import torch

    lib = load()
    key = (threading.get_ident(), device_index)
    h = _handles.get(key)
    if h is None:
        hp = _p()
        check(lib.mfgp_create(device_index, C.byref(hp)), "mfgp_create")
        h = hp
        _handles[key] = h
    stream = torch.cuda.current_stream(device_index).cuda_stream
    check(lib.mfgp_set_stream(h, _p(stream)), "mfgp_set_stream")
    return h


def ptr(t) -> int:
    """Device address of a torch tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()
