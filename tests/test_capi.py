"""The C-ABI library loads and exports every symbol include/mfgp.h declares (no GPU needed)."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "mfgp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mfgp_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from multi_fidelity_gpflow_amd import _lib
    from multi_fidelity_gpflow_amd.build import build_lib
    build_lib()
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    names = _declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/mfgp.h but not exported"


def test_python_binding_covers_header(lib):
    from multi_fidelity_gpflow_amd._lib import SIGNATURES
    assert set(SIGNATURES) == set(_declared())


def test_library_built_from_checked_out_sources(lib):
    """Build provenance: the library carries the hash of the sources it was compiled
    from, and it is the hash of csrc/ + include/mfgp.h as checked out now."""
    from multi_fidelity_gpflow_amd import _lib
    from multi_fidelity_gpflow_amd.build import built_id, source_hash
    assert lib.mfgp_build_id().decode() == source_hash() == built_id()
    _lib.check_provenance()


def test_host_only_entry_points(lib):
    assert lib.mfgp_version() >= 100
    assert lib.mfgp_error_string(-2).decode() == "workspace too small"
    h = C.c_void_p()
    assert lib.mfgp_create(0, C.byref(h)) == 0
    assert lib.mfgp_get_tile(h) in (32, 64)
    assert lib.mfgp_set_tile(h, 48) == -1
    assert lib.mfgp_set_tile(h, 64) == 0 and lib.mfgp_get_tile(h) == 64
    sz = C.c_size_t()
    assert lib.mfgp_gpr_workspace_size(h, 1164, 64, 10, C.byref(sz)) == 0
    # A (npad^2) + R + Xo (npad x (npad+ppad)) dominate: > 30 MB at Goku
    assert sz.value > 30e6
    assert lib.mfgp_gpr_workspace_size(h, 1164, 64, 33, C.byref(sz)) == -4    # d > 32 rejected
    assert lib.mfgp_svgp_workspace_size(h, 1164, 300, 15, 64, 10, C.byref(sz)) == 0
    # argument validation happens before any device work
    assert lib.mfgp_gpr_lml(h, 0, 1, 1, None, 2, None, 1, None, 0, None, 0, None, None) == -1
    assert lib.mfgp_mf_gram(h, 4, 4, 1, None, 2, None, 2, None, 0.0, None, 4) == -1
    # dtype-generic forms: MFGP_F64 (0) is the fp64 entry, MFGP_F32 (1) the fp32 tall-matrix layout
    s64, s32 = C.c_size_t(), C.c_size_t()
    assert lib.mfgp_gpr_workspace_size_ex(h, 0, 1164, 64, 10, C.byref(s64)) == 0
    assert lib.mfgp_gpr_workspace_size(h, 1164, 64, 10, C.byref(sz)) == 0 and s64.value == sz.value
    assert lib.mfgp_gpr_workspace_size_ex(h, 1, 18432, 512, 10, C.byref(s32)) == 0
    # the value-only refinement layout (default on): M = (T + Tp) x 128 rows + the L^T tiles + fp64
    # alpha / residual = 2.95 GB at the Synth config; without it, the gradient layout M = (T + Tp + T)
    # x 128 rows of Npad floats (K, Y^T, identity rows) = 2.76 GB
    assert 2.9e9 < s32.value < 3.0e9
    assert lib.mfgp_set_f32_refine(h, 3) == -1 and lib.mfgp_set_f32_refine(h, 0) == 0
    assert lib.mfgp_gpr_workspace_size_ex(h, 1, 18432, 512, 10, C.byref(s32)) == 0
    assert 2.7e9 < s32.value < 2.9e9
    assert lib.mfgp_set_f32_refine(h, 1) == 0
    assert lib.mfgp_gpr_workspace_size_ex(h, 2, 1164, 64, 10, C.byref(sz)) == -1     # unknown dtype
    assert lib.mfgp_gpr_lml_ex(h, 1, 0, 1, 1, None, 2, None, 1, None, 0, None, 0, None, None) == -1
    assert lib.mfgp_set_f32_panel(h, 0) == -1 and lib.mfgp_set_f32_panel(h, 6) == 0
    assert lib.mfgp_set_f32_reserve(h, -1) == -1 and lib.mfgp_set_f32_reserve(h, 32) == 0
    assert lib.mfgp_destroy(h) == 0


def test_flow_fence_nests_and_is_bounded(lib, monkeypatch):
    """mfgp_flow_fence: a thread's nested WAIT / RECORD brackets release the fence only
    at the outermost RECORD; another thread that finds it held waits at most the bound
    (MFGP_FENCE_BOUND_MS here) and gets MFGP_ERR_FENCE (-5) instead of blocking for ever.  Host
    logic only: with no GPU the event wait / record are no-ops."""
    import threading
    import time
    monkeypatch.setenv("MFGP_FENCE_BOUND_MS", "150")
    WAIT, RECORD = 0, 1
    ha, hb = C.c_void_p(), C.c_void_p()
    assert lib.mfgp_create(0, C.byref(ha)) == 0 and lib.mfgp_create(0, C.byref(hb)) == 0
    out = {}

    def other(key):
        t0 = time.perf_counter()
        rc = lib.mfgp_flow_fence(hb, WAIT)
        if rc == 0:
            lib.mfgp_flow_fence(hb, RECORD)
        out[key] = (rc, time.perf_counter() - t0)

    try:
        assert lib.mfgp_flow_fence(ha, WAIT) == 0
        assert lib.mfgp_flow_fence(ha, WAIT) == 0          # nested hold of the same thread
        assert lib.mfgp_flow_fence(ha, RECORD) == 0        # inner RECORD: still held
        th = threading.Thread(target=other, args=("held",))
        th.start()
        th.join(5.0)
        assert out["held"][0] == -5 and 0.1 < out["held"][1] < 3.0
        assert lib.mfgp_error_string(-5).decode().startswith("flow fence held")
        assert lib.mfgp_flow_fence(ha, RECORD) == 0        # outermost RECORD releases
        th = threading.Thread(target=other, args=("free",))
        th.start()
        th.join(5.0)
        assert out["free"][0] == 0 and out["free"][1] < 0.1
        assert lib.mfgp_flow_fence(ha, 7) == -1
        assert lib.mfgp_get_tiny(ha) in (0, 1) and lib.mfgp_set_tiny(ha, 0) == 0 and lib.mfgp_get_tiny(ha) == 0
        assert lib.mfgp_get_grad_chunk(ha) >= 1
    finally:
        lib.mfgp_destroy(ha)
        lib.mfgp_destroy(hb)
