"""Host-side coverage of libmfgp.so without a GPU: every workspace-size query over a sweep of
problem sizes and settings (the layout carves of mfgp_capi.hip / mfgp_svgp*.hip / mfgp_f32.hip),
argument validation of the compute entry points, and the handle settings.  Run as part of the CPU
suite, and under AddressSanitizer by tools/asan_host.sh (a -fsanitize=address host build loaded
through MFGP_LIB_PATH): any out-of-bounds host access in these paths aborts the run."""
import ctypes as C

import pytest
import torch

P = C.c_void_p
SZ = C.c_size_t


@pytest.fixture(scope="module")
def lib():
    from multi_fidelity_gpflow_amd import _lib
    from multi_fidelity_gpflow_amd.build import build_lib
    build_lib()
    return _lib.load()


@pytest.fixture
def h(lib):
    hp = P()
    assert lib.mfgp_create(0, C.byref(hp)) == 0
    yield hp
    assert lib.mfgp_destroy(hp) == 0


SIZES = [(1, 1, 1), (2, 3, 1), (31, 1, 2), (32, 32, 5), (33, 49, 5), (53, 49, 5), (64, 64, 16), (65, 65, 3),
         (255, 7, 10), (256, 64, 10), (1164, 64, 10), (4096, 8, 10), (1, 600, 32)]


def _size(fn, *args):
    out = SZ(0)
    rc = fn(*args, C.byref(out))
    return rc, out.value


@pytest.mark.parametrize("flow", [0, 1, 3])
@pytest.mark.parametrize("tile", [32, 64])
def test_gpr_workspace_sizes(lib, h, flow, tile):
    """mfgp_gpr_* / predict / predict_cov / graph-kernel sizes: positive, monotone in n for fixed
    (p, d), and the flow mode only ever adds space (its publication area, owner table, trace)."""
    assert lib.mfgp_set_tile(h, tile) == 0 and lib.mfgp_set_flow(h, flow) == 0
    prev = {}
    for n, p, d in SIZES:
        rc, g = _size(lib.mfgp_gpr_workspace_size, h, n, p, d)
        assert rc == 0 and g > 8 * n
        rc, g2 = _size(lib.mfgp_gpr_workspace_size_ex, h, 0, n, p, d)
        assert rc == 0 and g2 == g
        for ns in (1, 10, 64, 300):
            rc, pr = _size(lib.mfgp_gpr_predict_workspace_size, h, n, p, d, ns)
            assert rc == 0 and pr >= 8 * n * ns
            for nlf in (0, 1, 4):
                if d * (nlf + 1) > 32 and nlf:
                    continue
                rc, pc = _size(lib.mfgp_gpr_predict_cov_workspace_size, h, nlf, n, p, d, ns)
                assert rc == 0 and pc >= 8 * ns * ns
        for nlf in (1, 2, 4):
            rc, gm = _size(lib.mfgp_gmf_gpr_workspace_size, h, nlf, n, p, d)
            assert rc == 0 and gm > 0
        if (p, d) in prev:
            assert g >= prev[(p, d)]
        prev[(p, d)] = g
    assert lib.mfgp_set_flow(h, 1) == 0


def test_f32_and_svgp_workspace_sizes(lib, h):
    for n, p, d in SIZES:
        for refine in (0, 1, 2):
            assert lib.mfgp_set_f32_refine(h, refine) == 0
            for panel in (1, 6):
                assert lib.mfgp_set_f32_panel(h, panel) == 0
                rc, s = _size(lib.mfgp_gpr_workspace_size_ex, h, 1, n, p, d)
                assert rc == 0 and s > 4 * n
                rc, s = _size(lib.mfgp_gpr_predict_workspace_size_ex, h, 1, n, p, d, 33)
                assert rc == 0 and s > 0
                rc, s = _size(lib.mfgp_gpr_predict_cov_workspace_size_ex, h, 1, 0, n, p, d, 33)
                assert rc == 0 and s > 0
        for m, L in ((1, 1), (16, 3), (50, 49), (300, 15), (300, 64)):
            rc, s = _size(lib.mfgp_svgp_workspace_size, h, n, m, L, p, d)
            assert rc == 0 and s > 0
            rc, s = _size(lib.mfgp_svgp_grad_workspace_size, h, n, m, L, p, d)
            assert rc == 0 and s > 0
            rc, s = _size(lib.mfgp_svgp_predict_cov_workspace_size, h, 10, m, L, p, d)
            assert rc == 0 and s > 0
    for n, b in ((1, 1), (33, 3), (300, 64)):
        rc, s = _size(lib.mfgp_potrf_inv_workspace_size, h, n, b)
        assert rc == 0 and s >= 8 * n * n * b


def test_bad_arguments_rejected(lib, h):
    """Bad sizes, dimensions, dtypes and settings return an error code; nothing is launched."""
    out = SZ(0)
    assert lib.mfgp_gpr_workspace_size(h, 10, 5, 0, C.byref(out)) == -4       # d < 1
    assert lib.mfgp_gpr_workspace_size(h, 10, 5, 33, C.byref(out)) == -4      # d > MFGP_MAX_D
    assert lib.mfgp_gpr_workspace_size_ex(h, 7, 10, 5, 3, C.byref(out)) == -1
    assert lib.mfgp_set_tile(h, 16) == -1 and lib.mfgp_set_flow(h, 4) == -1 and lib.mfgp_set_flow(h, -1) == -1
    assert lib.mfgp_set_flow_timeout_us(h, -5) == -1
    assert lib.mfgp_set_f32_refine(h, -1) == -1 and lib.mfgp_set_f32_panel(h, 0) == -1
    assert lib.mfgp_get_tile(None) == -1 and lib.mfgp_get_flow(None) == -1 and lib.mfgp_get_tiny(None) == -1
    assert lib.mfgp_create(0, None) == -1
    for code in (0, -1, -2, -3, -4, -5, -99):
        assert len(lib.mfgp_error_string(code)) > 0


@pytest.mark.skipif(torch.cuda.is_available(), reason="null-pointer calls are a host-only check")
def test_compute_entries_validate_before_launch(lib, h):
    """Null / zero-size arguments fail validation in the host code (no device memory is touched)."""
    d = C.c_double(0.0)
    assert lib.mfgp_gpr_lml(h, 0, 1, 1, None, 2, None, 1, None, 0, None, 0, None, None) == -1
    assert lib.mfgp_gpr_lml(h, 10, 1, 1, None, 2, None, 1, None, 0, None, 0, None, None) == -1
    assert lib.mfgp_gpr_adam_step(h, 10, 1, 1, None, 2, None, 1, None, None, None, None, None, None, None,
                                  0.1, 0.9, 0.999, 1e-7, None, None, 0, None, None) == -1
    assert lib.mfgp_gpr_predict(h, 10, 1, 1, 3, None, 2, None, 1, None, 2, None, None, 0, None, 1, None,
                                None) == -1
    assert lib.mfgp_mf_kdiag(h, 4, 1, None, 2, None, None) == -1
    assert lib.mfgp_potrf_inv(h, 4, 1, None, 4, 16, None, 0, None, 4, 16, None, None) == -1
    assert lib.mfgp_svgp_elbo(h, 10, 4, 1, 1, 1, None, 2, None, 1, None, 2, None, None, None, None, 1.0, 1.0,
                              1e-6, None, 0, None, None, None, None) == -1
    assert lib.mfgp_theta_from_u(h, None, None, 6, 5) == -1
    del d
