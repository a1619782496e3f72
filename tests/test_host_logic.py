"""Host-side logic of the Python mirror (no GPU): transforms, parameters, layout."""
import numpy as np
import pytest

import multi_fidelity_gpflow_amd as M
from multi_fidelity_gpflow_amd.models import _ThetaMap
from multi_fidelity_gpflow_amd.params import tf_softplus, tf_softplus_inverse
from oracle import mfgp_oracle as O


def test_transforms_match_oracle():
    x = np.linspace(-40, 40, 801)
    np.testing.assert_array_equal(tf_softplus(x), O.softplus(x))
    y = np.logspace(-12, 3, 200)
    np.testing.assert_array_equal(tf_softplus_inverse(y), O.softplus_inverse(y))


def test_parameter_roundtrip_and_lower_bound():
    p = M.Parameter(1e-3, transform=M.positive(lower=1e-6))
    assert abs(float(p.numpy()) - 1e-3) < 1e-16      # TF softplus round trip (log(exp(x)+1))
    assert abs(float(p.unconstrained_variable) - O.softplus_inverse(1e-3 - 1e-6)) < 1e-15
    p.assign(0.5)
    assert abs(float(p.numpy()) - 0.5) < 1e-15
    q = M.Parameter(np.ones((3, 1)), transform=M.positive())
    assert q.shape == (3, 1)


def _model(P=2, D=3, ard=True):
    rng = np.random.default_rng(0)
    X = np.hstack([rng.random((8, D)), np.r_[np.zeros(5), np.ones(3)][:, None]])
    Y = rng.standard_normal((8, P))
    ls = np.ones(D) if ard else 1.0
    return M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=ls), M.SquaredExponential(lengthscales=ls))


def test_model_construction_semantics():
    m = _model(P=3)
    assert m.kernel.rho.shape == (3, 1)                      # linear.py:47-49 (P, 1)
    assert float(m.likelihood.variance.numpy()) == pytest.approx(1e-3, rel=1e-15)
    assert not m.likelihood.variance.trainable               # linear.py:154
    names = [n for n, _ in m.parameters_with_names()]
    assert "kernel.rho" in names and "likelihood.variance" in names
    assert all(p.trainable for p in m.kernel.parameters)


def test_theta_layout_and_ties():
    m = _model(D=3, ard=True)
    tm = _ThetaMap(m, 3)
    th = tm.theta()
    assert th.shape == (2 * 3 + 4,)
    np.testing.assert_allclose(th, [1, 1, 1, 1, 1, 1, 1, 1, 1, 1e-3], rtol=1e-12)
    assert len(set(tm.tie())) == len(th)
    assert list(tm.trainable()) == [True] * 9 + [False]
    iso = _model(D=3, ard=False)
    tie = _ThetaMap(iso, 3).tie()
    assert tie[1] == tie[2] == tie[3] and tie[5] == tie[6] == tie[7] and tie[1] != tie[5]
    u = _ThetaMap(iso, 3).u()
    u[1:4] = 0.25
    _ThetaMap(iso, 3).set_u(u)
    assert iso.kernel.kernel_L.lengthscales.shape == ()
    assert float(iso.kernel.kernel_L.lengthscales.numpy()) == pytest.approx(float(O.softplus(0.25)))


def test_parameter_dict_roundtrip():
    m = _model()
    d = M.parameter_dict(m)
    m2 = _model()
    m2.kernel.kernel_L.variance.assign(7.0)
    M.multiple_assign(m2, d)
    assert float(m2.kernel.kernel_L.variance.numpy()) == pytest.approx(1.0)


def test_powerspecs_loader_matches_oracle(hbs):
    from multi_fidelity_gpflow_amd.data import PowerSpecs, multifidelity_training_set
    from conftest import HBS_DIR
    ps = PowerSpecs()
    ps.read_from_txt(HBS_DIR)
    X, Y, Xt, Yt = multifidelity_training_set(ps)
    np.testing.assert_array_equal(X, hbs["X"])
    np.testing.assert_array_equal(Y, hbs["Y"])
    np.testing.assert_array_equal(Xt, hbs["Xtest"])
    assert ps.kf.shape == (49,)


def test_bin_blocks_partition():
    from multi_fidelity_gpflow_amd.distributed import bin_block
    for p in (1, 3, 49, 64, 512):
        for w in (1, 2, 3, 4, 8):
            if w > p:
                continue
            blocks = [bin_block(p, r, w) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == p
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in blocks) - min(b - a for a, b in blocks) <= 1


def test_compute_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    m = _model()
    with pytest.raises(M.MFGPError):
        m.log_marginal_likelihood()


def test_svgp_save_load_roundtrip(hbs, tmp_path):
    """save_model / load_model of both SVGP emulators (linear_svgp.py:206-221,
    singlebin_svgp.py:99-135): parameter_dict pickled, re-applied with multiple_assign onto a
    model rebuilt from the constructor arguments.  Host only (no compute)."""
    X, Y = hbs["X"], hbs["Y"]
    kL = M.SquaredExponential(lengthscales=np.ones(5))
    kD = M.SquaredExponential(lengthscales=np.ones(5))
    args = (X, Y, kL, kD, 4, 12, Y.shape[1])
    lat = M.LatentMFCoregionalizationSVGP(*args)
    lat.kernel.kernels[1].kernel_L.lengthscales.assign(np.linspace(0.3, 0.9, 5))
    lat.q_mu.assign(np.arange(12 * 4, dtype=float).reshape(12, 4) * 0.01)
    lat.kernel.W.assign(lat.kernel.W.numpy() * 1.5)
    f = str(tmp_path / "lat.pkl")
    lat.save_model(f)
    back = M.LatentMFCoregionalizationSVGP.load_model(f, *args)
    for (n1, p1), (n2, p2) in zip(lat.parameters_with_names(), back.parameters_with_names()):
        assert n1 == n2
        np.testing.assert_array_equal(p1.numpy(), p2.numpy())
    sb = M.SingleBinSVGP(X, Y[:, :3], kL, kD, 3, np.zeros((10, 6)))
    sb.q_mu.assign(np.ones((10, 3)) * 0.5)
    f2 = str(tmp_path / "sb.pkl")
    sb.save_model(f2)
    back2 = M.SingleBinSVGP.load_model(f2, X, Y[:, :3], kL, kD, 3, np.zeros((10, 6)))
    np.testing.assert_array_equal(back2.q_mu.numpy(), sb.q_mu.numpy())


def test_torch_cpu_baseline_matches_oracle(hbs):
    """oracle/torch_oracle.py (bench.py's timed CPU baseline) agrees with the KAT-pinned
    oracle/mfgp_oracle.py: LML 1e-13 rel, gradient 1e-10 of the largest component."""
    import torch
    from oracle import torch_oracle as TO
    X, Y = hbs["X"], hbs["Y"]
    rng = np.random.default_rng(2)
    p = O.MFParams(1.3, 0.5 + rng.random(5), 0.4, 0.5 + rng.random(5), np.full((49, 1), 0.8), 2e-3)
    lo, go = O.gpr_lml_and_grad(X, Y, p)
    gv = np.concatenate([[go["vL"]], go["lL"], [go["vD"]], go["lD"], [go["rho0"]], [go["noise"]]])
    args = (p.vL, torch.tensor(p.lL), p.vD, torch.tensor(p.lD), p.rho0, p.noise)
    l1, g1 = TO.lml_and_grad(torch.tensor(X), torch.tensor(Y), *args)
    assert abs(l1 - lo) < 1e-13 * abs(lo)
    assert abs(TO.lml(torch.tensor(X), torch.tensor(Y), *args) - lo) < 1e-13 * abs(lo)
    np.testing.assert_allclose(g1.numpy(), gv, rtol=0, atol=1e-10 * np.abs(gv).max())
