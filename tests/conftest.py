import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
HBS_DIR = os.path.join(GOLDEN, "data", "50_LR_3_HR")
GOKU_DIR = os.path.join(GOLDEN, "data", "matter_power_1128_Box1000_Part750_36_Box1000_Part3000_z0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running CPU oracle check")


_provenance_checked = []


def pytest_runtest_setup(item):
    """Before the first GPU test: the loaded libmfgp.so must be the one built from the sources
    checked out here (mfgp_build_id against build.source_hash())."""
    if "gpu" in item.keywords and not _provenance_checked:
        from multi_fidelity_gpflow_amd import _lib
        _lib.check_provenance()
        _provenance_checked.append(True)


@pytest.fixture(scope="session")
def kats():
    import json
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def hbs():
    from oracle.mfgp_oracle import load_powerspecs
    return load_powerspecs(HBS_DIR)


@pytest.fixture(scope="session")
def goku():
    from oracle.mfgp_oracle import load_powerspecs
    return load_powerspecs(GOKU_DIR)


def forrester_demo_data():
    """notebooks/demo.ipynb cell 2 (seed 42, RNG consumption order preserved)."""
    rs = np.random.RandomState(42)

    def forrester(x, sd=0):
        x = x.reshape((len(x), 1))
        n = x.shape[0]
        fval = ((6 * x - 2) ** 2) * np.sin(12 * x - 4)
        noise = np.zeros(n).reshape(n, 1) if sd == 0 else rs.normal(0, sd, n).reshape(n, 1)
        return fval.reshape(n, 1) + noise

    def forrester_low(x, sd=0):
        return 0.5 * forrester(x, 0) + 10 * (x[:, [0]] - 0.5) + 5 + rs.randn(x.shape[0], 1) * sd

    x_plot = np.linspace(0, 1, 200)[:, None]
    forrester_low(x_plot)
    forrester(x_plot)
    x_train_l = np.atleast_2d(rs.rand(40)).T
    x_train_h = np.atleast_2d(rs.permutation(x_train_l)[:13])
    y_train_l = forrester_low(x_train_l)
    y_train_h = forrester(x_train_h)
    X = np.vstack([np.hstack([x_train_l, np.zeros_like(x_train_l)]), np.hstack([x_train_h, np.ones_like(x_train_h)])])
    Y = np.vstack([y_train_l, y_train_h])
    return X, Y


def forrester_test_data(n_l=60, n_h=20, sd_l=0.05, sd_h=0.02):
    """tests/test_forrest.py:12-31 (seed 42)."""
    rs = np.random.RandomState(42)

    def forrester(x, sd=0):
        x = x.reshape((len(x), 1))
        fval = ((6 * x - 2) ** 2) * np.sin(12 * x - 4)
        noise = rs.normal(0, sd, x.shape) if sd > 0 else np.zeros_like(x)
        return fval + noise

    def forrester_low(x, sd=0):
        return 0.5 * forrester(x, 0) + 10 * (x - 0.5) + 5 + rs.randn(*x.shape) * sd

    x_l = rs.rand(n_l, 1)
    x_h = rs.permutation(x_l)[:n_h]
    y_l = forrester_low(x_l, sd=sd_l)
    y_h = forrester(x_h, sd=sd_h)
    X = np.vstack([np.hstack([x_l, np.zeros_like(x_l)]), np.hstack([x_h, np.ones_like(x_h)])])
    return X, np.vstack([y_l, y_h])


def sin_multi_output_data(P=1):
    """tests/test_scipy.py:9-20 (P=1) and tests/test_output_dim.py:13-31 (P=3), seed 42."""
    rs = np.random.RandomState(42)
    X_L = rs.uniform(-3, 3, (10, 1))
    Y_L = np.sin(X_L) + 0.1 * rs.randn(10, P)
    X_H = rs.uniform(-3, 3, (5, 1))
    Y_H = 1.2 * np.sin(X_H) + 0.05 * rs.randn(5, P)
    X = np.vstack([np.hstack([X_L, np.zeros((10, 1))]), np.hstack([X_H, np.ones((5, 1))])])
    return X, np.vstack([Y_L, Y_H])
