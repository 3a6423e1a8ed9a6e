import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm MI355X device (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    return {k: d[k] for k in d.files}


def params_of(fx, prefix="w::"):
    return {k[len(prefix):]: v for k, v in fx.items() if k.startswith(prefix)}


def maxnorm_rel(a, b):
    """Parity metric of SURVEY §8d: ||a - b||_inf / ||b||_inf."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.fixture(scope="session")
def golden():
    return load_golden
