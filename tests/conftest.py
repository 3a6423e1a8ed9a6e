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


# ------------------------------------------------------------------------------------------------
# measured parity errors: every check_rel() call records (test, quantity, error, bar); the terminal
# summary prints them and NONODE_PARITY_REPORT=<path> also writes them as JSON
_PARITY = []


def check_rel(name, got, ref, bar):
    """Assert maxnorm_rel(got, ref) < bar and record the measured error."""
    if hasattr(got, "detach"):
        got = got.detach().cpu().numpy()
    if hasattr(ref, "detach"):
        ref = ref.detach().cpu().numpy()
    err = maxnorm_rel(got, ref)
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    _PARITY.append({"test": test, "quantity": name, "maxnorm_rel": float(err), "bar": float(bar)})
    assert err < bar, (name, err, bar)
    return err


def pytest_terminal_summary(terminalreporter):
    if not _PARITY:
        return
    terminalreporter.write_sep("-", "measured parity (max-norm relative error / bar)")
    for r in _PARITY:
        terminalreporter.write_line(f"{r['maxnorm_rel']:.3e} / {r['bar']:.0e}  {r['quantity']:<48s} {r['test']}")
    path = os.environ.get("NONODE_PARITY_REPORT")
    if path:
        import json
        with open(path, "w") as f:
            json.dump(_PARITY, f, indent=1)
