import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")
if GOLDEN not in sys.path:  # the stand-in plants of the fixtures (toy_dynamics)
    sys.path.insert(1, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgpmpc_hip.so)")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def close(a, b, scale, rtol=1e-6):
    """SURVEY 8c tolerance: |a - b| <= rtol * max(|b|, scale)."""
    a = np.asarray(a, float); b = np.asarray(b, float)
    lim = rtol * np.maximum(np.abs(b), scale)
    return bool(np.all(np.abs(a - b) <= lim)), float(np.max(np.abs(a - b) / lim))


@pytest.fixture(scope="session")
def gpu_ctx():
    """One HIP context for the whole GPU session (one process, one context)."""
    from gp_mpc_rocket_landing_amd import _lib
    ctx = _lib.Context(0)
    yield ctx
    ctx.close()
