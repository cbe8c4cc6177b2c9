"""Isolated TRSM panel timing: trsm_lower / potrs at n = 128 (one panel launch)
and n = 1000, for a rocprofv3 --kernel-trace beside it."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402

ctx = _lib.default_context()
rs = np.random.RandomState(0)
for n, nrhs in ((128, 64), (128, 3), (1000, 3), (1000, 1000)):
    A = rs.randn(n, n)
    L = np.linalg.cholesky(A @ A.T / n + np.eye(n))
    B = rs.randn(n, nrhs)
    for _ in range(5):
        _lib.trsm_lower(ctx, L, B)
        _lib.potrs(ctx, L, B)
print("done", flush=True)
