"""gpmpc_gp_append timing: k rows into the n = 1000 exact GP, repeated,
for a rocprofv3 kernel trace of one append's launches and gaps (scripts/kstats.sh)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gp_mpc_rocket_landing_amd import _lib  # noqa: E402
from gp_mpc_rocket_landing_amd.data import synthetic_training_data  # noqa: E402
from gp_mpc_rocket_landing_amd.gp.features import Simple3DoFFeatureExtractor  # noqa: E402

if __name__ == "__main__":
    n, k = 1000, int(os.environ.get("APPEND_K", "10"))
    ctx = _lib.Context(0)
    X, U, D = synthetic_training_data(n + k, seed=0)
    Z = Simple3DoFFeatureExtractor().extract_batch(X, U)
    ta, tf = [], []
    for _ in range(6):
        h = _lib.ExactGPHandle(ctx, _lib.SE_ARD, Z[:n], D[:n], np.ones(11), 1.0, 1e-4)
        t0 = time.perf_counter()
        assert h.append(Z[n:], D)
        ta.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        h2 = _lib.ExactGPHandle(ctx, _lib.SE_ARD, Z, D, np.ones(11), 1.0, 1e-4)
        tf.append(time.perf_counter() - t0)
        del h, h2
    print({"append_ms": [round(t * 1e3, 3) for t in ta], "refit_ms": [round(t * 1e3, 3) for t in tf]})
