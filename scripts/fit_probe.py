"""Where Simple3DoFGP.fit's 3.4 ms go (BASELINE configs[1]): wall time of the
surface fit and of the bare C-ABI fit, repeated, for a rocprofv3 kernel/HIP-API
trace to be laid beside.  Run on the GPU box:
    rocprofv3 --kernel-trace --hip-trace --stats -d gpurun_out/fitprobe -o run -- python3 scripts/fit_probe.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402
from gp_mpc_rocket_landing_amd.data import synthetic_training_data  # noqa: E402
from gp_mpc_rocket_landing_amd.gp import Simple3DoFGP  # noqa: E402
from gp_mpc_rocket_landing_amd.gp.features import Simple3DoFFeatureExtractor  # noqa: E402

X, U, D = synthetic_training_data(1000, seed=0)
Z = Simple3DoFFeatureExtractor().extract_batch(X, U)
ctx = _lib.default_context()
for rep in range(8):
    gp = Simple3DoFGP(use_sparse=False)
    gp.add_data(X, U, D)
    t0 = time.perf_counter(); gp.fit(); t1 = time.perf_counter()
    h = _lib.ExactGPHandle(ctx, _lib.SE_ARD, Z, D, np.ones(Z.shape[1]), 1.0, 1e-4)
    t2 = time.perf_counter()
    del h
    t3 = time.perf_counter()
    print(f"rep {rep}: surface fit {1e3 * (t1 - t0):.3f} ms, C-ABI fit {1e3 * (t2 - t1):.3f} ms, "
          f"destroy {1e3 * (t3 - t2):.3f} ms", flush=True)
