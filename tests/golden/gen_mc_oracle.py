"""Generate tests/golden/mc_oracle_1024.npz: the CPU oracle's Monte-Carlo of
BASELINE configs[3] -- 1024 landings (initial conditions of seeds 42 + i,
run_experiments.py SimulationConfig, pinned by F7) flown to termination by
oracle.mc_oracle.closed_loop_landing (monte_carlo.py:401-583 restated, the
exact GP of generator G, the C OSQP-0.6 restatement).

Unlike gen_golden.py this does not touch the reference: it records the
oracle's own output at full size so the GPU test can compare the device
Monte-Carlo with it without re-running 400 core-seconds of oracle on the
box.  tests/test_mc_protocol.py re-derives a sample of rows live.

    python tests/golden/gen_mc_oracle.py        # ~1 min on 8 cores
"""
import os
import sys
from multiprocessing import Pool

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402

from gp_mpc_rocket_landing_amd.data import synthetic_training_data  # noqa: E402
from oracle import gp_oracle, mc_oracle  # noqa: E402

_ST = None


def _state():
    global _ST
    if _ST is None:
        X, U, D = synthetic_training_data(1000, seed=0)
        _ST = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
    return _ST


def fly(i):
    rec, x, _ = mc_oracle.closed_loop_landing(_state(), mc_oracle.sample_initial_condition(42 + i))
    return rec


def main():
    with Pool(min(8, os.cpu_count() or 1)) as p:
        R = np.array(p.map(fly, range(1024), chunksize=8))
    np.savez_compressed(os.path.join(HERE, "mc_oracle_1024.npz"), records=R,
                        seeds=42 + np.arange(1024))
    oc, cnt = np.unique(R[:, 0], return_counts=True)
    print(dict(zip(oc.astype(int).tolist(), cnt.tolist())), int(R[:, 1].sum()), int(R[:, 11].sum()))


if __name__ == "__main__":
    main()
