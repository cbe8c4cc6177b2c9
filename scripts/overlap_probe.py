"""Probe: do sub-fleets on separate HIP streams overlap the latency-bound control
kernel of one group with the MFMA posterior GEMM of another?  Prints one line
per configuration: groups x landings, control steps/s."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402
from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions  # noqa: E402


def run(groups, per, K=30, W=5):
    ctxs = [_lib.Context(0) for _ in range(groups)]
    gp = fit_gp(ctxs[0], n_train=1000)
    fls = []
    for g, c in enumerate(ctxs):
        f = Fleet(c, gp, per, horizon=20)
        f.reset(initial_conditions(per, seed0=42, first=g * per))
        fls.append(f)
    for _ in range(W):
        for f in fls:
            f.step(1)
    for c in ctxs:
        c.sync()
    r0 = sum(float(np.sum(f.read()[0][:, 1])) for f in fls)
    t0 = time.perf_counter()
    for _ in range(K):
        for f in fls:
            f.step(1)
    for c in ctxs:
        c.sync()
    el = time.perf_counter() - t0
    r1 = sum(float(np.sum(f.read()[0][:, 1])) for f in fls)
    print(f"groups={groups} per={per}: {(r1 - r0) / el:,.0f} steps/s, {el / K * 1e3:.3f} ms/step",
          flush=True)
    for f in fls:
        f.close()
    del gp
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    for g, p in [(1, 1024), (2, 512), (1, 2048), (2, 1024), (4, 512), (4, 256), (1, 1024)]:
        run(g, p)
