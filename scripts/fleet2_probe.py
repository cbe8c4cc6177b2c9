"""Control steps/s of the BASELINE configs[3] fleet (1024 landings, N = 20, 1000
GP points) as one fleet on one stream against G fleets of 1024/G landings on G
streams (contexts) of the same GPU, launched interleaved so one group's GP GEMM
(MFMA-bound) can overlap another's control kernel (latency-bound).  Prints JSON."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gp_mpc_rocket_landing_amd import _lib  # noqa: E402
from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions  # noqa: E402


def run(groups, B=1024, K=40, W=5):
    ctxs = [_lib.Context(0) for _ in range(groups)]
    gp = fit_gp(ctxs[0], n_train=1000)
    ctxs[0].sync()
    per = B // groups
    fls = [Fleet(ctxs[g], gp, per, horizon=20) for g in range(groups)]
    for g, f in enumerate(fls):
        f.reset(initial_conditions(per, seed0=42, first=g * per))
    for _ in range(W):
        for f in fls:
            f.step(1)
    for c in ctxs:
        c.sync()
    r0 = [f.read()[0] for f in fls]
    t0 = time.perf_counter()
    for _ in range(K):
        for f in fls:
            f.step(1)
    for c in ctxs:
        c.sync()
    el = time.perf_counter() - t0
    r1 = [f.read()[0] for f in fls]
    steps = sum(float(np.sum(b[:, 1] - a[:, 1])) for a, b in zip(r0, r1))
    for f in fls:
        f.close()
    return {"groups": groups, "ms_per_step": round(el / K * 1e3, 4), "steps_per_s": round(steps / el, 1)}


if __name__ == "__main__":
    out = [run(g) for g in (1, 2, 4, 1, 2, 4)]
    print(json.dumps(out))
