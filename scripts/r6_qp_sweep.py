"""at which ADMM settings does the configs[4] controller (6-DoF
GP-MPC, N = 30, config-5 FITC GP) return "solved" for >= 90% of its QPs?  For
each (max_iter, eps) the 64-rollout batch flies to termination once for the
status histogram (bench.rollouts6_qp_status) and once timed.  Prints one JSON
line per setting."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402
from gp_mpc_rocket_landing_amd.rollouts6 import Rollouts6, fit_structured_fitc, initial_conditions_6dof  # noqa: E402

if __name__ == "__main__":
    ctx = _lib.Context(0)
    gv, gw = fit_structured_fitc(ctx, n_train=4000, n_inducing=2000)
    B = int(os.environ.get("B", "64"))
    settings = [tuple(float(x) for x in t.split(":")) for t in
                os.environ.get("SETTINGS", "50:1e-4,100:1e-4,200:1e-4,400:1e-4,1000:1e-4,4000:1e-4").split(",")]
    for mi, eps in settings:
        qp = dict(max_iter=int(mi), eps_abs=eps, eps_rel=eps)
        st = bench.rollouts6_qp_status(ctx, gv, gw, B, **qp)
        ro = Rollouts6(ctx, gv, gw, B, **qp)
        ro.reset(initial_conditions_6dof(B)); ro.step(1); ctx.sync()
        ro.reset(initial_conditions_6dof(B)); ctx.sync()
        t0 = time.perf_counter(); steps = 0
        while steps < 301:
            ro.step(10); steps += 10
            rec, _ = ro.read()
            if np.all(rec[:, 0] != 0):
                break
        el = time.perf_counter() - t0
        ro.close()
        print(json.dumps({"max_iter": int(mi), "eps": eps, "ms_per_step": round(el / steps * 1e3, 3),
                          "rollouts_per_s": round(B / el, 1), **st}), flush=True)
