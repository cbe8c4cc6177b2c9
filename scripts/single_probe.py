"""The single-landing step (BASELINE configs[2]: the fleet at B = 1) for a kernel trace:
per-kernel durations of 100 control steps (scripts/kstats.sh single python3 scripts/single_probe.py)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402
from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions  # noqa: E402

if __name__ == "__main__":
    ctx = _lib.Context(0)
    gp = fit_gp(ctx, n_train=1000)
    f = Fleet(ctx, gp, 1)
    for _ in range(3):
        f.reset(initial_conditions(1))
        ctx.sync()
        t0 = time.perf_counter()
        f.step(100)
        ctx.sync()
        print(f"{(time.perf_counter() - t0) / 100 * 1e6:.1f} us per step", flush=True)
    f.close()
