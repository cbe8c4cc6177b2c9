"""The bench's control step alone (1024 landings, N = 20, GP n = 1000), for
profiling runs: fit, reset, 3 warm-up steps, STEPS timed steps (env)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402
from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions  # noqa: E402


def main():
    B = int(os.environ.get("LANDINGS", "1024"))
    steps = int(os.environ.get("STEPS", "10"))
    ctx = _lib.Context(0)
    gp = fit_gp(ctx, n_train=1000)
    fl = Fleet(ctx, gp, B)
    fl.reset(initial_conditions(B))
    fl.step(3)
    ctx.sync()
    t0 = time.perf_counter()
    fl.step(steps)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    print(f"{B} landings: {dt * 1e3:.3f} ms per step, {B / dt / 1e6:.3f} M steps/s", flush=True)
    fl.close()


if __name__ == "__main__":
    main()
