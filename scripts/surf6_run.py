"""The 14-state drop-in surface loop alone (bench.surface_gpmpc6_bench), for timing and profiles."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402

ctx = _lib.default_context()
if len(sys.argv) > 1 and sys.argv[1] == "prof":
    import cProfile
    import pstats
    bench.surface_gpmpc6_bench(ctx, steps=5, reps=1)
    pr = cProfile.Profile()
    pr.enable()
    print(bench.surface_gpmpc6_bench(ctx, steps=30, reps=1), flush=True)
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
else:
    print(json.dumps(bench.surface_gpmpc6_bench(ctx)), flush=True)
