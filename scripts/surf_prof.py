"""cProfile of the drop-in surface loop (bench.surface_single_landing_bench) on the GPU box:
where a GPMPC.solve step's host time goes.  python3 scripts/surf_prof.py [unc 0|1]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402

ctx = _lib.default_context()
bench.surface_single_landing_bench(ctx, steps=20, reps=1)  # warm
pr = cProfile.Profile()
pr.enable()
print(bench.surface_single_landing_bench(ctx, steps=100, reps=1), flush=True)
pr.disable()
st = pstats.Stats(pr).sort_stats("tottime")
st.print_stats(30)
st.sort_stats("cumulative").print_stats(40)
