"""The drop-in surface loop alone (bench.surface_single_landing_bench), for rocprofv3 runs."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402

ctx = _lib.default_context()
print(json.dumps(bench.surface_single_landing_bench(ctx, steps=100, reps=int(sys.argv[1]) if len(sys.argv) > 1 else 1)), flush=True)
