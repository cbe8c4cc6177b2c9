"""BASELINE configs[4] rollouts timing alone (bench.py rollouts6_bench): 64 and
512 rollouts flown to termination on the config-5 GP.  Prints the JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from gp_mpc_rocket_landing_amd import _lib  # noqa: E402

if __name__ == "__main__":
    batches = tuple(int(v) for v in os.environ.get("BATCHES", "64,512").split(","))
    import torch
    print(json.dumps(bench.rollouts6_bench(_lib.Context(0), torch, batches=batches)), flush=True)
