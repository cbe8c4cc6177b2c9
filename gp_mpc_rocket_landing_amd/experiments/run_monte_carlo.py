"""Sharded Monte-Carlo landings (scripts/run_monte_carlo.py / run_experiments.py
shapes) on one or more MI355X.

    python -m gp_mpc_rocket_landing_amd.experiments.run_monte_carlo --landings 1024
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m gp_mpc_rocket_landing_amd.experiments.run_monte_carlo --landings 1024

Each rank flies its contiguous shard of landings (initial conditions of seeds
42 + global index) to termination on its own GPU -- GP posterior, RTI QP and
ADMM, plant and the MonteCarloSimulator termination rules all device-resident
-- then the 16-double records are gathered to rank 0 with one collective and
summarised like MonteCarloSimulator's statistics (monte_carlo.py:186-272).

``--six-dof`` runs BASELINE configs[4] instead: 6-DoF GP-MPC rollouts (N = 30,
the StructuredRocketGP FITC pair at M = 2000 / N = 4000, every rank fitting it
deterministically), default 512 rollouts sharded the same way:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m gp_mpc_rocket_landing_amd.experiments.run_monte_carlo --six-dof
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np

OUTCOME_NAMES = {1: "SUCCESS", 2: "CRASH", 3: "FUEL_EXHAUSTED", 4: "CONSTRAINT_VIOLATION",
                 5: "TIMEOUT", 6: "DIVERGENCE"}


def summarise(records: np.ndarray) -> dict:
    from ..fleet import REC_ADMM_ITERS, REC_FUEL, REC_OUTCOME, REC_STEPS, REC_TIME
    oc = records[:, REC_OUTCOME].astype(int)
    ok = oc == 1
    out = {"n_landings": int(len(oc)),
           "outcomes": {OUTCOME_NAMES.get(c, str(c)): int(np.sum(oc == c)) for c in np.unique(oc)},
           "success_rate": float(np.mean(ok)) if len(oc) else 0.0,
           "control_steps": int(np.sum(records[:, REC_STEPS])),
           "admm_iterations": int(np.sum(records[:, REC_ADMM_ITERS]))}
    if np.any(ok):
        out["fuel_used_mean_success"] = float(np.mean(records[ok, REC_FUEL]))
        out["flight_time_mean_success"] = float(np.mean(records[ok, REC_TIME]))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--landings", type=int, default=None, help="default 1024 (512 with --six-dof)")
    ap.add_argument("--max-steps", type=int, default=300)
    ap.add_argument("--chunk", type=int, default=25, help="control steps between termination polls")
    ap.add_argument("--train", type=int, default=None, help="GP training rows, default 1000 (4000 with --six-dof)")
    ap.add_argument("--seed0", type=int, default=42)
    ap.add_argument("--out", default="")
    ap.add_argument("--six-dof", action="store_true", help="BASELINE configs[4]: 6-DoF rollouts")
    ap.add_argument("--inducing", type=int, default=2000, help="--six-dof: FITC inducing points")
    args = ap.parse_args(argv)
    if args.landings is None:
        args.landings = 512 if args.six_dof else 1024
    if args.train is None:
        args.train = 4000 if args.six_dof else 1000

    import torch
    import torch.distributed as dist
    from .. import _lib
    from ..fleet import REC_OUTCOME, Fleet, fit_gp, initial_conditions
    from ..sharding import gather_shard_records, shard_range

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    first, count = shard_range(args.landings, rank, world)
    ctx = _lib.Context(local)
    if args.six_dof:
        from ..rollouts6 import Rollouts6, fit_structured_fitc, initial_conditions_6dof
        gps = fit_structured_fitc(ctx, n_train=args.train, n_inducing=args.inducing)  # same on every rank
        fl = Rollouts6(ctx, *gps, max(count, 1), max_steps=args.max_steps)
        x0 = initial_conditions_6dof(count, args.seed0, first) if count else None
    else:
        gp = fit_gp(ctx, n_train=args.train)          # every rank fits the same GP deterministically
        # a shard of the whole fleet: kernel choices made for args.landings, so every
        # landing's record is bit-identical to the unsharded run's
        fl = Fleet(ctx, gp, max(count, 1), fleet_batch=max(args.landings, 1), max_steps=args.max_steps)
        x0 = initial_conditions(count, args.seed0, first) if count else None
    t0 = time.perf_counter()
    rec = np.zeros((0, _lib.REC_LEN))
    if count:
        fl.reset(x0)
        done = 0
        while done < args.max_steps + 1:
            fl.step(args.chunk)
            done += args.chunk
            rec, _ = fl.read()
            if np.all(rec[:, REC_OUTCOME] != 0):
                break
    ctx.sync()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
    # the one collective: the C-ABI's ncclGather of the device records (GPMPC_GATHER=torch:
    # torch.distributed.gather); a set-up failure on any rank is agreed and every rank
    # falls back together, and `gather` in the summary says what ran
    allrec, ginfo = gather_shard_records(ctx, fl.records_dev if count else None, rec, args.landings,
                                         device="cuda")
    if rank == 0:
        s = summarise(allrec)
        s.update(n_gpus=world, gather=ginfo, wall_s=round(el, 3), control_steps_per_s=round(s["control_steps"] / el, 1))
        if args.six_dof:
            s.update(config="configs[4] 6-DoF rollouts", rollouts_per_s=round(s["n_landings"] / el, 1))
        print(json.dumps(s), flush=True)
        if args.out:
            np.savez(args.out, records=allrec)
    fl.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
