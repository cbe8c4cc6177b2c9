#!/usr/bin/env python
"""bench.py -- GP-MPC control steps/s on MI355X (BASELINE.json metric).

Workload (BASELINE configs[3], the run_monte_carlo.py shapes of SURVEY 8d C4):
per GPU a fleet of ``--landings`` closed-loop 3-DoF GP-MPC landings (initial
conditions of scripts/run_experiments.py, seeds 42 + global index), horizon
N = 20, one exact GP on 1000 synthetic training points (generator G) shared by
every landing.  One "step" = one control step of every active landing: GP
posterior (mean + variance) at the 20 horizon points, RTI QP assembly with the
GP mean, OSQP-style ADMM (<= 50 iterations), plant step -- all device-resident.

N > 1: one process per GPU (torch.distributed.run), landings sharded (weak
scaling: a fixed fleet per GPU), no collective on the data path; the fleet
records are gathered to rank 0 with one RCCL gather after the timed region
(the JSON's `gather` says which path ran and how many ranks it spanned).

Prints ONE JSON line on rank 0.  ``value`` = landing control steps executed by
all ranks / max-over-ranks wall time of the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix (= vector) peak, spec
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)


def admm_flops(n=207, m=354, nnz=734, sz=10, cm=7):
    """Algorithmic flops of one ADMM iteration and of one (re)factorisation of
    the reduced KKT matrix in its block-tridiagonal form:
    forward 2*cm*sz and backward 2*cm*sz per block boundary, diagonal 2*sz^2 per
    block, two SpMVs with A, and the vector updates; the factor is Gauss-Jordan
    2*sz^3 + G_k 2*cm*sz^2 + Schur 2*cm^2*sz per block plus the assembly."""
    nblk = -(-n // sz)
    kkt = 2 * (nblk - 1) * 2 * cm * sz + nblk * 2 * sz * sz
    it = kkt + 2 * 2 * nnz + 12 * n + 14 * m
    fac = nblk * (2 * sz ** 3 + 2 * cm * sz * sz + 2 * cm * cm * sz) + 3 * 1500
    return it, fac


# the fleet's control kernel: the specialised solver unless GPMPC_FLEET_SOLVER=0
CONTROL_KERNEL = "k_fleet_control" if os.environ.get("GPMPC_FLEET_SOLVER", "1") == "0" else "k_fleet_control2<false>"


def pmc_traffic(kernel):
    """Per-launch HBM bytes of ``kernel`` from the committed rocprofv3 --pmc
    passes (profiles/*_pmc_traffic.json, scripts/pmc.py traffic), else None."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), reverse=True):
        try:
            ks = json.load(open(path))["kernels"]
        except Exception:  # noqa: BLE001
            continue
        # the horizon-templated kernels carry their namespace (r6n30::k_r6_control<false>)
        k = ks.get(kernel) or next((v for n, v in ks.items() if n.endswith("::" + kernel)), None)
        if k:
            return float(k["traffic_bytes"]), os.path.basename(path)
    return None, None


def _cpu_landing_loop(seconds, n_train=1000, horizon=20, seed=42, threads=1):
    """One landing closed loop of the reference CPU path restated (oracle):
    numpy/scipy GP posterior at the N horizon points (same LAPACK calls as
    exact_gp.py), numpy QP assembly (osqp_rti.py semantics) and the C
    restatement of the OSQP ADMM, BLAS on ``threads`` threads.  Returns (steps, seconds)."""
    from threadpoolctl import threadpool_limits
    from oracle import admm_ref, gp_oracle, mc_oracle, qp_oracle
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data

    X, U, D = synthetic_training_data(n_train, seed=0)
    with threadpool_limits(threads):
        st = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
        x = mc_oracle.sample_initial_condition(seed)
        tgt = mc_oracle.incremental_target(x)
        Xw, Uw = qp_oracle.initial_guess(x, tgt, horizon)
        P0, _ = qp_oracle.cost(horizon, np.tile(tgt, (horizon + 1, 1)))
        qp = admm_ref.RefQP(qp_oracle.N_X * (horizon + 1) + qp_oracle.n_vars(horizon))
        steps = 0
        t0 = time.perf_counter()
        deadline = t0 + seconds
        while time.perf_counter() < deadline:
            if mc_oracle.pre_step_outcome(x, 2.0):
                x = mc_oracle.sample_initial_condition(seed + 1 + steps)
                qp = admm_ref.RefQP(qp.y.size)
            tgt = mc_oracle.incremental_target(x)
            mean, var = gp_oracle.exact_predict(st, gp_oracle.features_3dof(Xw[:-1], Uw))
            _, q = qp_oracle.cost(horizon, np.tile(tgt, (horizon + 1, 1)))
            A, l, u = qp_oracle.constraints(Xw, Uw, x, 0.1, gp_dv=mean, sign=-1.0,
                                            filter_small=False)
            r = qp.solve(P0.diagonal(), q, A, l, u, qp_oracle.to_vector(Xw, Uw))
            Xo, Uo = qp_oracle.from_vector(r["x"], horizon)
            dr = qp_oracle.drag_residual(x)  # residual at the pre-step state
            x = qp_oracle.plant_step(x, Uo[0], 0.1)
            x[4:7] += dr * 0.1
            Xw = np.vstack([Xo[1:], Xo[-1:]]); Uw = np.vstack([Uo[1:], Uo[-1:]])
            steps += 1
        el = time.perf_counter() - t0
    return steps, el


def cpu_quota():
    """The CPU share this job is granted: the cgroup quota (v2 ``cpu.max``, v1
    ``cfs_quota_us / cfs_period_us``) when one is set, else the thread budget the
    box exports (``OMP_NUM_THREADS`` / ``MAX_JOBS``), else None.  Returns
    (cores or None, source)."""
    import math
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, math.floor(int(q) / int(p))), f"cgroup cpu.max {q}/{p}"
    except Exception:  # noqa: BLE001
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, math.floor(q / p)), f"cgroup v1 cfs {q}/{p}"
    except Exception:  # noqa: BLE001
        pass
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(var, "")
        if v.isdigit() and int(v) > 0:
            return int(v), f"{var}={v} (no cgroup CPU quota visible)"
    return None, "none (no cgroup quota, no thread budget in the environment)"


def cpu_baseline(seconds, n_train=1000, horizon=20, workers=None):
    """SURVEY 8d CPU baseline, throughput mode: one process per core of the job's
    CPU share (cpu_quota(); the affinity mask when no share is stated), one
    landing each, BLAS on one thread, for ``seconds``; value = all processes'
    control steps / the longest elapsed.  Runs before the GPU is initialised
    (spawned workers, fresh interpreters)."""
    import concurrent.futures as cf
    import multiprocessing as mp
    import platform
    aff = len(os.sched_getaffinity(0))
    quota, quota_src = cpu_quota()
    workers = workers or max(1, min(aff, quota) if quota else aff)
    with cf.ProcessPoolExecutor(workers, mp_context=mp.get_context("spawn")) as ex:
        res = list(ex.map(_cpu_landing_loop, [seconds] * workers, [n_train] * workers,
                          [horizon] * workers, [42 + 1000 * i for i in range(workers)]))
    steps = sum(r[0] for r in res)
    el = max(r[1] for r in res)
    per_core = float(np.mean([r[0] / r[1] for r in res]))
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name"))
    except Exception:  # noqa: BLE001
        pass
    try:
        blas = np.__config__.CONFIG["Build Dependencies"]["blas"]["name"]
    except Exception:  # noqa: BLE001
        blas = "unknown"
    # SURVEY 8d mode (i): one landing with BLAS on all the workers' cores
    st1, el1 = _cpu_landing_loop(min(5.0, seconds), n_train, horizon, 42, workers)
    return dict(value=steps / el, unit="control steps/s", cores=workers, kind="port",
                per_core=round(per_core, 3), affinity_cpus=aff, cpu_quota=quota,
                cpu_quota_source=quota_src,
                # landings are independent single-threaded processes, so per-core x
                # cores bounds a whole 64-core socket the job's share cannot run
                socket_64c_extrapolated=round(per_core * 64, 1),
                single_landing_all_cores=round(st1 / el1, 3),
                sample=f"{workers} processes x 1 landing closed loop, {steps} control steps in "
                       f"{el:.1f} s (numpy/scipy GP N={n_train}, P={horizon}; numpy QP assembly; "
                       f"C OSQP-0.6 ADMM restatement; {blas} on 1 thread per process; "
                       f"{aff} CPUs in affinity, CPU share {quota} from {quota_src}; {cpu})")


def cholesky_bench(ctx, torch, n=1000, batch=64, reps=3):
    """Batched fp64 potrf throughput (BASELINE metric: Cholesky %MFMA peak)."""
    from gp_mpc_rocket_landing_amd import _lib
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(0)
    G = torch.randn(batch, n, n, dtype=torch.float64, device=dev, generator=g) / n ** 0.5
    base = G @ G.transpose(1, 2) + torch.eye(n, dtype=torch.float64, device=dev)
    info = torch.zeros(batch, dtype=torch.int32, device=dev)
    A = base.clone()
    torch.cuda.synchronize()
    stream = torch.cuda.ExternalStream(ctx.stream)
    times = []
    for _ in range(reps):
        A.copy_(base)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        rc = _lib._L.gpmpc_potrf_batched_dev(ctx.h, n, batch, A.data_ptr(), n, n * n, info.data_ptr())
        e1.record(stream)
        _lib._chk(rc, "potrf_batched_dev")
        ctx.sync()
        times.append(e0.elapsed_time(e1) * 1e-3)
    assert int(info.abs().sum().item()) == 0
    t = min(times)
    flops = batch * (n ** 3 / 3.0 + n ** 2 / 2.0 + n / 6.0)
    tf = flops / t / 1e12
    # SYRK = the trailing updates of the two-level blocked potrf (outer panels of
    # 128): C[t0:n, t0:n] -= A[t0:n, K0:t0] A[t0:n, K0:t0]^T, lower, for
    # t0 = 128, 256, ...; timed alone on the same shapes and batch.
    shapes = [(n - t0, 128) for t0 in range(128, n, 128)]
    syrk_flops = sum(batch * r * (r + 1) * k for r, k in shapes)   # lower incl. diagonal, FMA = 2
    A.copy_(base)
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for r, k in shapes:
            t0 = n - r
            pa = A.data_ptr() + 8 * (t0 * n + t0 - k)
            pc = A.data_ptr() + 8 * (t0 * n + t0)
            _lib._chk(_lib._L.gpmpc_syrk_batched_dev(ctx.h, r, k, batch, pa, n, n * n, pc, n, n * n,
                                                     -1e-3, 1.0), "syrk")
        e1.record(stream)
        ctx.sync()
        el = e0.elapsed_time(e1) * 1e-3
        best = el if best is None else min(best, el)
    syrk_tf = syrk_flops / best / 1e12
    # the FITC SYRK of BASELINE config 5: B = I + A_s A_s^T, A_s (M x N) = 2000 x 4000
    m2, k2 = 2000, 4000
    As = torch.randn(m2, k2, dtype=torch.float64, device=dev, generator=g) / k2 ** 0.5
    Bm = torch.eye(m2, dtype=torch.float64, device=dev)
    fb = None
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        _lib._chk(_lib._L.gpmpc_syrk_batched_dev(ctx.h, m2, k2, 1, As.data_ptr(), k2, 0, Bm.data_ptr(),
                                                 m2, 0, 1.0, 1.0), "syrk")
        e1.record(stream)
        ctx.sync()
        el = e0.elapsed_time(e1) * 1e-3
        fb = el if fb is None else min(fb, el)
    fitc_tf = m2 * (m2 + 1) * k2 / fb / 1e12
    del A, base, G, As, Bm
    # the same factorisation at the other batch sizes of SURVEY 8d (1, 64, 256, 1024)
    by_batch = {}
    for bb in (1, 256, 1024):
        Gb = torch.randn(bb, n, n, dtype=torch.float64, device=dev, generator=g) / n ** 0.5
        Bb = torch.baddbmm(torch.eye(n, dtype=torch.float64, device=dev).expand(bb, n, n), Gb,
                           Gb.transpose(1, 2))
        del Gb
        Ab = Bb.clone()
        ib = torch.zeros(bb, dtype=torch.int32, device=dev)
        tb = None
        for _ in range(reps):
            Ab.copy_(Bb)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            _lib._chk(_lib._L.gpmpc_potrf_batched_dev(ctx.h, n, bb, Ab.data_ptr(), n, n * n,
                                                       ib.data_ptr()), "potrf_batched_dev")
            e1.record(stream)
            ctx.sync()
            el = e0.elapsed_time(e1) * 1e-3
            tb = el if tb is None else min(tb, el)
        assert int(ib.abs().sum().item()) == 0
        fb_ = bb * (n ** 3 / 3.0 + n ** 2 / 2.0 + n / 6.0) / tb / 1e12
        by_batch[str(bb)] = {"ms": round(tb * 1e3, 3), "tflops": round(fb_, 3),
                             "frac_fp64_peak": round(fb_ / FP64_PEAK_TFLOPS, 4)}
        del Ab, Bb, ib
    by_batch[str(batch)] = {"ms": round(t * 1e3, 3), "tflops": round(tf, 3),
                            "frac_fp64_peak": round(tf / FP64_PEAK_TFLOPS, 4)}
    return dict(n=n, batch=batch, ms=round(t * 1e3, 3), tflops=round(tf, 3),
                frac_fp64_peak=round(tf / FP64_PEAK_TFLOPS, 4),
                by_batch=dict(sorted(by_batch.items(), key=lambda kv: int(kv[0]))),
                syrk_potrf={"shapes": "trailing updates (n-t0) x 128, t0 = 128..896", "gflop": round(syrk_flops / 1e9, 2),
                            "ms": round(best * 1e3, 3), "tflops": round(syrk_tf, 3),
                            "frac_fp64_peak": round(syrk_tf / FP64_PEAK_TFLOPS, 4)},
                syrk_fitc={"shape": "B = I + A A^T, A 2000 x 4000 (config 5 FITC)",
                           "gflop": round(m2 * (m2 + 1) * k2 / 1e9, 2), "ms": round(fb * 1e3, 3),
                           "tflops": round(fitc_tf, 3), "frac_fp64_peak": round(fitc_tf / FP64_PEAK_TFLOPS, 4)})


def lml_bench(ctx, n=1000, sets=14, reps=3, cpu=True):
    """one finite-difference gradient of ExactGP.optimize_hyperparameters
    (exact_gp.py:357-421) for the default 3-DoF GP -- the LML at 14 parameter sets
    (13 SE-ARD parameters + the base point), n = 1000 training points -- as one
    gpmpc_gp_lml_batched call (host-boundary time), next to the numpy restatement
    (the reference's per-set ExactGP.fit, one host core)."""
    from gp_mpc_rocket_landing_amd import _lib
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.gp.features import Simple3DoFFeatureExtractor
    X, U, D = synthetic_training_data(n, seed=0)
    Z = Simple3DoFFeatureExtractor().extract_batch(X, U)
    rs = np.random.RandomState(2)
    P = np.concatenate([np.zeros(12), [np.log(1e-4)]]) + 0.2 * rs.normal(size=(sets, 13))
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        lml, _ = _lib.gp_lml_batched(ctx, _lib.SE_ARD, Z, D[:, 1], np.exp(P[:, 1:-1]),
                                     np.exp(P[:, 0]), np.exp(P[:, -1]))
        ts.append(time.perf_counter() - t0)
    out = {"workload": f"LML at {sets} SE-ARD parameter sets, n = {n} (one FD gradient)",
           "ms": round(min(ts) * 1e3, 3), "gradients_per_s": round(1.0 / min(ts), 2)}
    if cpu:
        from threadpoolctl import threadpool_limits
        from oracle import gp_oracle   # the CPU leg: the restatement, timed as the baseline
        with threadpool_limits(1):
            t0 = time.perf_counter()
            ref = [gp_oracle.lml_at(Z, D[:, 1], np.exp(p[0]), np.exp(p[1:-1]), np.exp(p[-1]))[0] for p in P]
            tc = time.perf_counter() - t0
        out["cpu_ms_1core"] = round(tc * 1e3, 2)
        out["max_rel_diff_vs_cpu"] = float(np.max(np.abs(lml - ref) / np.abs(ref)))
    return out


def append_bench(ctx, n=1000, k=10, reps=3):
    """k new residual observations into the n = 1000 exact GP of
    the control loop -- the O(n^2 k) device append (gpmpc_gp_append) vs the full
    device refit of the n + k rows it is equivalent to (host-boundary times)."""
    from gp_mpc_rocket_landing_amd import _lib
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.gp.features import Simple3DoFFeatureExtractor
    X, U, D = synthetic_training_data(n + k, seed=0)
    Z = Simple3DoFFeatureExtractor().extract_batch(X, U)
    ta, tf = [], []
    for _ in range(reps):
        h = _lib.ExactGPHandle(ctx, _lib.SE_ARD, Z[:n], D[:n], np.ones(11), 1.0, 1e-4)
        t0 = time.perf_counter()
        ok = h.append(Z[n:], D)
        ta.append(time.perf_counter() - t0)
        assert ok
        t0 = time.perf_counter()
        h2 = _lib.ExactGPHandle(ctx, _lib.SE_ARD, Z, D, np.ones(11), 1.0, 1e-4)
        tf.append(time.perf_counter() - t0)
        del h, h2
    return {"workload": f"append {k} rows to the n = {n} exact GP (3 outputs)",
            "append_ms": round(min(ta) * 1e3, 3), "refit_ms": round(min(tf) * 1e3, 3),
            "speedup": round(min(tf) / min(ta), 2)}


def simple3dof_gp_bench(ctx, n=1000, p=20, reps=5, cpu=True):
    """BASELINE configs[1] / SURVEY 8d C2: the Simple3DoFGP(use_sparse=False)
    surface -- add_data(N = 1000) + fit() (features, Gram, Cholesky with the
    jitter ladder, alpha, W = L^-1, LML; 3 outputs, one shared factor) and
    predict_batch of the P = 20 horizon points -- on the GPU (host-boundary
    times: H2D inputs and D2H results included), next to the CPU restatement
    (numpy/scipy with the reference's LAPACK calls) on all the box's BLAS
    threads.  Best of ``reps``."""
    from threadpoolctl import threadpool_limits
    from gp_mpc_rocket_landing_amd.data import query_points, synthetic_training_data
    from gp_mpc_rocket_landing_amd.gp import Simple3DoFGP
    X, U, D = synthetic_training_data(n, seed=0)
    Xq, Uq = query_points(X, U, p, seed=7)
    tf, tp = [], []
    for _ in range(reps):
        gp = Simple3DoFGP(use_sparse=False)
        gp.add_data(X, U, D)
        t0 = time.perf_counter(); gp.fit(); tf.append(time.perf_counter() - t0)
        t0 = time.perf_counter(); m, v = gp.predict_batch(Xq, Uq); tp.append(time.perf_counter() - t0)
    out = {"workload": f"Simple3DoFGP(use_sparse=False) fit N={n} + predict {p} points (3 outputs)",
           "fit_ms": round(min(tf) * 1e3, 3), "predict_ms": round(min(tp) * 1e3, 3)}
    if cpu:
        from oracle import gp_oracle   # the CPU leg: the restatement, timed as the baseline
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        cf, cp = [], []
        with threadpool_limits(threads):
            for _ in range(max(2, reps // 2)):
                t0 = time.perf_counter()
                st = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
                cf.append(time.perf_counter() - t0)
                t0 = time.perf_counter()
                mo, vo = gp_oracle.exact_predict(st, gp_oracle.features_3dof(Xq, Uq))
                cp.append(time.perf_counter() - t0)
        out.update(cpu_fit_ms=round(min(cf) * 1e3, 3), cpu_predict_ms=round(min(cp) * 1e3, 3),
                   cpu_threads=threads, fit_speedup=round(min(cf) / min(tf), 2),
                   predict_speedup=round(min(cp) / min(tp), 2),
                   max_rel_mean_diff=float(np.max(np.abs(m - mo) / np.maximum(np.abs(mo), st["y_std"]))))
    return out


def single_landing_bench(ctx, gp, steps=100, reps=3):
    """BASELINE configs[2] / SURVEY 8d C3: ONE closed-loop landing (seed 42,
    108 control steps to touchdown) on one MI355X -- the fleet with B = 1, every
    control step = features + K* Gram, variance/mean GEMM, QP + ADMM + plant
    (the 1024-landing step's kernels at batch 1).  Times ``steps`` steps from
    the initial state (device-resident, one sync at the end)."""
    from gp_mpc_rocket_landing_amd.fleet import Fleet, initial_conditions
    f = Fleet(ctx, gp, 1)
    ts = []
    try:
        x0 = initial_conditions(1)
        for _ in range(reps):
            f.reset(x0)
            ctx.sync()
            t0 = time.perf_counter()
            f.step(steps)
            ctx.sync()
            ts.append(time.perf_counter() - t0)
        rec, _ = f.read()
    finally:
        f.close()
    t = min(ts)
    return {"workload": "1 landing (seed 42), GP N=1000 + RTI QP per step, fleet B=1",
            "steps": int(rec[0, 1]), "us_per_step": round(t / steps * 1e6, 2),
            "steps_per_s": round(steps / t, 1)}


def surface_single_landing_bench(ctx, steps=100, reps=2):
    """the drop-in surface timed, as an unchanged reference caller
    drives it -- MonteCarloSimulator.run_single (monte_carlo.py:491-516): per control
    step the incremental target (:497-500), ``GPMPC(dyn, Simple3DoFGP(use_sparse=False),
    GPMPCConfig(N=20)).solve(x, target)``, u0 into the plant (+ the drag residual the GP
    learns).  Each solve is the host mirror's path: one device GP posterior call for
    the N horizon points, host QP assembly (mpc/qp_builder.py), one device ADMM call;
    with GPMPCConfig's default use_gp_uncertainty=True also the covariance
    propagation (one batched GP call + the device covariance kernel).  Beside it the
    same loop with use_gp_uncertainty=False.  The fleet's B = 1 figure
    (``single_landing``) is the device-resident form of the same step."""
    from gp_mpc_rocket_landing_amd.data import drag_accel, synthetic_training_data
    from gp_mpc_rocket_landing_amd.dynamics import create_normalized_rocket
    from gp_mpc_rocket_landing_amd.fleet import initial_conditions
    from gp_mpc_rocket_landing_amd.gp import Simple3DoFGP
    from gp_mpc_rocket_landing_amd.mpc import GPMPC, GPMPCConfig
    X, U, D = synthetic_training_data(1000, seed=0)
    gp = Simple3DoFGP(use_sparse=False)
    gp.add_data(X, U, D)
    gp.fit()
    dyn = create_normalized_rocket()
    x0 = initial_conditions(1)[0]
    out = {"workload": "1 landing (seed 42), GPMPC(dyn, Simple3DoFGP(use_sparse=False), GPMPCConfig(N=20))"
                       ".solve per step, monte_carlo.py:491-516 protocol", "steps": steps}
    for name, unc in (("us_per_step", True), ("us_per_step_no_uncertainty", False)):
        ts = []
        for _ in range(reps):
            ctl = GPMPC(dyn, gp, GPMPCConfig(N=20, dt=0.1, use_gp_uncertainty=unc))
            x = x0.copy()
            done = 0
            t0 = time.perf_counter()
            for _ in range(steps):
                tgt = x.copy(); tgt[4:7] = 0.0; tgt[1] = max(0.5, x[1] - 2.0)
                sol = ctl.solve(x, tgt)
                if not sol.success:
                    break
                xn = dyn.step(x, sol.u0, 0.1)
                xn[4:7] += drag_accel(x)[0] * 0.1
                x = xn
                done += 1
                if x[1] < 1.0:   # the protocol's landing check (altitude < 1) ends the flight
                    break
            ts.append((time.perf_counter() - t0) / max(done, 1))
        out[name] = round(min(ts) * 1e6, 1)
        out["steps_flown" if unc else "steps_flown_no_uncertainty"] = done
    out["steps_per_s"] = round(1e6 / out["us_per_step"], 1)
    out["us_per_step_host_propagation"] = _host_propagation_us(
        lambda: GPMPC(dyn, gp, GPMPCConfig(N=20, dt=0.1)), dyn, x0, steps)
    return out


def _host_propagation_us(make, dyn, x0, steps, drag=True):
    """The same loop with UncertaintyPropagator's per-step host loop (use_device False: one
    batched GP call per horizon step + host dynamics, as before the device recursion)."""
    from gp_mpc_rocket_landing_amd.data import drag_accel
    from gp_mpc_rocket_landing_amd.mpc import UncertaintyPropagator
    UncertaintyPropagator.use_device = False
    ctl = make()
    try:
        x = x0.copy()
        done = 0
        t0 = time.perf_counter()
        for _ in range(steps):
            tgt = x.copy(); tgt[4:7] = 0.0; tgt[1] = max(0.5, x[1] - 2.0)
            sol = ctl.solve(x, tgt)
            if not sol.success:
                break
            xn = dyn.step(x, sol.u0, 0.1)
            if drag:
                xn[4:7] += drag_accel(x)[0] * 0.1
            x = xn
            done += 1
            if drag and x[1] < 1.0:
                break
        return round((time.perf_counter() - t0) / max(done, 1) * 1e6, 1)
    finally:
        UncertaintyPropagator.use_device = True
        if hasattr(ctl, "close"):
            ctl.close()


def surface_gpmpc6_bench(ctx, steps=30, reps=2):
    """The reference's own 14-state surface as an unchanged caller drives it:
    ``GPMPC(Rocket6DoFDynamics(), StructuredRocketGP(StructuredGPConfig()), GPMPCConfig())``
    (the reference defaults: FITC, 50 inducing points, 1000 rows; N = 20) ``.solve(x, target)``
    per step under the Monte-Carlo protocol (monte_carlo.py:495-512: incremental target, u0
    into the plant).  Each solve is one gpmpc_rollout6_solve call (batch 1); with the default
    use_gp_uncertainty=True also the host-loop covariance propagation (one batched GP call
    per horizon step + the device covariance kernel).  Beside it the same loop without."""
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFDynamics
    from gp_mpc_rocket_landing_amd.mpc import GPMPC, GPMPCConfig
    from gp_mpc_rocket_landing_amd.rollouts6 import fit_structured_gp, initial_conditions_6dof
    gp = fit_structured_gp(1000, 50, seed=0)
    dyn = Rocket6DoFDynamics()
    x0 = initial_conditions_6dof(1)[0]
    out = {"workload": "1 landing, GPMPC(Rocket6DoFDynamics(), StructuredRocketGP() [FITC M=50, 1000 rows], "
                       "GPMPCConfig()).solve per step, monte_carlo.py:495-512 protocol", "steps": steps}
    for name, unc in (("us_per_step", True), ("us_per_step_no_uncertainty", False)):
        ts = []
        for _ in range(reps):
            ctl = GPMPC(dyn, gp, GPMPCConfig(use_gp_uncertainty=unc))
            try:
                x = x0.copy()
                done = 0
                t0 = time.perf_counter()
                for _ in range(steps):
                    tgt = x.copy(); tgt[4:7] = 0.0; tgt[1] = max(0.5, x[1] - 2.0)
                    sol = ctl.solve(x, tgt)
                    x = dyn.step(x, sol.u0, 0.1)
                    done += 1
                ts.append((time.perf_counter() - t0) / max(done, 1))
            finally:
                ctl.close()
        out[name] = round(min(ts) * 1e6, 1)
    out["steps_per_s"] = round(1e6 / out["us_per_step"], 1)
    out["us_per_step_host_propagation"] = _host_propagation_us(lambda: GPMPC(dyn, gp, GPMPCConfig()), dyn, x0,
                                                               steps, drag=False)
    return out


def fleet_fitc_bench(ctx, batch=1024, steps=20, warmup=5):
    """the fleet on the reference-default Simple3DoFGP() -- FITC,
    50 kmeans2 inducing points (structured_gp.py:423-428) -- gpmpc_fleet_create_fitc:
    the BASELINE configs[3] fleet with that GP, timed like the headline (device-resident,
    one sync at the end)."""
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp_sparse, initial_conditions
    h = fit_gp_sparse(n_train=1000, n_inducing=50, seed=0)
    fl = Fleet(ctx, h, batch)
    try:
        fl.reset(initial_conditions(batch))
        fl.step(warmup)
        ctx.sync()
        rec0, _ = fl.read()
        t0 = time.perf_counter()
        fl.step(steps)
        ctx.sync()
        el = time.perf_counter() - t0
        rec1, _ = fl.read()
    finally:
        fl.close()
    done = float(np.sum(rec1[:, 1] - rec0[:, 1]))
    return {"workload": f"{batch} landings, Simple3DoFGP() default: FITC M=50 (mean as written), N=20, RTI",
            "steps": steps, "ms_per_step": round(el / steps * 1e3, 4),
            "control_steps_per_s": round(done / el, 1),
            "admm_iters_per_solve": round(float(np.sum(rec1[:, 11] - rec0[:, 11])) / max(done, 1.0), 2)}


def qp_status_histogram(fl, steps=10):
    """Status of every landing's QP over ``steps`` further control steps of the
    bench fleet (untimed): solved / solved inaccurate / maximum iterations
    reached, and the ADMM iteration counts (25 or 50: termination is checked
    every 25 iterations, max_iter 50)."""
    from gp_mpc_rocket_landing_amd.fleet import REC_ADMM_ITERS, REC_LAST_STATUS, REC_OUTCOME
    names = {1: "solved", 2: "solved_inaccurate", -2: "max_iter_reached"}
    hist, iters = {}, {}
    rec0, _ = fl.read()
    for _ in range(steps):
        fl.step(1)
        rec1, _ = fl.read()
        run = (rec0[:, REC_OUTCOME] == 0) & (rec1[:, 1] > rec0[:, 1])
        for s_, c in zip(*np.unique(rec1[run, REC_LAST_STATUS].astype(int), return_counts=True)):
            k = names.get(int(s_), str(int(s_)))
            hist[k] = hist.get(k, 0) + int(c)
        d = (rec1[run, REC_ADMM_ITERS] - rec0[run, REC_ADMM_ITERS]).astype(int)
        for s_, c in zip(*np.unique(d, return_counts=True)):
            iters[str(int(s_))] = iters.get(str(int(s_)), 0) + int(c)
        rec0 = rec1
    tot = max(1, sum(hist.values()))
    return {"solves": tot, "status": hist, "status_frac": {k: round(v / tot, 4) for k, v in hist.items()},
            "admm_iterations": iters}


def gpmpc_loop_bench(ctx, gp, batch=1024, reps=3, sqp_iters=10):
    """GPMPC.solve's own loop on the fleet (gp_mpc.py:296-353; sqp_iters = 10,
    stop at 1e-4): every control step = up to 10 passes of GP posterior at the
    current plan + QP around it.  With the 1e-4 ADMM the loop never meets the
    1e-4 stop within 10 passes (DESIGN D14), so every landing runs all 10
    passes of its first step and ends DIVERGENCE, as the oracle does: one
    timed step from reset = 10 full passes over the fleet."""
    from gp_mpc_rocket_landing_amd.fleet import Fleet, initial_conditions
    f = Fleet(ctx, gp, batch, sqp_iters=sqp_iters, sqp_tol=1e-4)
    ts = []
    try:
        x0 = initial_conditions(batch)
        for _ in range(reps):
            f.reset(x0)
            ctx.sync()
            t0 = time.perf_counter()
            f.step(1)
            ctx.sync()
            ts.append(time.perf_counter() - t0)
        rec, _ = f.read()
    finally:
        f.close()
    t = min(ts)
    out = {"workload": f"{batch} landings, one GPMPC.solve each = {sqp_iters} passes of "
                       "(GP posterior N=20 x 1000 pts + RTI QP), stop 1e-4",
           "ms": round(t * 1e3, 3), "solves_per_s": round(batch / t, 1),
           "qp_solves_per_s": round(batch * sqp_iters / t, 1),
           "admm_iters_per_qp": round(float(rec[:, 11].sum()) / (batch * sqp_iters), 2),
           "outcomes": {str(int(c)): int(np.sum(rec[:, 0] == c)) for c in np.unique(rec[:, 0])}}
    # the SQP passes' own tight QP settings (gpmpc_fleet_config.sqp_qp, DESIGN D14) and
    # 100 passes: the loop converges at 1e-4 for the first control steps, then a
    # step fails to converge and the landing ends DIVERGENCE
    nb, passes = 64, 100
    f = Fleet(ctx, gp, nb, sqp_iters=passes, sqp_tol=1e-4, sqp_qp=dict(eps_abs=1e-7, eps_rel=1e-7, max_iter=2000))
    try:
        f.reset(initial_conditions(nb))
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(12):
            f.step(1)
        ctx.sync()
        t = time.perf_counter() - t0
        rec, _ = f.read()
    finally:
        f.close()
    out["tight_qp"] = {"workload": f"{nb} landings, up to 12 control steps of up to {passes} passes, "
                                   "sqp_qp eps 1e-7 / max_iter 2000, stop 1e-4",
                       "s": round(t, 3), "steps_flown_mean": round(float(rec[:, 1].mean()), 2),
                       "steps_flown_max": int(rec[:, 1].max()),
                       "admm_iters": int(rec[:, 11].sum()),
                       "outcomes": {str(int(c)): int(np.sum(rec[:, 0] == c)) for c in np.unique(rec[:, 0])}}
    return out


def r6_admm_flops(N=30, nx=14, nu=3):
    """Algorithmic fp64 flop of the 6-DoF QP (csrc/fleet6.hip; FMA = 2): per ADMM
    iteration (A'(rho z - y) and A x~ over the constraint non-zeros, the block-
    tridiagonal KKT solve: forward G products, 31 diagonal S^-1 products,
    backward G^T products, ~10 vector ops per variable and row), and per
    factorisation (assembly of P + sigma I + A'RA per stage block, Gauss-Jordan
    S^-1, G = C S^-1, the Schur update)."""
    sz = nx + nu
    n, m = N * sz + nx, nx * (N + 1) + (N * sz + nx) + N + 4 * (N - 1)
    nnz = nx + N * nx * (sz + 1) + n + 3 * N + 2 * 4 * (N - 1)
    kkt = 2 * (N * nx * sz) + 2 * ((N + 1) * sz * sz) + 2 * (N * sz * nx)
    it = 2 * 2 * nnz + kkt + 10 * (n + m)
    fac = (N + 1) * (2 * sz ** 3 + 2 * nx * sz * sz + 2 * nx * nx * sz + 2 * nx * sz * sz)
    return it, fac


def rollouts6_qp_status(ctx, gv, gw, B, max_steps=300, **cfg):
    """Fly B rollouts to termination one step at a time and histogram the status
    of every QP solve (a solve without a solution ends its rollout)."""
    from gp_mpc_rocket_landing_amd.rollouts6 import Rollouts6, initial_conditions_6dof
    names = {1: "solved", 2: "solved_inaccurate", -2: "max_iter_reached", -3: "primal_infeasible",
             3: "primal_infeasible_inaccurate", -4: "dual_infeasible", 4: "dual_infeasible_inaccurate",
             -100: "kkt_factor_failed"}
    ro = Rollouts6(ctx, gv, gw, B, max_steps=max_steps, **cfg)
    hist = {}
    try:
        ro.reset(initial_conditions_6dof(B))
        rec0, _ = ro.read()
        for _ in range(max_steps + 1):
            ro.step(1)
            rec1, _ = ro.read()
            failed = (rec1[:, 0] == 6) & ~np.isin(rec1[:, 14], (1, 2, -2))   # a solve without a solution
            adv = (rec0[:, 0] == 0) & ((rec1[:, 1] > rec0[:, 1]) | failed)
            for s_, c in zip(*np.unique(rec1[adv, 14].astype(int), return_counts=True)):
                k = names.get(int(s_), str(int(s_)))
                hist[k] = hist.get(k, 0) + int(c)
            rec0 = rec1
            if np.all(rec1[:, 0] != 0):
                break
    finally:
        ro.close()
    tot = max(1, sum(hist.values()))
    return {"rollouts": B, "solves": tot, "status": hist, "status_frac": {k: round(v / tot, 4) for k, v in hist.items()},
            "outcomes": {str(int(c)): int(np.sum(rec1[:, 0] == c)) for c in np.unique(rec1[:, 0])},
            "admm_iters_per_solve": round(float(rec1[:, 11].sum()) / max(float(rec1[:, 1].sum()), 1.0), 2)}


# the 6-DoF ADMM setting at which >= 90% of the configs[4] QPs return "solved"
SOLVED_QP6 = dict(max_iter=4000, eps_abs=1e-4, eps_rel=1e-4)


def rollouts6_timed(ctx, gv, gw, batches, max_steps=300, **qp):
    """The configs[4] rollouts flown to termination at the ADMM settings ``qp``
    (timed per batch), plus the QP status of every solve of the first batch."""
    from gp_mpc_rocket_landing_amd.rollouts6 import Rollouts6, initial_conditions_6dof
    out = {"qp": {k: v for k, v in qp.items()}}
    for B in batches:
        ro = Rollouts6(ctx, gv, gw, B, max_steps=max_steps, **qp)
        try:
            ro.reset(initial_conditions_6dof(B)); ro.step(1); ctx.sync()
            ro.reset(initial_conditions_6dof(B)); ctx.sync()
            t0 = time.perf_counter()
            steps = 0
            while steps < max_steps + 1:
                ro.step(10)
                steps += 10
                rec, _ = ro.read()
                if np.all(rec[:, 0] != 0):
                    break
            el = time.perf_counter() - t0
        finally:
            ro.close()
        ctrl = float(rec[:, 1].sum())
        out[str(B)] = {"s": round(el, 4), "rollouts_per_s": round(B / el, 1), "ms_per_step": round(el / steps * 1e3, 3),
                       "control_steps_per_s": round(ctrl / el, 1), "mean_steps_per_rollout": round(ctrl / B, 1),
                       "admm_iters_per_solve": round(float(rec[:, 11].sum()) / max(ctrl, 1.0), 2),
                       "outcomes": {str(int(c)): int(np.sum(rec[:, 0] == c)) for c in np.unique(rec[:, 0])}}
    out["qp_status"] = rollouts6_qp_status(ctx, gv, gw, batches[0], max_steps=max_steps, **qp)
    return out


def rollouts6_bench(ctx, torch=None, batches=(64, 512), max_steps=300):
    """BASELINE configs[4]: 6-DoF GP-MPC rollouts, N = 30, the StructuredRocketGP
    FITC pair at M = 2000 inducing / N = 4000 training rows (csrc/fleet6.hip).
    Every rollout flies to termination (run_experiments initial conditions + a
    random tilt); 64 = one GPU's share of the config's 512 over 8 GPUs, 512 =
    the whole config on one GPU.  The GP fit (host kmeans2 + two device FITC
    fits) is outside the timed region.  Then, untimed: per-kernel times of the
    64-rollout batch (HIP events around each phase on the context stream) with
    the control kernel's roofline object, and the QP status of every solve."""
    from gp_mpc_rocket_landing_amd.rollouts6 import Rollouts6, fit_structured_fitc, initial_conditions_6dof
    t0 = time.perf_counter()
    gv, gw = fit_structured_fitc(ctx, n_train=4000, n_inducing=2000)
    fit_s = time.perf_counter() - t0
    out = {"workload": "6-DoF GPMPC rollouts, N=30, FITC M=2000 / N_train=4000 x 2 GPs, to termination",
           "gp_fit_ms": round(fit_s * 1e3, 1),
           "mean": "as written: K*u alpha, the reference's arithmetic (sparse_gp.py:280-283, SURVEY D1; "
                   "Rollouts6 default); 'corrected_mean' is the same flight with K*u L_uu^-T alpha"}
    for B in batches:
        ro = Rollouts6(ctx, gv, gw, B, max_steps=max_steps)
        try:
            ro.reset(initial_conditions_6dof(B))
            ro.step(1)          # warm-up: first launch of each kernel
            ctx.sync()
            ro.reset(initial_conditions_6dof(B))
            ctx.sync()
            t0 = time.perf_counter()
            steps = 0
            while steps < max_steps + 1:
                ro.step(10)
                steps += 10
                rec, _ = ro.read()
                if np.all(rec[:, 0] != 0):
                    break
            el = time.perf_counter() - t0
        finally:
            ro.close()
        ctrl = float(rec[:, 1].sum())
        out[str(B)] = {"s": round(el, 4), "rollouts_per_s": round(B / el, 1),
                       "control_steps_per_s": round(ctrl / el, 1), "launched_steps": steps,
                       "ms_per_step": round(el / steps * 1e3, 3),
                       "mean_steps_per_rollout": round(ctrl / B, 1),
                       "admm_iters_per_solve": round(float(rec[:, 11].sum()) / max(ctrl, 1.0), 2),
                       "outcomes": {str(int(c)): int(np.sum(rec[:, 0] == c)) for c in np.unique(rec[:, 0])}}
    # per-kernel times (first 20 steps of 64 rollouts) and the QP status of every solve
    B = batches[0]
    ro = Rollouts6(ctx, gv, gw, B, max_steps=max_steps)
    names = {1: "solved", 2: "solved_inaccurate", -2: "max_iter_reached", -3: "primal_infeasible",
             3: "primal_infeasible_inaccurate", -4: "dual_infeasible", 4: "dual_infeasible_inaccurate",
             -100: "kkt_factor_failed"}
    hist = {}
    try:
        ro.reset(initial_conditions_6dof(B))
        ph = []
        if torch is not None:
            stream = torch.cuda.ExternalStream(ctx.stream)
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(20)]
            for k in range(20):
                ev[k][0].record(stream); ro.phases(1)
                ev[k][1].record(stream); ro.phases(2)
                ev[k][2].record(stream); ro.phases(4)
                ev[k][3].record(stream)
            ctx.sync()
            ph = np.array([[ev[k][i].elapsed_time(ev[k][i + 1]) for i in range(3)] for k in range(20)]) * 1e-3
        ro.reset(initial_conditions_6dof(B))
        rec0, _ = ro.read()
        for _ in range(max_steps + 1):
            ro.step(1)
            rec1, _ = ro.read()
            failed = (rec1[:, 0] == 6) & ~np.isin(rec1[:, 14], (1, 2, -2))   # a solve without a solution
            adv = (rec0[:, 0] == 0) & ((rec1[:, 1] > rec0[:, 1]) | failed)
            for s_, c in zip(*np.unique(rec1[adv, 14].astype(int), return_counts=True)):
                k = names.get(int(s_), str(int(s_)))
                hist[k] = hist.get(k, 0) + int(c)
            rec0 = rec1
            if np.all(rec1[:, 0] != 0):
                break
    finally:
        ro.close()
    tot = max(1, sum(hist.values()))
    out["qp_status"] = {"rollouts": B, "solves": tot, "status": hist,
                        "status_frac": {k: round(v / tot, 4) for k, v in hist.items()}}
    # the same controller with ADMM settings at which >= 90% of its QPs
    # return "solved" (scripts/probe.py qp_sweep: max_iter 50 / 100 / 200 / 400 / 1000 / 4000
    # at eps 1e-4 gave 12 / 53 / 75 / 83 / 89 / 96% solved), beside the osqp_rti setting
    out["solved_setting"] = rollouts6_timed(ctx, gv, gw, batches, max_steps, **SOLVED_QP6)
    # the FITC posterior mean (K*u L_uu^-T alpha, SURVEY D1 fixed): the same rollouts timed
    # and their QP statuses, beside the reference's arithmetic above
    out["corrected_mean"] = rollouts6_timed(ctx, gv, gw, batches, max_steps, fitc_mean_as_written=0)
    out["corrected_mean"]["mean"] = "K*u L_uu^-T alpha (fitc_mean_as_written=0)"
    if len(ph):
        pm = ph.mean(axis=0)
        it_f, fac_f = r6_admm_flops()
        iters = float(out[str(B)]["admm_iters_per_solve"])
        # per control launch: B solves x (iterations x per-iteration flop + ~2 factorisations)
        ctl_flop = B * (iters * it_f + 2.0 * fac_f)
        tr, tr_src = pmc_traffic("k_r6_control<false>")
        out["kernels"] = {"predict": {"kernel": "k_r6_predict<false>", "ms": round(pm[0] * 1e3, 4)},
                          "control": {"kernel": "k_r6_control<false>", "ms": round(pm[1] * 1e3, 4)},
                          "plant": {"kernel": "k_r6_plant", "ms": round(pm[2] * 1e3, 4)}}
        out["roofline"] = {"kernel": "k_r6_control<false>", "bound": "mfma", "achieved": round(ctl_flop / pm[1] / 1e12, 5),
                           "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(ctl_flop / pm[1] / 1e12 / FP64_PEAK_TFLOPS, 5),
                           "traffic": tr, "traffic_source": tr_src,
                           "per_launch": f"{B} solves x (iterations x {it_f} + 2 x {fac_f}) fp64 flop",
                           "limiter": "latency: the block-tridiagonal KKT chains (twisted, 15 block steps per end) and the factor sweep, one rollout per CU"}
    return out


def structured_fitc_bench(ctx, reps=2):
    """BASELINE config 5 GP: StructuredRocketGP with FITC M = 2000, N_train = 4000
    (two 3-output GPs, D = 13 translational / 12 rotational features), and one
    batched predict over 512 rollouts x 30 horizon points.  Synthetic features;
    inducing points are a random training subset (host kmeans2 is not timed)."""
    import time
    from gp_mpc_rocket_landing_amd import _lib
    rs = np.random.RandomState(11)
    M, N, P = 2000, 4000, 512 * 30
    fit_t, pred_t = [], []
    for _ in range(reps):
        hs = []
        t0 = time.perf_counter()
        for d in (13, 12):
            X = rs.uniform(0.0, 1.5, (N, d))
            Y = np.stack([np.sin(X.sum(1)), np.cos(X[:, 0]), X[:, 1] ** 2], 1)
            hs.append(_lib.FITCHandle(ctx, X[rs.choice(N, M, replace=False)], X, Y, np.ones(d), 1.0, 1e-4))
        fit_t.append(time.perf_counter() - t0)
        Q = [rs.uniform(0.0, 1.5, (P, d)) for d in (13, 12)]
        t0 = time.perf_counter()
        for h, q in zip(hs, Q):
            h.predict(q)
        pred_t.append(time.perf_counter() - t0)
    f, p = min(fit_t), min(pred_t)
    return {"workload": "StructuredRocketGP FITC, M=2000, N=4000, 2 x 3 outputs (config 5)",
            "fit_ms": round(f * 1e3, 2), "predict_points": P, "predict_ms": round(p * 1e3, 2),
            "predict_points_per_s": round(P / p, 1),
            "note": "host-boundary times (H2D inputs, D2H results) around the device fit/predict"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--landings", type=int, default=1024, help="landings per GPU")
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--train", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-chol", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    # the CPU baseline first: its worker processes start before this process
    # touches the GPU
    cb = None
    if rank == 0 and world0 == 1 and not args.no_cpu:
        cb = cpu_baseline(args.cpu_seconds, n_train=args.train, horizon=args.horizon)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from gp_mpc_rocket_landing_amd import _lib
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions

    ctx = _lib.Context(local)
    gp = fit_gp(ctx, n_train=args.train)
    B = args.landings
    fl = Fleet(ctx, gp, B, horizon=args.horizon)
    fl.reset(initial_conditions(B, seed0=42, first=rank * B))
    for _ in range(args.warmup):
        fl.step(1)
    ctx.sync()
    rec0, _ = fl.read()

    stream = torch.cuda.ExternalStream(ctx.stream)
    K = args.steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(K)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(); ctx.sync()
    t0 = time.perf_counter()
    for k in range(K):
        e = ev[k]
        e[0].record(stream); fl.phases(1)   # query features (+ the K* gram on the GPMPC_POST_CS=0 path)
        e[1].record(stream); fl.phases(4)   # posterior: variance + mean in one MFMA pass
        e[2].record(stream); fl.phases(8)   # posterior finish
        e[3].record(stream); fl.phases(2)   # QP assembly + ADMM + plant
        e[4].record(stream)
    ctx.sync(); torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    rec1, _ = fl.read()
    steps_done = float(np.sum(rec1[:, 1] - rec0[:, 1]))
    admm_iters = float(np.sum(rec1[:, 11] - rec0[:, 11]))
    ph = np.array([[ev[k][i].elapsed_time(ev[k][i + 1]) for i in range(4)] for k in range(K)]) * 1e-3
    ph_mean = ph.mean(axis=0)

    # ---- aggregate over ranks (max time, summed work); one RCCL gather of records
    t = torch.tensor([el, steps_done, admm_iters], dtype=torch.float64, device="cuda")
    if world > 1:
        tmax = t.clone(); dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone(); dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        el_max, steps_all, iters_all = float(tmax[0]), float(tsum[1]), float(tsum[2])
    else:
        el_max, steps_all, iters_all = el, steps_done, admm_iters
    # the one collective, after the timed region: the C-ABI's RCCL gather of the device
    # records (a communicator of one at N = 1).  A set-up failure on any rank is agreed by
    # every rank and falls back to torch.distributed.gather together; `gather` records
    # which path ran and how many ranks RCCL's communicator spanned.
    from gp_mpc_rocket_landing_amd.sharding import gather_shard_records
    all_rec, gather_info = gather_shard_records(ctx, fl.records_dev, rec1, world * B, device="cuda")
    if rank == 0 and world == 1 and gather_info["path"] == "rccl" and not np.array_equal(all_rec, rec1):
        raise RuntimeError("RCCL gather of a world of one does not reproduce the fleet records")

    if rank == 0:
        P = B * args.horizon
        n = args.train
        # per-launch algorithmic work: variance GEMM n^2 P flop
        # (lower-triangular L^-1 times K*^T), K* gram 8 n P bytes written
        var_flops = float(n) * n * P + 2.0 * 3 * n * P      # W K*^T (triangular) + alpha^T K*^T
        gram_bytes = 8.0 * n * P + 8.0 * (P * 12 + n * 12)
        nrt = -(-(n + 3) // 64)
        fin_bytes = 8.0 * P * (nrt + 3 + 6)                 # partials + means in, mean/var out
        it_f, fac_f = admm_flops()
        steps_rank0 = steps_done / K
        admm_flop = (admm_iters / K) * it_f + steps_rank0 * 1.5 * fac_f
        # GPMPC_POST_CS=1 (n <= 1008): the column-stationary kernel forms K* inside its MFMA
        # pass (post.hip), so phase 1 is only the query features; the K* exponentials
        # (P n, ~26 flop each) are extra work not counted in var_flops.  Off by default.
        cs = os.environ.get("GPMPC_POST_CS", "0") != "0" and n <= 1008
        q_bytes = 8.0 * B * ((args.horizon + 1) * 7 + args.horizon * 3) + 8.0 * P * 12
        kern = {
            "gram_Kstar": dict(kernel="k_gram_rows<11, 0>", ms=ph_mean[0] * 1e3, bound="hbm",
                               achieved=gram_bytes / ph_mean[0] / 1e9, peak=HBM_PEAK_GBS, unit="GB/s"),
            "var_mean_gemm_mfma": dict(kernel="k_gemm128<1>", ms=ph_mean[1] * 1e3, bound="mfma",
                                       achieved=var_flops / ph_mean[1] / 1e12, peak=FP64_PEAK_TFLOPS,
                                       unit="TFLOP/s"),
            "post_finish": dict(kernel="k_post_finish", ms=ph_mean[2] * 1e3, bound="hbm",
                                achieved=fin_bytes / ph_mean[2] / 1e9, peak=HBM_PEAK_GBS,
                                unit="GB/s"),
            "qp_admm_plant": dict(kernel=CONTROL_KERNEL, ms=ph_mean[3] * 1e3, bound="mfma",
                                  achieved=admm_flop / ph_mean[3] / 1e12, peak=FP64_PEAK_TFLOPS,
                                  unit="TFLOP/s"),
        }
        if cs:
            kern.pop("gram_Kstar")
            kern.pop("var_mean_gemm_mfma")
            kern = {"query_features": dict(kernel="k_fleet_queries", ms=ph_mean[0] * 1e3, bound="hbm",
                                           achieved=q_bytes / ph_mean[0] / 1e9, peak=HBM_PEAK_GBS, unit="GB/s"),
                    "posterior_mfma": dict(kernel="k_post_cs<11>", ms=ph_mean[1] * 1e3, bound="mfma",
                                           achieved=var_flops / ph_mean[1] / 1e12, peak=FP64_PEAK_TFLOPS,
                                           unit="TFLOP/s"),
                    **kern}
        if os.environ.get("GPMPC_FLEET_FUSE_POST", "1") != "0":
            # the posterior finish runs inside the control kernel (each landing
            # finishes its own 20 queries while it assembles its QP)
            kern.pop("post_finish")
        for v in kern.values():
            v["frac"] = v["achieved"] / v["peak"]
            for kk in ("ms", "achieved", "frac"):
                v[kk] = round(v[kk], 5)
            tb, src = pmc_traffic(v["kernel"])
            v["traffic"] = tb
        # roofline object: the kernel that dominates the step's time.  The control
        # kernel (ADMM) is priced against the FP64 compute ceiling (vector = matrix,
        # 78.6 TF); its limiter is the serial KKT dependency chain of one wave per
        # landing, not HBM or MFMA.
        dom = max(kern, key=lambda k: kern[k]["ms"])
        d = kern[dom]
        roof = dict(kernel=d["kernel"], bound=d["bound"], achieved=d["achieved"], peak=d["peak"],
                    unit=d["unit"], frac=d["frac"], traffic=d["traffic"],
                    per_launch={"qp_admm_plant": "ADMM iterations x block-KKT iteration flops + "
                                                 "factorisations (admm_flops)",
                                "var_mean_gemm_mfma": "n^2 P + 6 n P flop",
                                "posterior_mfma": "n^2 P + 6 n P flop (W K*^T, lower-triangular W, "
                                                  "and alpha^T K*^T; K* formed in the pass, not counted)",
                                "query_features": "8 B ((N+1) 7 + 3 N) + 96 P bytes",
                                "gram_Kstar": "8 n P + 8 d (P+n) bytes",
                                "post_finish": "8 P (row tiles + 9) bytes"}[dom],
                    traffic_source=pmc_traffic(d["kernel"])[1], launches_per_step=1)
        ctl_limiter = ("latency: serial block-tridiagonal KKT chain, one chain wave per landing "
                       "(each on its own SIMD), four landings per CU; ~10 KB of state in/out per "
                       "landing-step, the rest of the measured traffic is register-spill scratch")
        kern["qp_admm_plant"]["limiter"] = ctl_limiter
        if dom == "qp_admm_plant":
            roof["limiter"] = ctl_limiter
        out = {
            "metric": "GP-MPC control steps/sec (N=20, 1000 GP pts)",
            "value": round(steps_all / el_max, 2),
            "unit": "control steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(el_max / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (generator G training set; run_experiments.py initial conditions)",
            "config": {"workload": "fleet of closed-loop 3-DoF GP-MPC landings (BASELINE configs[3] "
                                   "shapes), RTI QP per step",
                       "landings_per_gpu": B, "horizon": args.horizon, "gp_train_points": n,
                       "qp": "n=207 m=354, OSQP settings of osqp_rti.py", "parallelism": f"dp{world}"},
            "roofline": roof,
            "kernels": kern,
            "admm_iters_per_solve": round(iters_all / max(steps_all, 1.0), 2),
            "landing_steps_per_gpu_step": round(steps_done / K, 1),
        }
        out["gather"] = gather_info
        if all_rec is not None:
            oc = all_rec[:, 0]
            out["outcomes"] = {str(int(c)): int(np.sum(oc == c)) for c in np.unique(oc)}
        out["qp_status"] = qp_status_histogram(fl)
        if not args.no_chol and world == 1:  # single-GPU legs: the N > 1 runs keep to the metric
            legs = [("single_landing", lambda: single_landing_bench(ctx, gp)),
                    ("surface_single_landing", lambda: surface_single_landing_bench(ctx)),
                    ("surface_gpmpc6", lambda: surface_gpmpc6_bench(ctx)),
                    ("fleet_fitc", lambda: fleet_fitc_bench(ctx)),
                    ("gpmpc_loop", lambda: gpmpc_loop_bench(ctx, gp)),
                    ("simple3dof_gp", lambda: simple3dof_gp_bench(ctx, cpu=not args.no_cpu)),
                    ("cholesky", lambda: cholesky_bench(ctx, torch)),
                    ("structured_fitc", lambda: structured_fitc_bench(ctx)),
                    ("rollouts6", lambda: rollouts6_bench(ctx, torch)),
                    ("lml_batched", lambda: lml_bench(ctx, cpu=not args.no_cpu)),
                    ("gp_append", lambda: append_bench(ctx))]
            for name, leg in legs:   # a failing leg is recorded as such; the others still run
                try:
                    out[name] = leg()
                except Exception as e:  # noqa: BLE001
                    out[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
        if cb is not None:
            cb["value"] = round(cb["value"], 3)
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    fl.close()


if __name__ == "__main__":
    main()
