"""Measurement probes for the GPU box, one subcommand each (run from the repo root,
through gpurun, alone or under scripts/profile.sh for a kernel trace / PMC pass):

  single                    the single-landing step (configs[2]: the fleet at B = 1), 100 steps x 3
  step [B] [steps]          the bench's control step alone (B landings, N = 20, GP n = 1000)
  stamps [B] [steps]        landing 0's control-kernel phase cycles (gpmpc_fleet_set_stamps)
  placement [B]             where the control kernel's waves land (HW_ID) and per-landing spans
  streams                   the fleet as 1 / 2 / 4 shards on as many streams: free-running, and
                            pipelined (shard posteriors serialised, controls beside them)
  fit                       Simple3DoFGP.fit through the surface and the bare C-ABI fit, x 8
  append [k]                gpmpc_gp_append of k rows into the n = 1000 GP against a refit
  chol                      bench.py's Cholesky leg (JSON)
  potrf [NxB,...]           batched potrf ms / TFLOP/s / error per shape
  potrf_streams             batched potrf split over 1 / 2 / 4 streams
  syrk_fitc                 the config-5 FITC SYRK (2000 x 4000), 30 launches (JSON)
  gemm_loop [n]             the 128-tile MFMA loop's steady state: lower SYRK n = k (JSON)
  trsm                      trsm_lower / potrs at n = 128 and 1000, for a kernel trace
  rollouts6 [64,512]        bench.py's configs[4] rollouts leg (JSON)
  qp_sweep [B] [mi:eps,..]  configs[4] ADMM settings: status histogram and timing per setting
  surface [reps] [prof]     bench.py's 3-DoF drop-in surface leg (JSON); prof: under cProfile
  surface6 [reps] [prof]    bench.py's 14-state drop-in surface leg (JSON); prof: under cProfile
                            (GPMPC_QP_STAMPS=1 beside either: k_qp_batched phase cycles on stderr,
                            summarised by scripts/pmc.py qpstamps)
"""
import json
import os
import sys
import time
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gp_mpc_rocket_landing_amd import _lib  # noqa: E402

FP64_PEAK = 78.6e12


def _torch():
    import torch
    return torch


def _fleet():
    from gp_mpc_rocket_landing_amd import fleet
    return fleet


def _events(torch, stream, fn):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    fn()
    e1.record(stream)
    return e0, e1


# ---- the 3-DoF fleet -------------------------------------------------------------------
def single():
    F = _fleet()
    ctx = _lib.Context(0)
    f = F.Fleet(ctx, F.fit_gp(ctx, n_train=1000), 1)
    for _ in range(3):
        f.reset(F.initial_conditions(1))
        ctx.sync()
        t0 = time.perf_counter()
        f.step(100)
        ctx.sync()
        print(f"{(time.perf_counter() - t0) / 100 * 1e6:.1f} us per step", flush=True)
    f.close()


def step(B="1024", steps="10"):
    F = _fleet()
    B, steps = int(B), int(steps)
    ctx = _lib.Context(0)
    fl = F.Fleet(ctx, F.fit_gp(ctx, n_train=1000), B)
    fl.reset(F.initial_conditions(B))
    fl.step(3)
    ctx.sync()
    t0 = time.perf_counter()
    fl.step(steps)
    ctx.sync()
    dt = (time.perf_counter() - t0) / steps
    print(f"{B} landings: {dt * 1e3:.3f} ms per step, {B / dt / 1e6:.3f} M steps/s", flush=True)
    fl.close()


def stamps(B="1024", steps="4"):
    """Slots: 0 assembly, 1 scaling, 2 factor, 3 rhs, 4 KKT block solve (rest), 5 x/z/y
    update, 6 checks + adaptive rho, 7 plant + tail, 8-10 the KKT solve's forward chain /
    diagonal blocks / backward chain, 11/12 the rhs and update compute before their
    barriers, 14 realtime (100 MHz), 15 total shader cycles."""
    torch, F = _torch(), _fleet()
    B, steps = int(B), int(steps)
    ctx = _lib.Context(0)
    fl = F.Fleet(ctx, F.fit_gp(ctx, n_train=1000), B, horizon=20)
    fl.reset(F.initial_conditions(B))
    fl.step(3)
    st = torch.zeros(16, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    _lib._chk(_lib._L.gpmpc_fleet_set_stamps(fl.h, st.data_ptr()), "stamps")
    rec0, _ = fl.read()
    fl.step(steps)
    ctx.sync()
    rec1, _ = fl.read()
    s = st.cpu().numpy().astype(np.float64)
    it = rec1[0, 11] - rec0[0, 11]
    names = ["assembly", "scaling", "factor", "rhs", "kkt_solve(rest)", "update", "checks", "tail",
             "kkt_forward", "kkt_diagonal", "kkt_backward", "rhs_compute", "update_compute", "unused"]
    tot = s[15]
    print(f"B={B} landing 0: {steps} steps, {it:.0f} ADMM iterations, {tot:.0f} shader cycles "
          f"({s[14] / 100e6 * 1e6:.1f} us realtime)")
    for i, nm in enumerate(names):
        print(f"  {nm:10s} {s[i]:10.0f} cycles  {s[i] / tot * 100:5.1f}%  {s[i] / max(it, 1):8.0f} per iteration")
    fl.close()


def placement(B="1024"):
    """HW_ID (SIMD, CU, SE, XCC) of each landing's two waves and its start / end realtime
    over one control step; chain-wave sharing per SIMD and span by ADMM iterations.
    (GPMPC_FLEET_SIMD=0 for the chain-sharing lines: by default each workgroup claims
    its chain SIMD at run time.)"""
    torch, F = _torch(), _fleet()
    B = int(B)
    ctx = _lib.Context(0)
    fl = F.Fleet(ctx, F.fit_gp(ctx, n_train=1000), B, horizon=20)
    fl.reset(F.initial_conditions(B))
    fl.step(3)
    tr = torch.zeros(B * 4, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    _lib._chk(_lib._L.gpmpc_fleet_set_trace(fl.h, tr.data_ptr()), "trace")
    rec0, _ = fl.read()
    fl.step(1)
    ctx.sync()
    rec1, _ = fl.read()
    t = tr.cpu().numpy().reshape(B, 4).view(np.uint64)
    its = rec1[:, 11] - rec0[:, 11]
    span = (t[:, 1].astype(np.float64) - t[:, 0].astype(np.float64)) / 100.0

    def decode(v):
        v = int(v)
        hw = v & 0xFFFFFFFF
        return (((v >> 32) & 15), (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15), (hw >> 4) & 3

    w = [decode(v) for v in t[:, 2]]
    w1 = [decode(v) for v in t[:, 3]]
    per_cu = Counter(c for c, _ in w)
    print(f"{len(per_cu)} CUs used, landings per CU {Counter(per_cu.values())}")
    print(f"both waves on one CU: {sum(a[0] == b[0] for a, b in zip(w, w1))}/{B}")
    print(f"chain waves per SIMD: {Counter(Counter(w).values())}; all waves per SIMD: "
          f"{Counter(Counter(w + w1).values())}")
    for k in sorted(set(its.astype(int))):
        m = its == k
        print(f"  it={k:3d}: {m.sum():4d} landings, span {span[m].mean():7.1f} us "
              f"(min {span[m].min():.1f}, max {span[m].max():.1f})")
    fl.close()


def streams(steps="20", warm="3"):
    """The 1024-landing fleet as S shards (fleet_batch 1024: every landing's bits are the
    whole fleet's) on S streams.  Free-running: each shard steps on its own stream.
    Pipelined: the shards' posterior phases (mask 13) serialised in shard order through
    events, each shard's control kernel (mask 2) beside the next shard's posterior.
    Checks the pipelined records against the whole fleet's."""
    torch, F = _torch(), _fleet()
    steps, warm, B = int(steps), int(warm), 1024
    ctx0 = _lib.Context(0)
    gp = F.fit_gp(ctx0, n_train=1000)
    x0 = F.initial_conditions(B)

    def timed(ctxs, fn):
        for c in ctxs:
            c.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        for c in ctxs:
            c.sync()
        return round((time.perf_counter() - t0) / steps * 1e3, 4)

    out = {}
    whole = F.Fleet(ctx0, gp, B, horizon=20)
    whole.reset(x0)
    whole.step(warm)
    out["whole_step_ms"] = timed([ctx0], lambda: whole.step(1))
    out["whole_post_ms"] = timed([ctx0], lambda: whole.phases(13))
    out["whole_ctl_ms"] = timed([ctx0], lambda: whole.phases(2))
    whole.close()
    for S in (2, 4):
        n = B // S
        ctxs = [ctx0] + [_lib.Context(0) for _ in range(S - 1)]
        strm = [torch.cuda.ExternalStream(c.stream) for c in ctxs]

        def shards():
            sh = []
            for s in range(S):
                f = F.Fleet(ctxs[s], gp, n, fleet_batch=B, horizon=20)
                f.reset(x0[s * n:(s + 1) * n])
                sh.append(f)
            for c in ctxs:
                c.sync()
            return sh

        sh = shards()
        for f in sh:
            f.step(warm)
        out[f"S{S}_free_step_ms"] = timed(ctxs, lambda: [f.step(1) for f in sh])
        out[f"S{S}_post_one_shard_ms"] = timed(ctxs, lambda: sh[0].phases(13))
        out[f"S{S}_ctl_one_shard_ms"] = timed(ctxs, lambda: sh[0].phases(2))
        for f in sh:
            f.close()
        sh = shards()
        evs = [torch.cuda.Event() for _ in range(S)]
        prev = [None]

        def pipelined():
            for s in range(S):
                if prev[0] is not None:
                    strm[s].wait_event(prev[0])
                sh[s].phases(13)
                evs[s].record(strm[s])
                prev[0] = evs[s]
                sh[s].phases(2)

        for _ in range(warm):
            pipelined()
        out[f"S{S}_pipelined_step_ms"] = timed(ctxs, pipelined)
        rec_p = np.concatenate([f.read()[0] for f in sh])
        w = F.Fleet(ctx0, gp, B, horizon=20)
        w.reset(x0)
        w.step(warm + steps)
        out[f"S{S}_pipelined_bits_equal"] = bool(np.array_equal(rec_p, w.read()[0], equal_nan=True))
        w.close()
        for f in sh:
            f.close()
    print(json.dumps(out), flush=True)


# ---- GP fit / append ---------------------------------------------------------------------
def fit():
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.gp import Simple3DoFGP
    from gp_mpc_rocket_landing_amd.gp.features import Simple3DoFFeatureExtractor
    X, U, D = synthetic_training_data(1000, seed=0)
    Z = Simple3DoFFeatureExtractor().extract_batch(X, U)
    ctx = _lib.default_context()
    for rep in range(8):
        gp = Simple3DoFGP(use_sparse=False)
        gp.add_data(X, U, D)
        t0 = time.perf_counter(); gp.fit(); t1 = time.perf_counter()
        h = _lib.ExactGPHandle(ctx, _lib.SE_ARD, Z, D, np.ones(Z.shape[1]), 1.0, 1e-4)
        t2 = time.perf_counter()
        del h
        print(f"rep {rep}: surface fit {1e3 * (t1 - t0):.3f} ms, C-ABI fit {1e3 * (t2 - t1):.3f} ms", flush=True)


def append(k="10"):
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.gp.features import Simple3DoFFeatureExtractor
    n, k = 1000, int(k)
    ctx = _lib.Context(0)
    X, U, D = synthetic_training_data(n + k, seed=0)
    Z = Simple3DoFFeatureExtractor().extract_batch(X, U)
    ta, tf = [], []
    for _ in range(6):
        h = _lib.ExactGPHandle(ctx, _lib.SE_ARD, Z[:n], D[:n], np.ones(11), 1.0, 1e-4)
        t0 = time.perf_counter()
        assert h.append(Z[n:], D)
        ta.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        h2 = _lib.ExactGPHandle(ctx, _lib.SE_ARD, Z, D, np.ones(11), 1.0, 1e-4)
        tf.append(time.perf_counter() - t0)
        del h, h2
    print(json.dumps({"append_ms": [round(t * 1e3, 3) for t in ta], "refit_ms": [round(t * 1e3, 3) for t in tf]}))


# ---- Cholesky / SYRK / GEMM / TRSM -------------------------------------------------------
def chol():
    import bench
    print(json.dumps(bench.cholesky_bench(_lib.Context(0), _torch())), flush=True)


def potrf(shapes="1000x1,1000x14,1000x64,1000x256,2000x1,2000x8"):
    torch = _torch()
    ctx = _lib.Context(0)
    stream = torch.cuda.ExternalStream(ctx.stream)
    for n, batch in (tuple(int(v) for v in t.split("x")) for t in shapes.split(",")):
        g = torch.Generator(device="cuda").manual_seed(0)
        G = torch.randn(batch, n, n, dtype=torch.float64, device="cuda", generator=g) / n ** 0.5
        base = torch.baddbmm(torch.eye(n, dtype=torch.float64, device="cuda").expand(batch, n, n), G,
                             G.transpose(1, 2))
        del G
        A = base.clone()
        info = torch.zeros(batch, dtype=torch.int32, device="cuda")
        ts = []
        for _ in range(4):
            A.copy_(base)
            torch.cuda.synchronize()
            e0, e1 = _events(torch, stream, lambda: _lib._chk(_lib._L.gpmpc_potrf_batched_dev(
                ctx.h, n, batch, A.data_ptr(), n, n * n, info.data_ptr()), "potrf"))
            ctx.sync()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        assert int(info.abs().sum()) == 0
        pick = [0, batch - 1]
        err = float((torch.tril(A[pick]) - torch.linalg.cholesky(base[pick])).abs().max())
        t = min(ts[1:])
        fl = batch * (n ** 3 / 3 + n ** 2 / 2 + n / 6)
        print(f"n={n} batch={batch}: {t * 1e3:.3f} ms  {fl / t / 1e12:.2f} TFLOP/s  "
              f"{fl / t / FP64_PEAK * 100:.1f}% fp64 peak  maxerr {err:.2e}", flush=True)
        del A, base


def potrf_streams():
    torch = _torch()
    n = 1000
    for total, groups in [(64, 1), (64, 2), (64, 4), (256, 1), (256, 2), (256, 4), (1024, 1), (1024, 4)]:
        ctxs = [_lib.Context(0) for _ in range(groups)]
        g = torch.Generator(device="cuda").manual_seed(0)
        G = torch.randn(total, n, n, dtype=torch.float64, device="cuda", generator=g) / n ** 0.5
        base = torch.baddbmm(torch.eye(n, dtype=torch.float64, device="cuda").expand(total, n, n), G,
                             G.transpose(1, 2))
        del G
        A = base.clone()
        info = torch.zeros(total, dtype=torch.int32, device="cuda")
        per, best = total // groups, None
        for _ in range(4):
            A.copy_(base)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i, c in enumerate(ctxs):
                _lib._chk(_lib._L.gpmpc_potrf_batched_dev(c.h, n, per, A[i * per].data_ptr(), n, n * n,
                                                           info[i * per:].data_ptr()), "potrf")
            for c in ctxs:
                c.sync()
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        assert int(info.abs().sum()) == 0
        print(f"total={total} groups={groups}: {best * 1e3:.3f} ms  "
              f"{total * n ** 3 / 3 / best / FP64_PEAK * 100:.1f}% peak", flush=True)
        del A, base
        for c in ctxs:
            c.close()


def _syrk_timed(n, k, beta, seed, reps):
    torch = _torch()
    ctx = _lib.Context(0)
    stream = torch.cuda.ExternalStream(ctx.stream)
    g = torch.Generator(device="cuda").manual_seed(seed)
    A = torch.randn(n, k, dtype=torch.float64, device="cuda", generator=g) / k ** 0.5
    C = torch.eye(n, dtype=torch.float64, device="cuda") if beta else torch.zeros(n, n, dtype=torch.float64,
                                                                                   device="cuda")
    ts = []
    for it in range(reps + 3):
        e0, e1 = _events(torch, stream, lambda: _lib._chk(_lib._L.gpmpc_syrk_batched_dev(
            ctx.h, n, k, 1, A.data_ptr(), k, 0, C.data_ptr(), n, 0, 1.0, beta), "syrk"))
        ctx.sync()
        if it >= 3:
            ts.append(e0.elapsed_time(e1) * 1e-3)
    fl = n * (n + 1) * k  # lower triangle incl. diagonal, 2 flop per multiply-add
    return A, C, dict(n=n, k=k, min_ms=round(min(ts) * 1e3, 4), median_ms=round(float(np.median(ts)) * 1e3, 4),
                      frac_min=round(fl / min(ts) / FP64_PEAK, 4),
                      frac_median=round(fl / float(np.median(ts)) / FP64_PEAK, 4))


def syrk_fitc():
    print(json.dumps(_syrk_timed(2000, 4000, 1.0, 3, 30)[2]))


def gemm_loop(n="3968"):
    """n = k = 3968: 31 row tiles, 496 lower tiles, one round of 512 resident workgroups,
    248 K steps each (STORE epilogue, beta = 0: no split-K / stream-K)."""
    torch = _torch()
    A, C, r = _syrk_timed(int(n), int(n), 0.0, 5, 10)
    r["maxerr"] = float((torch.tril(C[:256, :256]) - torch.tril(A[:256] @ A[:256].T)).abs().max())
    print(json.dumps(r))


def trsm():
    ctx = _lib.default_context()
    rs = np.random.RandomState(0)
    for n, nrhs in ((128, 64), (128, 3), (1000, 3), (1000, 1000)):
        A = rs.randn(n, n)
        L = np.linalg.cholesky(A @ A.T / n + np.eye(n))
        B = rs.randn(n, nrhs)
        for _ in range(5):
            _lib.trsm_lower(ctx, L, B)
            _lib.potrs(ctx, L, B)
    print("done", flush=True)


# ---- configs[4] ----------------------------------------------------------------------------
def rollouts6(batches="64,512"):
    import bench
    bs = tuple(int(v) for v in batches.split(","))
    print(json.dumps(bench.rollouts6_bench(_lib.Context(0), _torch(), batches=bs)), flush=True)


def qp_sweep(B="64", settings="50:1e-4,100:1e-4,200:1e-4,400:1e-4,1000:1e-4,4000:1e-4"):
    """At which ADMM settings does the configs[4] controller return "solved" for >= 90% of
    its QPs?  Per (max_iter, eps): the status histogram and the to-termination timing."""
    import bench
    from gp_mpc_rocket_landing_amd.rollouts6 import Rollouts6, fit_structured_fitc, initial_conditions_6dof
    ctx = _lib.Context(0)
    gv, gw = fit_structured_fitc(ctx, n_train=4000, n_inducing=2000)
    B = int(B)
    for mi, eps in (tuple(float(x) for x in t.split(":")) for t in settings.split(",")):
        qp = dict(max_iter=int(mi), eps_abs=eps, eps_rel=eps)
        st = bench.rollouts6_qp_status(ctx, gv, gw, B, **qp)
        ro = Rollouts6(ctx, gv, gw, B, **qp)
        ro.reset(initial_conditions_6dof(B)); ro.step(1); ctx.sync()
        ro.reset(initial_conditions_6dof(B)); ctx.sync()
        t0 = time.perf_counter(); steps = 0
        while steps < 301:
            ro.step(10); steps += 10
            if np.all(ro.read()[0][:, 0] != 0):
                break
        el = time.perf_counter() - t0
        ro.close()
        print(json.dumps({"max_iter": int(mi), "eps": eps, "ms_per_step": round(el / steps * 1e3, 3),
                          "rollouts_per_s": round(B / el, 1), **st}), flush=True)


def _surface(leg, reps, prof):
    import bench
    ctx = _lib.default_context()
    fn = getattr(bench, leg)
    if prof != "prof":
        print(json.dumps(fn(ctx, reps=int(reps))), flush=True)
        return
    import cProfile
    import pstats
    fn(ctx, reps=1)  # warm
    pr = cProfile.Profile()
    pr.enable()
    print(json.dumps(fn(ctx, reps=1)), flush=True)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(40)


def surface(reps="2", prof=""):
    _surface("surface_single_landing_bench", reps, prof)


def surface6(reps="2", prof=""):
    _surface("surface_gpmpc6_bench", reps, prof)


COMMANDS = dict(single=single, step=step, stamps=stamps, placement=placement, streams=streams, fit=fit,
                append=append, chol=chol, potrf=potrf, potrf_streams=potrf_streams, syrk_fitc=syrk_fitc,
                gemm_loop=gemm_loop, trsm=trsm, rollouts6=rollouts6, qp_sweep=qp_sweep, surface=surface,
                surface6=surface6)

if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in COMMANDS:
        sys.exit(__doc__)
    COMMANDS[sys.argv[1]](*sys.argv[2:])
