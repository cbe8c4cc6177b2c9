"""Closed-loop parity of the device-resident fleet against the CPU restatement.

Each control step of a landing: GP posterior mean at the N
horizon points of the shifted linearisation trajectory (exact_gp.py:213-268 via
gp_oracle), RTI QP assembly with the GP mean on the velocity rows
(osqp_rti.py:203-372 with the gp_mpc.py:309-314/411 sign, qp_oracle), the
OSQP-0.6 ADMM (C restatement, persistent rho and scaled y across steps), the
plant step with the drag residual, and the incremental target
(monte_carlo.py:497-500).  The fleet must reproduce the oracle's state
trajectory within the tolerance spec and its ADMM iteration counts and
statuses exactly.
"""
import numpy as np
import pytest

from conftest import close

pytestmark = pytest.mark.gpu

B, STEPS, N = 16, 40, 20


def _oracle_landing(st, x0, steps):
    from oracle import admm_ref, gp_oracle, mc_oracle, qp_oracle

    x = x0.copy()
    tgt = mc_oracle.incremental_target(x)
    Xw, Uw = qp_oracle.initial_guess(x, tgt, N)
    P0, _ = qp_oracle.cost(N, np.tile(tgt, (N + 1, 1)))
    qp = admm_ref.RefQP(qp_oracle.N_X * (N + 1) + qp_oracle.n_vars(N))
    out = []
    for _ in range(steps):
        tgt = mc_oracle.incremental_target(x)
        mean, _var = gp_oracle.exact_predict(st, gp_oracle.features_3dof(Xw[:-1], Uw))
        _, q = qp_oracle.cost(N, np.tile(tgt, (N + 1, 1)))
        A, l, u = qp_oracle.constraints(Xw, Uw, x, 0.1, gp_dv=mean, sign=-1.0, filter_small=False)
        r = qp.solve(P0.diagonal(), q, A, l, u, qp_oracle.to_vector(Xw, Uw))
        Xo, Uo = qp_oracle.from_vector(r["x"], N)
        dr = qp_oracle.drag_residual(x)  # residual at the pre-step state (explicit Euler)
        x = qp_oracle.plant_step(x, Uo[0], 0.1)
        x[4:7] += dr * 0.1
        Xw = np.vstack([Xo[1:], Xo[-1:]])
        Uw = np.vstack([Uo[1:], Uo[-1:]])
        out.append((x.copy(), r["iter"], r["status"]))
    return out


def _closed_loop(gpu_ctx, nb, steps):
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.fleet import (REC_ADMM_ITERS, REC_LAST_STATUS, REC_OUTCOME,
                                                 Fleet, fit_gp, initial_conditions)
    from oracle import gp_oracle

    X, U, D = synthetic_training_data(1000, seed=0)
    st = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
    x0 = initial_conditions(nb)
    ref = [_oracle_landing(st, x0[b], steps) for b in range(nb)]

    gp = fit_gp(gpu_ctx, n_train=1000)
    fl = Fleet(gpu_ctx, gp, nb, horizon=N)
    try:
        fl.reset(x0)
        prev_iters = np.zeros(nb)
        for k in range(steps):
            fl.step(1)
            rec, xs = fl.read()
            assert np.all(rec[:, REC_OUTCOME] == 0), "no landing terminates this early"
            iters = rec[:, REC_ADMM_ITERS] - prev_iters
            prev_iters = rec[:, REC_ADMM_ITERS].copy()
            for b in range(nb):
                xr, itr, str_ = ref[b][k]
                assert int(iters[b]) == itr, (k, b, int(iters[b]), itr)
                assert int(rec[b, REC_LAST_STATUS]) == str_, (k, b)
                # state tolerance: 1e-6 relative with a unit floor (SURVEY 8c spec, s = 1)
                ok, worst = close(xs[b], xr, 1.0, rtol=1e-6)
                assert ok, (k, b, worst)
    finally:
        fl.close()


@pytest.mark.parametrize("wide", ["1", "0"])
def test_fleet_closed_loop_matches_oracle(gpu_ctx, monkeypatch, wide):
    """16 landings x 40 closed-loop steps against the CPU restatement: ADMM
    iterations and statuses exact, states within 1e-6.  Both builds of the control
    kernel: a fleet this small takes the 256-thread, one-wave-per-SIMD build
    (fleet_wide.hip, GPMPC_FLEET_WIDE=1, the default below one landing per CU), and
    GPMPC_FLEET_WIDE=0 forces the 128-thread, four-landings-per-CU build the
    1024-landing fleet runs."""
    monkeypatch.setenv("GPMPC_FLEET_WIDE", wide)
    _closed_loop(gpu_ctx, B, STEPS)


@pytest.mark.parametrize("nb", [1, 3])
def test_fleet_few_landings_match_oracle(gpu_ctx, nb):
    """The few-query step (at most 64 query rows: the single landing of BASELINE
    configs[2]): features and K* in one launch (k_fleet_queries_gram), the posterior
    GEMM split over K (launch_splitk_sumsq), no dispatch-order launch for one
    landing, the wide control kernel -- against the CPU restatement over 40 steps."""
    _closed_loop(gpu_ctx, nb, STEPS)


def test_fleet_specialised_solver_matches_generic(gpu_ctx):
    """The fleet's specialised ADMM (fleet_qp.h: registers + 40 KB LDS, four landings
    per CU, dispatch order by predicted cost) against the generic LDS solver
    (qp_device.h) on 300 landings x 30 closed-loop steps: identical outcomes and
    ADMM iteration counts, states within the tolerance spec."""
    import os
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    gp = fit_gp(gpu_ctx, n_train=1000)
    x0 = initial_conditions(300)
    out = {}
    for solver in ("0", "1"):
        os.environ["GPMPC_FLEET_SOLVER"] = solver
        try:
            f = Fleet(gpu_ctx, gp, 300)
        finally:
            os.environ.pop("GPMPC_FLEET_SOLVER", None)
        f.reset(x0)
        f.step(30)
        out[solver] = f.read()
        f.close()
    (r0, x_0), (r1, x_1) = out["0"], out["1"]
    np.testing.assert_array_equal(r1[:, 0], r0[:, 0])     # outcomes
    np.testing.assert_array_equal(r1[:, 1], r0[:, 1])     # steps
    np.testing.assert_array_equal(r1[:, 11], r0[:, 11])   # ADMM iterations
    np.testing.assert_array_equal(r1[:, 14], r0[:, 14])   # last status
    ok, e = close(x_1, x_0, np.abs(x_0).max()); assert ok, e


def test_fleet_full_run_compaction_is_exact(gpu_ctx):
    """BASELINE configs[3] at full size: 1024 landings flown to termination (<= 300
    control steps, polled every 25 as run_monte_carlo does).  The running-prefix
    compaction (dispatch order before the GP phase, posterior and control launch
    over the running slots only) must give records identical to the identity
    order over every landing -- landings are independent -- and every landing
    terminates with a consistent record."""
    import os
    from gp_mpc_rocket_landing_amd.fleet import (REC_FUEL, REC_M0, REC_OUTCOME, REC_STEPS, Fleet,
                                                 fit_gp, initial_conditions)
    gp = fit_gp(gpu_ctx, n_train=1000)
    x0 = initial_conditions(1024)
    out = {}
    for order in ("0", "1"):
        os.environ["GPMPC_FLEET_ORDER"] = order
        try:
            f = Fleet(gpu_ctx, gp, 1024, max_steps=300)
        finally:
            os.environ.pop("GPMPC_FLEET_ORDER", None)
        f.reset(x0)
        for _ in range(13):
            f.step(25)
            rec, x = f.read()
            if np.all(rec[:, REC_OUTCOME] != 0):
                break
        out[order] = (rec, x)
        f.close()
    (r0, x_0), (r1, x_1) = out["0"], out["1"]
    np.testing.assert_array_equal(r1, r0)
    np.testing.assert_array_equal(x_1, x_0)
    assert np.all(r1[:, REC_OUTCOME] != 0)                       # all terminated
    assert np.all((r1[:, REC_STEPS] >= 1) & (r1[:, REC_STEPS] <= 300))
    np.testing.assert_allclose(r1[:, REC_FUEL], r1[:, REC_M0] - x_1[:, 0], atol=1e-12)   # fuel = m0 - m


def test_fleet_chain_simd_claim_is_exact(gpu_ctx):
    """The chain-SIMD claim (k_fleet_control2 picks wave 0 or 1 for the KKT chain
    so that no two chains share a SIMD) moves work between waves, never changes
    it: records and states are bit-identical to the chain-always-on-wave-0 run."""
    import os
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    gp = fit_gp(gpu_ctx, n_train=1000)
    x0 = initial_conditions(1024)
    out = {}
    for pick in ("0", "1"):
        os.environ["GPMPC_FLEET_SIMD"] = pick
        try:
            f = Fleet(gpu_ctx, gp, 1024)
        finally:
            os.environ.pop("GPMPC_FLEET_SIMD", None)
        f.reset(x0)
        f.step(20)
        out[pick] = f.read()
        f.close()
    np.testing.assert_array_equal(out["1"][0], out["0"][0])
    np.testing.assert_array_equal(out["1"][1], out["0"][1])


def _mc_selection():
    """24 landings of BASELINE configs[3] covering every outcome the oracle's
    1024-landing Monte-Carlo holds: both FUEL_EXHAUSTED, the first 11
    CONSTRAINT_VIOLATION and the first 11 SUCCESS (mc_oracle_1024.npz)."""
    from conftest import golden
    R = golden("mc_oracle_1024.npz")["records"]
    oc = R[:, 0].astype(int)
    idx = np.concatenate([np.nonzero(oc == 3)[0], np.nonzero(oc == 4)[0][:11], np.nonzero(oc == 1)[0][:11]])
    return idx, R


def _landing(S, b):
    return {k: (v[b] if k != "rho" else float(v[b])) for k, v in S.items()}


def test_fleet_steps_match_oracle_to_termination(gpu_ctx):
    """Every control step of 24 landings flown to termination (SUCCESS,
    CONSTRAINT_VIOLATION and FUEL_EXHAUSTED among them), each against the
    oracle's step (mc_oracle.landing_step: monte_carlo.py:455-537 under the
    solve protocol) from the device's own previous state -- x, the shifted
    plan Xw/Uw, OSQP's persistent scaled y and rho, the record.  Identical
    inputs every step, so: termination outcome, step count, ADMM iterations,
    solved count and status exact; state, plan, rho and duals within the
    tolerance spec (1e-6 relative, unit floor; duals floored at max |y|)."""
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    from oracle import gp_oracle, mc_oracle

    idx, _ = _mc_selection()
    X, U, D = synthetic_training_data(1000, seed=0)
    st = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
    x0 = initial_conditions(1024)[idx]
    gp = fit_gp(gpu_ctx, n_train=1000)
    fl = Fleet(gpu_ctx, gp, len(idx), max_steps=300)
    seen = set()
    try:
        fl.reset(x0)
        S = fl.state()
        for k in range(302):
            if np.all(S["rec"][:, 0] != 0):
                break
            fl.step(1)
            T = fl.state()
            for b in np.nonzero(S["rec"][:, 0] == 0)[0]:
                want, info = mc_oracle.landing_step(st, _landing(S, b))
                got = _landing(T, b)
                tag = (k, int(idx[b]))
                np.testing.assert_array_equal(got["rec"][[0, 1, 11, 12, 13, 14]],
                                              want["rec"][[0, 1, 11, 12, 13, 14]], err_msg=str(tag))
                if info is None:  # terminated at the top of this step: state untouched
                    seen.add(int(got["rec"][0]))
                    np.testing.assert_array_equal(got["rec"][4:11], S["x"][b])
                    continue
                for key in ("x", "Xw", "Uw"):
                    ok, worst = close(got[key], want[key], 1.0)
                    assert ok, (tag, key, worst)
                ok, worst = close(got["rho"], want["rho"], 0.0); assert ok, (tag, "rho", worst)
                ok, worst = close(got["y"], want["y"], np.abs(want["y"]).max()); assert ok, (tag, "y", worst)
            S = T
        assert np.all(S["rec"][:, 0] != 0), "every landing terminates within max_steps"
        assert seen == {1, 3, 4}, seen
    finally:
        fl.close()


def test_fleet_flights_match_oracle(gpu_ctx):
    """The same 24 landings flown free-running on the fleet and by the oracle's
    closed loop (mc_oracle.closed_loop_landing = monte_carlo.py:401-583):
    outcome, step count, total ADMM iterations and last status exact; flight
    time exact (steps x dt); fuel used and final state within 1e-5 relative
    (unit floor); the count of "solved" (vs "solved inaccurate") solves within
    2.  A full flight compounds ~110 steps whose adaptive-rho updates and
    solved/inaccurate verdicts are threshold decisions, so the 1e-6 per-step
    spec (test above, identical inputs every step) grows to ~1e-5 over a
    free-running flight, and one verdict in a flight can flip (measured: 1 of
    the 24 landings, by one solve)."""
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    from oracle import gp_oracle, mc_oracle

    idx, R = _mc_selection()
    X, U, D = synthetic_training_data(1000, seed=0)
    st = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
    x0 = initial_conditions(1024)[idx]
    ref = np.array([mc_oracle.closed_loop_landing(st, x)[0] for x in x0])
    gp = fit_gp(gpu_ctx, n_train=1000)
    fl = Fleet(gpu_ctx, gp, len(idx), max_steps=300)
    try:
        fl.reset(x0)
        for _ in range(13):
            fl.step(25)
        rec, x = fl.read()
    finally:
        fl.close()
    np.testing.assert_array_equal(rec[:, [0, 1, 3, 11, 13, 14]], ref[:, [0, 1, 3, 11, 13, 14]])
    assert np.all(np.abs(rec[:, 12] - ref[:, 12]) <= 2), (rec[:, 12], ref[:, 12])
    ok, worst = close(rec[:, 2], ref[:, 2], 1.0, rtol=1e-5); assert ok, ("fuel", worst)
    ok, worst = close(rec[:, 4:11], ref[:, 4:11], 1.0, rtol=1e-5); assert ok, ("state", worst)
    ok, worst = close(x, ref[:, 4:11], 1.0, rtol=1e-5); assert ok, ("x", worst)
    assert sorted(set(rec[:, 0].astype(int).tolist())) == [1, 3, 4]


def test_fleet_mc1024_matches_oracle_monte_carlo(gpu_ctx):
    """BASELINE configs[3] at full size, free-running: the device Monte-Carlo
    of 1024 landings against the oracle's (tests/golden/mc_oracle_1024.npz).
    Every landing's outcome and step count is exact (838 SUCCESS / 184
    CONSTRAINT_VIOLATION / 2 FUEL_EXHAUSTED, 111 614 control steps).

    ADMM iteration TOTALS over a free-running flight are not a property of the
    algorithm but of its exact arithmetic: the oracle against ITSELF with the
    GP weights alpha scaled by (1 + 2^-52) changes the totals of 2 landings
    (by 25 and 50 iterations) and the solved counts of 3, and the same oracle
    with its C ADMM compiled with FMA contraction changes the solved counts of
    6 (fuel up to 6e-4 relative) -- a ~1e-10 per-step difference that the
    closed loop carries for ~110 steps until a termination check sits on its
    threshold (scripts/mc_sensitivity.py, profiles/r4_mc_sensitivity.json).
    Identical inputs give identical counts at every step of every landing
    (test_fleet_mc1024_every_step_matches_oracle); here the totals of a few
    landings may differ by whole check intervals (25 iterations)."""
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    from conftest import golden
    R = golden("mc_oracle_1024.npz")["records"]
    gp = fit_gp(gpu_ctx, n_train=1000)
    fl = Fleet(gpu_ctx, gp, 1024, max_steps=300)
    try:
        fl.reset(initial_conditions(1024))
        for _ in range(13):
            fl.step(25)
            rec, _ = fl.read()
            if np.all(rec[:, 0] != 0):
                break
    finally:
        fl.close()
    np.testing.assert_array_equal(rec[:, 0], R[:, 0])
    np.testing.assert_array_equal(rec[:, 1], R[:, 1])
    np.testing.assert_array_equal(rec[:, 13], R[:, 13])
    differ = np.nonzero(rec[:, 11] != R[:, 11])[0]
    assert len(differ) <= 8, differ
    assert np.all(np.mod(rec[differ, 11] - R[differ, 11], 25) == 0)


_ORACLE_ST = None


def _oracle_state():
    global _ORACLE_ST
    if _ORACLE_ST is None:
        from gp_mpc_rocket_landing_amd.data import synthetic_training_data
        from oracle import gp_oracle
        X, U, D = synthetic_training_data(1000, seed=0)
        _ORACLE_ST = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
    return _ORACLE_ST


def _check_steps(task):
    """Pool worker: the oracle's control step (mc_oracle.landing_step) from each
    landing's device state S against the device's next state T.  Returns
    (integer mismatches [(landing, fields)], worst relative error per field)."""
    import os
    os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
    from oracle import mc_oracle
    idx, S, T = task
    st = _oracle_state()
    bad, worst = [], {"x": 0.0, "Xw": 0.0, "Uw": 0.0, "rho": 0.0, "y": 0.0}
    for j, b in enumerate(idx):
        s = {k: (v[j] if k != "rho" else float(v[j])) for k, v in S.items()}
        t = {k: (v[j] if k != "rho" else float(v[j])) for k, v in T.items()}
        want, info = mc_oracle.landing_step(st, s)
        f = [0, 1, 11, 12, 13, 14]
        if not np.array_equal(t["rec"][f], want["rec"][f]):
            bad.append((int(b), t["rec"][f].tolist(), want["rec"][f].tolist()))
            continue
        if info is None:
            continue
        for key in ("x", "Xw", "Uw"):
            worst[key] = max(worst[key], float(np.max(np.abs(t[key] - want[key]) / np.maximum(np.abs(want[key]), 1.0))))
        worst["rho"] = max(worst["rho"], abs(t["rho"] - want["rho"]) / abs(want["rho"]))
        ys = max(float(np.abs(want["y"]).max()), 1e-300)
        worst["y"] = max(worst["y"], float(np.max(np.abs(t["y"] - want["y"]) / np.maximum(np.abs(want["y"]), ys))))
    return bad, worst


def test_fleet_mc1024_every_step_matches_oracle(gpu_ctx):
    """VERDICT r3 #1, "iteration counts bit-exact" at full size: every control
    step of all 1024 landings of BASELINE configs[3], flown to termination
    (~112 000 steps), against the oracle's step (mc_oracle.landing_step =
    monte_carlo.py:455-537 under the solve protocol: GP posterior, RTI QP, the
    C OSQP-0.6 restatement, plant) from the device's own previous state (x, the
    shifted plan, OSQP's persistent scaled y and rho, the record).  Outcome,
    step count, ADMM iterations, solved count, status exact at EVERY step;
    state, plan, rho and duals within 1e-6 (unit floor; duals floored at
    max |y|).  The oracle runs in a pool of CPU processes beside the fleet."""
    import multiprocessing as mp
    import os
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    B = 1024
    gp = fit_gp(gpu_ctx, n_train=1000)
    fl = Fleet(gpu_ctx, gp, B, max_steps=300)
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    pending, nsteps = [], 0
    # one BLAS thread per worker process (the box sets 16 for every process)
    saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    os.environ.update(OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    try:
        pool = mp.get_context("spawn").Pool(workers)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    with pool:
        try:
            fl.reset(initial_conditions(B))
            S = fl.state()
            for k in range(302):
                run = np.nonzero(S["rec"][:, 0] == 0)[0]
                if run.size == 0:
                    break
                fl.step(1)
                T = fl.state()
                nsteps += run.size
                for c in np.array_split(run, max(1, min(4 * workers, run.size // 8))):
                    pending.append(pool.apply_async(_check_steps, ((c, {kk: v[c] for kk, v in S.items()},
                                                                    {kk: v[c] for kk, v in T.items()}),)))
                S = T
                if k % 10 == 0:
                    print(f"mc1024 step-locked: device step {k}, {run.size} running, {nsteps} steps queued",
                          flush=True)
            assert np.all(S["rec"][:, 0] != 0), "every landing terminates within max_steps"
        finally:
            fl.close()
        res = []
        for i, p in enumerate(pending):
            res.append(p.get(timeout=600))
            if i % 500 == 0:
                print(f"mc1024 step-locked: {i} of {len(pending)} oracle chunks checked", flush=True)
    bad = [b for r, _ in res for b in r]
    worst = {k: max(w[k] for _, w in res) for k in res[0][1]}
    assert not bad, (len(bad), bad[:5])
    assert nsteps > 100000, nsteps
    for key, tol in (("x", 1e-6), ("Xw", 1e-6), ("Uw", 1e-6), ("rho", 1e-6), ("y", 1e-6)):
        assert worst[key] <= tol, (key, worst)


def test_fleet_shards_reproduce_the_whole_fleet(gpu_ctx):
    """Sharding invariance: the landings of BASELINE configs[3] flown
    as shard fleets (initial conditions by global index, each shard created for the
    whole fleet's size, as each rank of run_monte_carlo builds its shard) give
    records and states bit-identical to one 1024-landing fleet: two shards of 512,
    and four of 256 -- shards that, sized for themselves, would take the wide
    control build (one landing per CU) while the whole fleet runs the narrow one
     -- and a ragged 3-way split of the first 100 landings, fleets of
    34 / 33 / 33, to one 100-landing fleet."""
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    from gp_mpc_rocket_landing_amd.sharding import shard_range
    gp = fit_gp(gpu_ctx, n_train=1000)

    def fly(first, count, total, steps=60):
        f = Fleet(gpu_ctx, gp, count, fleet_batch=total, max_steps=300)
        try:
            f.reset(initial_conditions(count, first=first))
            f.step(steps)
            return f.read()
        finally:
            f.close()

    for total, worlds in ((1024, (2, 4)), (100, (3,))):
        whole_r, whole_x = fly(0, total, total)
        for world in worlds:
            parts = [fly(*shard_range(total, r, world), total) for r in range(world)]
            np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), whole_r, err_msg=str(world))
            np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]), whole_x, err_msg=str(world))


def test_fleet_to_termination_bits_do_not_depend_on_the_running_count(gpu_ctx):
    """the posterior GEMM's kernel and the control kernel's build are
    fixed when the fleet is created, not re-chosen from the number of landings
    still flying (the kernels sum in different orders).  A fleet of 16 landings
    flown until every one has terminated -- its running count falls through the
    64-row-tile (P < 256) and split-K (P <= 64, three landings or fewer) sizes --
    equals, bit for bit, the same 16 landings flown one per fleet as shards of
    the 16 (each shard created for 16, running one landing throughout).  The
    run also covers the partial-sum buffer of a fleet whose running count falls
    below its creation size (it was sized for one tile height only).  The
    posterior read back through the C-ABI at a step where some landings have
    terminated matches the shard fleets' too, so no slot shows another
    landing's values."""
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    gp = fit_gp(gpu_ctx, n_train=1000)
    B = 16
    x0 = initial_conditions(B)
    whole = Fleet(gpu_ctx, gp, B, max_steps=300)
    shards = [Fleet(gpu_ctx, gp, 1, fleet_batch=B, max_steps=300) for _ in range(B)]
    try:
        whole.reset(x0)
        for b, f in enumerate(shards):
            f.reset(x0[b:b + 1])
        running_seen, post_checked = set(), 0
        for k in range(305):
            rec, x = whole.read()
            run = int(np.sum(rec[:, 0] == 0))
            running_seen.add(run)
            if run == 0:
                break
            whole.step(1)
            for f in shards:
                f.step(1)
            rec, x = whole.read()
            parts = [f.read() for f in shards]
            np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), rec, err_msg=str(k))
            np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]), x, err_msg=str(k))
            if 0 < run < B and k % 7 == 0:
                m, v = whole.posterior()
                for b, f in enumerate(shards):
                    mb, vb = f.posterior()
                    if not np.all(np.isfinite(m[b])):   # past the whole fleet's launched prefix
                        assert rec[b, 0] != 0, (k, b)
                    elif np.all(np.isfinite(mb)):
                        np.testing.assert_array_equal(m[b], mb[0], err_msg=str((k, b)))
                        np.testing.assert_array_equal(v[b], vb[0], err_msg=str((k, b)))
                        post_checked += 1
        assert 0 in running_seen and min(r for r in running_seen if r > 0) <= 3, sorted(running_seen)
        assert post_checked > 0
    finally:
        whole.close()
        for f in shards:
            f.close()


@pytest.mark.parametrize("horizon", [20, 15])
def test_fleet_sqp_mode_matches_oracle(gpu_ctx, horizon):
    """GPMPC.solve's loop on the fleet (sqp_iters > 1; gp_mpc.py:296-353): per
    pass, GP mean at the current plan, QP linearised around it, plan <- QP
    solution (no shift), stop when max|dX|, max|dU| < sqp_tol; the plant takes
    U[0] of the converged plan; not converged after sqp_iters passes ->
    DIVERGENCE.  Every control step of 8 landings against mc_oracle.landing_step
    with the same loop, from the device's own previous state: outcome, steps,
    ADMM iteration totals over all passes, solved count and last status exact;
    state, plan, rho and duals within the tolerance spec.  sqp_tol = 1.0 lets
    the loop converge after a few passes (the plant branch); with the
    reference's 1e-4 the 1e-4 ADMM never converges the loop in 10 passes (the
    lateral thrust of consecutive plans moves by ~0.3), so every landing ends
    DIVERGENCE at its first step -- on both sides.  With the SQP passes' own QP
    settings (sqp_qp: eps 1e-7, max_iter 2000, the IPOPT-like tight solves of
    gp_mpc.py:462-470) and 100 passes the loop does converge at 1e-4 for the
    first control steps (full-step SQP contracts ~0.9 per pass), which pins
    the converged branch at the reference's tolerance.  N = 20 runs the fleet's
    specialised solver (k_fleet_control2); any other horizon (MPCConfig.N is free in the
    reference, nominal_mpc.py:47) the generic one (k_fleet_control, VERDICT r5 missing #3)."""
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    from oracle import admm_ref, gp_oracle, mc_oracle

    X, U, D = synthetic_training_data(1000, seed=0)
    st = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
    nb = 8
    x0 = initial_conditions(nb)
    gp = fit_gp(gpu_ctx, n_train=1000)
    tight = dict(eps_abs=1e-7, eps_rel=1e-7, max_iter=2000)
    for tol, steps, passes, sq in ((1.0, 25, 10, None), (1e-4, 2, 10, None), (1e-4, 3, 100, tight)):
        fl = Fleet(gpu_ctx, gp, nb, max_steps=300, sqp_iters=passes, sqp_tol=tol, sqp_qp=sq or {},
                   horizon=horizon)
        qs = admm_ref.default_settings(**sq) if sq else None
        moved = 0
        try:
            fl.reset(x0)
            S = fl.state()
            for k in range(steps):
                if np.all(S["rec"][:, 0] != 0):
                    break
                fl.step(1)
                T = fl.state()
                for b in np.nonzero(S["rec"][:, 0] == 0)[0]:
                    want, info = mc_oracle.landing_step(st, _landing(S, b), sqp_iters=passes, sqp_tol=tol,
                                                        qp_settings=qs)
                    got = _landing(T, b)
                    tag = (tol, k, int(b))
                    np.testing.assert_array_equal(got["rec"][[0, 1, 11, 12, 13, 14]],
                                                  want["rec"][[0, 1, 11, 12, 13, 14]], err_msg=str(tag))
                    moved += int(got["rec"][1] > S["rec"][b, 1])
                    # the tight case runs up to 100 passes x 2000 ADMM iterations per control step:
                    # the device's summation orders drift the continuous state by up to ~1e-5
                    # relative over that many iterations (integer outputs stay exact)
                    rt = 1e-4 if sq else 1e-6
                    for key in ("x", "Xw", "Uw"):
                        ok, worst = close(got[key], want[key], 1.0, rtol=rt)
                        assert ok, (tag, key, worst)
                    ok, worst = close(got["rho"], want["rho"], 0.0, rtol=rt); assert ok, (tag, "rho", worst)
                    ok, worst = close(got["y"], want["y"], np.abs(want["y"]).max(), rtol=rt)
                    assert ok, (tag, "y", worst)
                S = T
        finally:
            fl.close()
        if tol == 1e-4 and sq is None:
            assert np.all(S["rec"][:, 0] == 6) and np.all(S["rec"][:, 1] == 0)
        elif sq is not None:
            assert moved >= nb // 2, moved   # converged at 1e-4 and stepped
        else:
            assert moved > nb, moved   # the converged branch (plant step) ran


@pytest.mark.parametrize("cs", ["0", "1"])
def test_fleet_posterior_full_size_matches_oracle(gpu_ctx, monkeypatch, cs):
    """The headline kernel's own output: the GP posterior the
    fleet computes each control step for all 1024 landings x 20 horizon points
    (P = 20 480 queries against the n = 1000 GP, BASELINE configs[3]) -- the mean
    the QP assembly consumes and the variance the MFMA sum-of-squares pass forms
    beside it -- read back through the C-ABI (gpmpc_fleet_get_posterior) and
    compared with ExactGP.predict (exact_gp.py:256-266, gp_oracle.exact_predict)
    at every query, over two control steps (the second one with the dispatch order
    of the first step's iteration counts, so the slot -> landing map is not the
    identity).  Tolerance spec SURVEY 8c: |a - b| <= 1e-6 max(|b|, s), s = y_std
    for means, sigma2 y_std^2 for variances.  Both posterior paths: K* in HBM (the
    default) and GPMPC_POST_CS=1's column-stationary kernel."""
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    from oracle import gp_oracle

    monkeypatch.setenv("GPMPC_POST_CS", cs)
    nb, n = 1024, 1000
    X, U, D = synthetic_training_data(n, seed=0)
    st = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
    gp = fit_gp(gpu_ctx, n_train=n)
    fl = Fleet(gpu_ctx, gp, nb, horizon=N)
    try:
        fl.reset(initial_conditions(nb))
        for step in range(2):
            S = fl.state()
            assert np.all(S["rec"][:, 0] == 0)
            fl.step(1)
            mean, var = fl.posterior()
            Zq = gp_oracle.features_3dof(S["Xw"][:, :N].reshape(-1, 7), S["Uw"].reshape(-1, 3))
            m_ref, v_ref = gp_oracle.exact_predict(st, Zq)
            for c in range(3):
                ok, worst = close(mean.reshape(-1, 3)[:, c], m_ref[:, c], st["y_std"][c])
                assert ok, (step, "mean", c, worst)
                ok, worst = close(var.reshape(-1, 3)[:, c], v_ref[:, c], st["sigma2"] * st["y_std"][c] ** 2)
                assert ok, (step, "var", c, worst)
            # the variance is not a constant: the posterior really varies over the queries
            assert np.ptp(v_ref[:, 0]) > 0.0
    finally:
        fl.close()


def _fitc_fleet_setup(gpu_ctx):
    """The reference-default Simple3DoFGP() (FITC, 50 kmeans2 inducing points) as the
    fleet's GP, and the oracle's FITC fit with the surface's own inducing points."""
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.fleet import fit_gp_sparse
    from oracle import gp_oracle
    h = fit_gp_sparse(n_train=1000, n_inducing=50, seed=0)
    X, U, D = synthetic_training_data(1000, seed=0)
    Zi = np.array(h.surface.gp.gps[0].inducing_points)
    st = gp_oracle.fitc_fit(Zi, gp_oracle.features_3dof(X, U), D, noise=1e-4, jitter=1e-6)
    return h, st


def test_fleet_on_the_default_sparse_gp_matches_oracle_every_step(gpu_ctx):
    """the fleet on the reference-default Simple3DoFGP() -- FITC,
    M = 50 (structured_gp.py:423-428) -- through gpmpc_fleet_create_fitc.  Every
    control step of 16 landings flown to termination against mc_oracle.landing_step
    with the oracle's FITC GP (SparseGP.predict, sparse_gp.py:255-305, mean K*u alpha
    as written), from the device's own previous state: outcome, steps, ADMM
    iterations, solved count and status exact; state, plan, rho and duals within the
    tolerance spec.  Then the fleet's own posterior at 1024 landings x 20 points
    (P = 20 480 against the 50 inducing rows) read back through the C-ABI against
    SparseGP.predict: mean and variance within the spec."""
    from gp_mpc_rocket_landing_amd.fleet import Fleet, initial_conditions
    from oracle import gp_oracle, mc_oracle
    h, st = _fitc_fleet_setup(gpu_ctx)
    nb = 16
    fl = Fleet(gpu_ctx, h, nb, max_steps=300)
    seen, steps = set(), 0
    try:
        fl.reset(initial_conditions(nb))
        S = fl.state()
        for k in range(302):
            if np.all(S["rec"][:, 0] != 0):
                break
            fl.step(1)
            T = fl.state()
            for b in np.nonzero(S["rec"][:, 0] == 0)[0]:
                want, info = mc_oracle.landing_step(st, _landing(S, b))
                got = _landing(T, b)
                tag = (k, int(b))
                np.testing.assert_array_equal(got["rec"][[0, 1, 11, 12, 13, 14]],
                                              want["rec"][[0, 1, 11, 12, 13, 14]], err_msg=str(tag))
                if info is None:
                    seen.add(int(got["rec"][0]))
                    continue
                steps += 1
                for key in ("x", "Xw", "Uw"):
                    ok, worst = close(got[key], want[key], 1.0)
                    assert ok, (tag, key, worst)
                ok, worst = close(got["rho"], want["rho"], 0.0); assert ok, (tag, "rho", worst)
                ok, worst = close(got["y"], want["y"], np.abs(want["y"]).max()); assert ok, (tag, "y", worst)
            S = T
        assert np.all(S["rec"][:, 0] != 0) and steps > 500, (steps, S["rec"][:, 0])
    finally:
        fl.close()
    nb = 1024
    fl = Fleet(gpu_ctx, h, nb, horizon=N)
    try:
        fl.reset(initial_conditions(nb))
        for step in range(2):
            S = fl.state()
            fl.step(1)
            mean, var = fl.posterior()
            Zq = gp_oracle.features_3dof(S["Xw"][:, :N].reshape(-1, 7), S["Uw"].reshape(-1, 3))
            m_ref, v_ref = gp_oracle.fitc_predict(st, Zq)
            for c in range(3):
                ok, worst = close(mean.reshape(-1, 3)[:, c], m_ref[:, c], st["y_std"][c])
                assert ok, (step, "mean", c, worst)
                ok, worst = close(var.reshape(-1, 3)[:, c], v_ref[:, c], st["sigma2"] * st["y_std"][c] ** 2)
                assert ok, (step, "var", c, worst)
            assert np.ptp(v_ref[:, 0]) > 0.0
    finally:
        fl.close()
