"""Monte-Carlo landing protocol restatement (TEST INFRASTRUCTURE ONLY).

Reference: src/experiments/monte_carlo.py -- initial-condition sampler
(:368-399), landing check (:54-104), per-step termination rules (:455-516).
Outcome codes follow LandingOutcome (enum.auto from 1, :25-33).
"""
from __future__ import annotations

import numpy as np

SUCCESS, CRASH, FUEL_EXHAUSTED, CONSTRAINT_VIOLATION, TIMEOUT, DIVERGENCE = 1, 2, 3, 4, 5, 6

RUN_EXPERIMENTS_CFG = dict(altitude_mean=30.0, altitude_std=5.0, horizontal_std=3.0,
                           velocity_mean=(-3.0, 0.0, 0.0), velocity_std=(1.0, 0.5, 0.5),
                           mass_mean=2.0, mass_std=0.1, pos_tol_xy=5.0, pos_tol_z=1.0,
                           vel_tol_xy=1.0, vel_tol_z=3.0, min_fuel_margin=0.05)
DEFAULT_CFG = dict(altitude_mean=500.0, altitude_std=100.0, horizontal_std=50.0,
                   velocity_mean=(0.0, 0.0, -75.0), velocity_std=(20.0, 20.0, 15.0),
                   mass_mean=2.0, mass_std=0.1, pos_tol_xy=5.0, pos_tol_z=1.0,
                   vel_tol_xy=1.0, vel_tol_z=2.0, min_fuel_margin=0.05)


def sample_initial_condition(seed, cfg=RUN_EXPERIMENTS_CFG):
    """monte_carlo.py:368-399 -- draw order m, alt, r_y, r_z, v_x, v_y, v_z on the
    legacy MT19937 stream; clips m to [1.5, 2.5], alt to [10, 100], v_x <= -1."""
    rs = np.random.RandomState(seed)
    m = np.clip(cfg["mass_mean"] + rs.randn() * cfg["mass_std"], 1.5, 2.5)
    alt = np.clip(cfg["altitude_mean"] + rs.randn() * cfg["altitude_std"], 10, 100)
    ry = rs.randn() * cfg["horizontal_std"]
    rz = rs.randn() * cfg["horizontal_std"]
    vm, vs = cfg["velocity_mean"], cfg["velocity_std"]
    vx = min(vm[0] + rs.randn() * vs[0], -1)
    vy = vm[1] + rs.randn() * vs[1]
    vz = vm[2] + rs.randn() * vs[2]
    return np.array([m, alt, ry, rz, vx, vy, vz], dtype=float)


def check_landing(state, m0, cfg=RUN_EXPERIMENTS_CFG):
    """LandingConstraints.check_landing (monte_carlo.py:54-104) -> (ok, reason tag)."""
    m, alt, y, z, vv, vy, vz = state[:7]
    if abs(alt) > cfg["pos_tol_z"]:
        return False, "Altitude error"
    if abs(y) > cfg["pos_tol_xy"] or abs(z) > cfg["pos_tol_xy"]:
        return False, "Horizontal position error"
    if abs(vv) > cfg["vel_tol_z"]:
        return False, "Vertical velocity"
    if abs(vy) > cfg["vel_tol_xy"] or abs(vz) > cfg["vel_tol_xy"]:
        return False, "Horizontal velocity"
    if 1.0 - m / m0 > 1.0 - cfg["min_fuel_margin"]:
        return False, "Fuel margin"
    return True, "Success"


def pre_step_outcome(x, m0, cfg=RUN_EXPERIMENTS_CFG):
    """Termination checks at the top of each step (monte_carlo.py:458-488).
    Returns 0 (continue) or an outcome code."""
    if x[1] < 0:
        return CRASH
    if x[0] <= 1.0 + 0.01:
        return FUEL_EXHAUSTED
    if np.any(np.abs(x) > 1e6) or np.any(np.isnan(x)):
        return DIVERGENCE
    if x[1] < 1.0 and abs(x[4]) < 5.0:
        ok, _ = check_landing(x, m0, cfg)
        return SUCCESS if ok else CONSTRAINT_VIOLATION
    return 0


def incremental_target(x):
    """The per-step target of the solve-protocol (monte_carlo.py:497-500)."""
    t = x.copy()
    t[4:7] = 0.0
    t[1] = max(0.5, x[1] - 2.0)
    return t



REC_LEN = 16  # the fleet's record layout (include/gpmpc.h GPMPC_REC_LEN)


def new_landing(x0, horizon=20):
    """Controller + loop state at the start of MonteCarloSimulator.run_single
    (monte_carlo.py:418-433): the first incremental target, the RTI guess of
    osqp_rti.py:425-446 and OSQP's fresh rho / y.  Dict keys follow the fleet
    (Fleet.state()): x, Xw, Uw, y (scaled), rho, rec."""
    from . import admm_ref, qp_oracle
    x = np.array(x0, float)
    Xw, Uw = qp_oracle.initial_guess(x, incremental_target(x), horizon)
    m = qp_oracle.N_X * (horizon + 1) + qp_oracle.n_vars(horizon)
    rho0 = admm_ref.default_settings().rho
    rec = np.zeros(REC_LEN)
    rec[4:11] = x
    rec[13] = x[0]
    return dict(x=x, Xw=Xw, Uw=Uw, y=np.zeros(m), rho=rho0, rec=rec)


def landing_step(st, S, max_steps=300, dt=0.1, cfg=RUN_EXPERIMENTS_CFG, use_gp=True,
                 residual_model=True, sqp_iters=1, sqp_tol=1e-4, qp_settings=None):
    """One pass of the run_single loop body (monte_carlo.py:455-537) under the
    solve protocol (:495-512) with the 3-DoF GPMPC adapter as the controller,
    from the full state S (new_landing / Fleet.state() layout).  Returns the
    next state; rec[0] != 0 once the landing has terminated:

    * the loop's ``else`` (:539-542): TIMEOUT once max_steps steps ran;
    * the checks at the top of the step (:455-488): crash, fuel, divergence,
      landing check -> SUCCESS / CONSTRAINT_VIOLATION;
    * the incremental target (:497-500), GP mean at the horizon points of the
      shifted previous plan (exact_gp.py:213-268), the RTI QP with
      x+ = A x + B u + c (gp_mpc.py:410-411 sign), the C OSQP-0.6 restatement
      warm-started from the plan with OSQP's persistent rho / scaled y;
    * a solve without a solution -> DIVERGENCE (:506-508);
    * plant step with the pre-step drag residual, plan shifted (X[1:], X[-1]).

    ``sqp_iters`` > 1: GPMPC.solve's loop (gp_mpc.py:296-353) instead of the RTI
    step -- up to sqp_iters passes of GP mean at the current plan, QP linearised
    around it (warm start = the plan, persistent rho / y), plan <- QP solution
    (no shift); stop when max|dX| and max|dU| < sqp_tol, then the plant takes
    U[0]; not converged -> success False -> DIVERGENCE.  Every pass's ADMM
    iterations go to rec[11].

    Also returns (iterations, status) of the (last) solve, or None at termination.
    """
    if sqp_iters > 1:
        return _sqp_landing_step(st, S, max_steps, dt, cfg, use_gp, residual_model, sqp_iters, sqp_tol,
                                 qp_settings)
    from . import admm_ref, gp_oracle, qp_oracle

    x = S["x"].copy(); Xw = S["Xw"].copy(); Uw = S["Uw"].copy(); rec = S["rec"].copy()
    N = Uw.shape[0]
    m0 = rec[13]
    out = dict(x=x, Xw=Xw, Uw=Uw, y=S["y"].copy(), rho=float(S["rho"]), rec=rec)
    if rec[0] != 0:
        return out, None
    o = TIMEOUT if rec[1] >= max_steps else pre_step_outcome(x, m0, cfg)
    if o:
        rec[0] = o
        rec[2] = m0 - x[0]
        rec[4:11] = x
        return out, None
    tgt = incremental_target(x)
    mean = None
    if use_gp:
        mean, _var = gp_oracle.predict(st, gp_oracle.features_3dof(Xw[:-1], Uw))
    P0, q = qp_oracle.cost(N, np.tile(tgt, (N + 1, 1)))
    A, l, u = qp_oracle.constraints(Xw, Uw, x, dt, gp_dv=mean, sign=-1.0, filter_small=False)
    qp = admm_ref.RefQP(len(out["y"]), settings=qp_settings)
    qp.y = out["y"]; qp.rho = np.array([out["rho"]])
    try:
        r = qp.solve(P0.diagonal(), q, A, l, u, qp_oracle.to_vector(Xw, Uw))
    except RuntimeError:  # reduced KKT not positive definite: the device's factor_fail
        rec[0] = DIVERGENCE; rec[14] = -100; rec[2] = m0 - x[0]; rec[4:11] = x
        return out, (0, -100)
    if r["status"] not in (1, 2, -2):   # MPCSolution.success False -> DIVERGENCE
        rec[0] = DIVERGENCE; rec[14] = r["status"]; rec[2] = m0 - x[0]; rec[4:11] = x
        return out, (r["iter"], r["status"])
    Xo, Uo = qp_oracle.from_vector(r["x"], N)
    dr = qp_oracle.drag_residual(x) if residual_model else np.zeros(3)
    xn = qp_oracle.plant_step(x, Uo[0], dt)
    xn[4:7] += dr * dt
    out.update(x=xn, Xw=np.vstack([Xo[1:], Xo[-1:]]), Uw=np.vstack([Uo[1:], Uo[-1:]]),
               y=qp.y, rho=float(qp.rho[0]))
    rec[1] += 1
    rec[2] = m0 - xn[0]
    rec[3] = rec[1] * dt
    rec[4:11] = xn
    rec[11] += r["iter"]
    rec[12] += r["status"] == 1
    rec[14] = r["status"]
    rec[15] = qp.rho[0]
    return out, (r["iter"], r["status"])


def _sqp_landing_step(st, S, max_steps, dt, cfg, use_gp, residual_model, sqp_iters, sqp_tol,
                      qp_settings=None):
    """The sqp_iters > 1 branch of landing_step (gp_mpc.py:296-353)."""
    from . import admm_ref, gp_oracle, qp_oracle

    x = S["x"].copy(); Xw = S["Xw"].copy(); Uw = S["Uw"].copy(); rec = S["rec"].copy()
    N = Uw.shape[0]
    m0 = rec[13]
    out = dict(x=x, Xw=Xw, Uw=Uw, y=S["y"].copy(), rho=float(S["rho"]), rec=rec)
    if rec[0] != 0:
        return out, None
    Xw[0] = x          # X_pred[0] = x0 (gp_mpc.py:263): the unshifted plan starts at the state
    o = TIMEOUT if rec[1] >= max_steps else pre_step_outcome(x, m0, cfg)
    if o:
        rec[0] = o
        rec[2] = m0 - x[0]
        rec[4:11] = x
        return out, None
    tgt = incremental_target(x)
    P0, q = qp_oracle.cost(N, np.tile(tgt, (N + 1, 1)))
    qp = admm_ref.RefQP(len(out["y"]), settings=qp_settings)
    qp.y = out["y"]; qp.rho = np.array([out["rho"]])
    info = None
    for it in range(sqp_iters):
        mean = None
        if use_gp:
            mean, _var = gp_oracle.predict(st, gp_oracle.features_3dof(Xw[:-1], Uw))
        A, l, u = qp_oracle.constraints(Xw, Uw, x, dt, gp_dv=mean, sign=-1.0, filter_small=False)
        try:
            r = qp.solve(P0.diagonal(), q, A, l, u, qp_oracle.to_vector(Xw, Uw))
        except RuntimeError:
            rec[0] = DIVERGENCE; rec[14] = -100; rec[2] = m0 - x[0]; rec[4:11] = x
            out.update(Xw=Xw, Uw=Uw, y=qp.y, rho=float(qp.rho[0]))
            return out, (0, -100)
        info = (r["iter"], r["status"])
        if r["status"] not in (1, 2, -2):
            rec[0] = DIVERGENCE; rec[14] = r["status"]; rec[2] = m0 - x[0]; rec[4:11] = x
            out.update(Xw=Xw, Uw=Uw, y=qp.y, rho=float(qp.rho[0]))
            return out, info
        Xo, Uo = qp_oracle.from_vector(r["x"], N)
        conv = max(np.max(np.abs(Xo - Xw)), np.max(np.abs(Uo - Uw))) < sqp_tol
        Xw, Uw = Xo, Uo
        rec[11] += r["iter"]
        rec[12] += r["status"] == 1
        rec[14] = r["status"]
        rec[15] = qp.rho[0]
        if conv:
            dr = qp_oracle.drag_residual(x) if residual_model else np.zeros(3)
            xn = qp_oracle.plant_step(x, Uo[0], dt)
            xn[4:7] += dr * dt
            rec[1] += 1
            rec[2] = m0 - xn[0]
            rec[3] = rec[1] * dt
            rec[4:11] = xn
            out.update(x=xn, Xw=Xw, Uw=Uw, y=qp.y, rho=float(qp.rho[0]))
            return out, info
    rec[0] = DIVERGENCE              # MPCSolution.success False (monte_carlo.py:506-508)
    rec[2] = m0 - x[0]
    rec[4:11] = x
    out.update(Xw=Xw, Uw=Uw, y=qp.y, rho=float(qp.rho[0]))
    return out, info


def closed_loop_landing(st, x0, max_steps=300, horizon=20, **kw):
    """MonteCarloSimulator.run_single (monte_carlo.py:401-583), flown to
    termination by repeated landing_step.  Returns (record (16,), final state,
    per-step list of (iterations, status))."""
    S = new_landing(x0, horizon)
    trace = []
    while S["rec"][0] == 0:
        S, info = landing_step(st, S, max_steps=max_steps, **kw)
        if info is not None:
            trace.append(info)
    return S["rec"], S["x"], trace
