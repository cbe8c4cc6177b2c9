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
