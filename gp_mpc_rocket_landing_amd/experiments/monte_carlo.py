"""Monte-Carlo landing protocol, batched and sharded (reference
src/experiments/monte_carlo.py).

The reference runs landings one after another in Python (``n_workers`` is
ignored, monte_carlo.py:617-631).  Here a whole shard of landings advances
together on one GPU (``gp_mpc_rocket_landing_amd.fleet``), shards are
contiguous blocks of landings per rank, and the fixed-size per-landing records
are gathered to rank 0 with one collective (RCCL over xGMI on MI355X).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum

import numpy as np


class LandingOutcome(Enum):
    """monte_carlo.py:25-33 (enum.auto starts at 1)."""
    SUCCESS = 1
    CRASH = 2
    FUEL_EXHAUSTED = 3
    CONSTRAINT_VIOLATION = 4
    TIMEOUT = 5
    DIVERGENCE = 6


@dataclass
class LandingConstraints:
    """monte_carlo.py:36-52."""
    pos_tol_xy: float = 5.0
    pos_tol_z: float = 1.0
    vel_tol_xy: float = 1.0
    vel_tol_z: float = 2.0
    tilt_max: float = 0.1
    min_fuel_margin: float = 0.05

    def check_landing(self, state, initial_mass):
        """monte_carlo.py:54-104: (success, reason) for a final state (x = altitude axis)."""
        m, alt, y, z, vv, vy, vz = [float(v) for v in np.asarray(state)[:7]]
        if abs(alt) > self.pos_tol_z:
            return False, f"Altitude error: {alt:.2f} m"
        if abs(y) > self.pos_tol_xy or abs(z) > self.pos_tol_xy:
            return False, f"Horizontal position error: ({y:.2f}, {z:.2f}) m"
        if abs(vv) > self.vel_tol_z:
            return False, f"Vertical velocity: {vv:.2f} m/s"
        if abs(vy) > self.vel_tol_xy or abs(vz) > self.vel_tol_xy:
            return False, f"Horizontal velocity: ({vy:.2f}, {vz:.2f}) m/s"
        used = 1.0 - m / initial_mass
        if used > (1.0 - self.min_fuel_margin):
            return False, f"Fuel margin: {(1 - used) * 100:.1f}%"
        return True, "Success"


@dataclass
class SimulationConfig:
    """monte_carlo.py:107-130."""
    dt: float = 0.1
    max_time: float = 100.0
    altitude_mean: float = 500.0
    altitude_std: float = 100.0
    horizontal_std: float = 50.0
    velocity_mean: np.ndarray = field(default_factory=lambda: np.array([0, 0, -75]))
    velocity_std: np.ndarray = field(default_factory=lambda: np.array([20, 20, 15]))
    mass_mean: float = 2.0
    mass_std: float = 0.1
    wind_enabled: bool = False
    aero_dispersion: float = 0.0
    thrust_dispersion: float = 0.0
    landing_constraints: LandingConstraints = field(default_factory=LandingConstraints)

    @classmethod
    def run_experiments(cls):
        """The SimulationConfig of scripts/run_experiments.py:359-371 (BASELINE C3/C4)."""
        return cls(dt=0.1, max_time=30.0, altitude_mean=30.0, altitude_std=5.0,
                   horizontal_std=3.0, velocity_mean=np.array([-3, 0, 0]),
                   velocity_std=np.array([1, 0.5, 0.5]),
                   landing_constraints=LandingConstraints(pos_tol_xy=5.0, vel_tol_z=3.0))


def sample_initial_condition(seed, cfg: SimulationConfig):
    """MonteCarloSimulator.sample_initial_condition (monte_carlo.py:368-399): seven
    legacy-MT19937 normal draws in the order m, altitude, r_y, r_z, v_x, v_y, v_z;
    m clipped to [1.5, 2.5], altitude to [10, 100], v_x <= -1."""
    rs = np.random.RandomState(seed)
    m = np.clip(cfg.mass_mean + rs.randn() * cfg.mass_std, 1.5, 2.5)
    alt = np.clip(cfg.altitude_mean + rs.randn() * cfg.altitude_std, 10, 100)
    ry = rs.randn() * cfg.horizontal_std
    rz = rs.randn() * cfg.horizontal_std
    vx = min(cfg.velocity_mean[0] + rs.randn() * cfg.velocity_std[0], -1)
    vy = cfg.velocity_mean[1] + rs.randn() * cfg.velocity_std[1]
    vz = cfg.velocity_mean[2] + rs.randn() * cfg.velocity_std[2]
    return np.array([m, alt, ry, rz, vx, vy, vz], dtype=float)
