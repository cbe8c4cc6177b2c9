"""Constraint parameters and chance-constraint tightening (reference
src/mpc/constraints.py:35-71 ``ConstraintParams``, :427-509
``TightenedConstraints``).

Host-side configuration, same fields, defaults and arithmetic as the
reference.  As there, the tightened parameters are v_max, theta_max and
omega_max (with floors); thrust bounds and the glideslope are passed through
unchanged, so GPMPC's QP -- which uses only T_min, T_max and gamma_gs
(gp_mpc.py:414-428) -- is not changed by the tightening.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class ConstraintParams:
    """constraints.py:35-71."""
    T_min: float = 0.5
    T_max: float = 5.0
    delta_max: float = 20.0
    theta_max: float = 90.0
    gamma_gs: float = 30.0
    omega_max: float = 60.0
    v_max: float = 50.0
    r_tol: float = 0.1
    v_tol: float = 0.1
    q_tol: float = 5.0
    omega_tol: float = 1.0

    def __post_init__(self):
        self.delta_max_rad = np.deg2rad(self.delta_max)
        self.theta_max_rad = np.deg2rad(self.theta_max)
        self.gamma_gs_rad = np.deg2rad(self.gamma_gs)
        self.omega_max_rad = np.deg2rad(self.omega_max)
        self.q_tol_rad = np.deg2rad(self.q_tol)
        self.omega_tol_rad = np.deg2rad(self.omega_tol)


@dataclass
class TightenedConstraints:
    """constraints.py:427-509: g(mu) - kappa sigma_g >= 0, kappa = Phi^-1(confidence)."""
    base_params: ConstraintParams
    confidence_level: float = 0.99

    def __post_init__(self):
        from scipy.stats import norm
        self.kappa = norm.ppf(self.confidence_level)

    def tighten_scalar_constraint(self, constraint_value: float, constraint_std: float) -> float:
        return constraint_value - self.kappa * constraint_std

    def get_tightened_params(self, position_std: float = 0.0, velocity_std: float = 0.0,
                             attitude_std: float = 0.0, omega_std: float = 0.0) -> ConstraintParams:
        b = self.base_params
        p = ConstraintParams(T_min=b.T_min, T_max=b.T_max, delta_max=b.delta_max,
                             theta_max=b.theta_max - np.rad2deg(self.kappa * attitude_std),
                             gamma_gs=b.gamma_gs,
                             omega_max=b.omega_max - np.rad2deg(self.kappa * omega_std),
                             v_max=b.v_max - self.kappa * velocity_std,
                             r_tol=b.r_tol, v_tol=b.v_tol, q_tol=b.q_tol, omega_tol=b.omega_tol)
        # floors (constraints.py:503-507); the *_rad fields keep the pre-floor value, as there
        p.theta_max = max(p.theta_max, 10.0)
        p.omega_max = max(p.omega_max, 10.0)
        p.v_max = max(p.v_max, 1.0)
        return p
