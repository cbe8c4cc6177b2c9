"""MPC cost weights (reference src/mpc/cost_functions.py:39-105, ``CostWeights``).

Host-side configuration with the reference's fields, defaults and matrix
construction (14-state Q / R / P as used by the reference GPMPC).  The 3-DoF
RTI QP of this path uses its own fixed diag weights (osqp_rti.py:171-182,
mpc/qp_builder.py); ``CostWeights.q_3dof`` gives the 7-state view of Q.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np


@dataclass
class CostWeights:
    """cost_functions.py:39-105: stage l = (x - x_ref)' Q (x - x_ref) + u' R u, terminal P."""
    Q: Optional[np.ndarray] = None
    R: Optional[np.ndarray] = None
    P: Optional[np.ndarray] = None
    w_position: float = 10.0
    w_velocity: float = 1.0
    w_attitude: float = 5.0
    w_omega: float = 0.1
    w_mass: float = 0.0
    w_thrust: float = 0.01
    w_fuel: float = 0.1
    terminal_weight: float = 10.0

    def __post_init__(self):
        if self.Q is None:
            self.Q = self._build_Q_matrix()
        if self.R is None:
            self.R = self._build_R_matrix()
        if self.P is None:
            self.P = self.terminal_weight * self.Q

    def _build_Q_matrix(self) -> np.ndarray:
        Q = np.zeros((14, 14))
        Q[0, 0] = self.w_mass
        Q[1:4, 1:4] = self.w_position * np.eye(3)
        Q[4:7, 4:7] = self.w_velocity * np.eye(3)
        Q[8, 8] = self.w_attitude   # qx
        Q[9, 9] = self.w_attitude   # qy
        Q[11:14, 11:14] = self.w_omega * np.eye(3)
        return Q

    def _build_R_matrix(self) -> np.ndarray:
        return self.w_thrust * np.eye(3)

    @property
    def q_3dof(self) -> np.ndarray:
        """The [m, r, v] block of Q (7 x 7)."""
        return np.asarray(self.Q)[:7, :7].copy()
