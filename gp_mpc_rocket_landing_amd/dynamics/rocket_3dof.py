"""3-DoF point-mass rocket (reference src/dynamics/rocket_3dof.py).

The reference delegates integration to the undeclared ``simdyn`` package; the
model is restated from the 3-DoF Euler equations of nominal_mpc.py:585-605
(m+ = m - dt alpha |u|, r+ = r + dt v, v+ = v + dt (u/m + g)) with the
normalised defaults of Rocket3DoFConfig (rocket_3dof.py:34-66): I_sp = 30,
g0 = 1, alpha = 1/(I_sp g0), g_I = [-1, 0, 0].  State x = [m, r(3), v(3)],
control u = thrust (3) in the inertial frame.  Host-side plumbing (one state
per call); the batched closed loop runs the same model on the GPU (fleet).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np


@dataclass
class Rocket3DoFConfig:
    """rocket_3dof.py:34-66 (drag options are not part of the restated plant)."""
    m_dry: float = 1.0
    m_wet: float = 2.0
    I_sp: float = 30.0
    g0: float = 1.0
    T_min: float = 0.0
    T_max: float = 6.5
    g_I: Optional[np.ndarray] = None
    gamma_gs: float = float(np.deg2rad(30.0))
    v_max: float = float(np.inf)
    default_dt: float = 0.1

    def __post_init__(self):
        if self.g_I is None:
            self.g_I = np.array([-1.0, 0.0, 0.0])


@dataclass
class Rocket3DoFParams:
    """The ``dynamics.params`` fields the controllers read (g, g0, g_vec, alpha)."""
    m_dry: float
    m_wet: float
    g0: float
    alpha: float
    g_vec: np.ndarray = field(default_factory=lambda: np.array([-1.0, 0.0, 0.0]))
    T_min: float = 0.0
    T_max: float = 6.5

    @property
    def g(self) -> float:
        return float(np.linalg.norm(self.g_vec))


class Rocket3DoFDynamics:
    N_STATE = 7
    N_CONTROL = 3

    def __init__(self, config: Optional[Rocket3DoFConfig] = None):
        self.config = config or Rocket3DoFConfig()
        c = self.config
        self._params = Rocket3DoFParams(m_dry=c.m_dry, m_wet=c.m_wet, g0=c.g0,
                                        alpha=1.0 / (c.I_sp * c.g0), g_vec=np.asarray(c.g_I, float),
                                        T_min=c.T_min, T_max=c.T_max)

    @property
    def params(self) -> Rocket3DoFParams:
        return self._params

    @property
    def n_state(self) -> int:
        return self.N_STATE

    @property
    def n_control(self) -> int:
        return self.N_CONTROL

    def dynamics(self, x, u) -> np.ndarray:
        """Continuous-time f(x, u)."""
        x = np.asarray(x, float); u = np.asarray(u, float)
        out = np.empty(7)
        out[0] = -self._params.alpha * np.sqrt(u @ u)
        out[1:4] = x[4:7]
        out[4:7] = u / x[0] + self._params.g_vec
        return out

    f = dynamics

    def step(self, x, u, dt: Optional[float] = None) -> np.ndarray:
        """One explicit-Euler step x+ = x + dt f(x, u)."""
        dt = self.config.default_dt if dt is None else dt
        x = np.asarray(x, float)
        return x + dt * self.dynamics(x, u)

    f_discrete = step

    def jacobian_x(self, x, u) -> np.ndarray:
        x = np.asarray(x, float); u = np.asarray(u, float)
        A = np.zeros((7, 7))
        A[1:4, 4:7] = np.eye(3)
        A[4:7, 0] = -u / x[0] ** 2
        return A

    def jacobian_u(self, x, u) -> np.ndarray:
        x = np.asarray(x, float); u = np.asarray(u, float)
        B = np.zeros((7, 3))
        B[0, :] = -self._params.alpha * u / (np.sqrt(u @ u) + 1e-10)
        B[4:7, :] = np.eye(3) / x[0]
        return B

    def linearize(self, x, u, dt: Optional[float] = None) -> Tuple[np.ndarray, np.ndarray]:
        """rocket_3dof.py:341-367: continuous Jacobians, or I + A dt, B dt."""
        A, B = self.jacobian_x(x, u), self.jacobian_u(x, u)
        if dt is not None:
            return np.eye(7) + A * dt, B * dt
        return A, B

    def hover_thrust(self, x) -> np.ndarray:
        return -np.asarray(x, float)[0] * self._params.g_vec

    def get_altitude(self, x) -> float:
        return float(np.asarray(x)[1])

    def __repr__(self) -> str:
        return f"Rocket3DoFDynamics(alpha={self._params.alpha:.4g}, g={self._params.g_vec.tolist()})"


def create_normalized_rocket() -> Rocket3DoFDynamics:
    return Rocket3DoFDynamics(Rocket3DoFConfig())
