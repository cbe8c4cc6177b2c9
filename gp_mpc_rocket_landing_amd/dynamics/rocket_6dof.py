"""6-DoF rocket (reference src/dynamics/rocket_6dof.py), host mirror.

The reference wraps ``simdyn.Rocket6DoF``, which is absent (undeclared, not
installed).  The model is restated from the 14-state equations the reference
spells out in nominal_mpc.py:163-203 (the CasADi 6-DoF model of the same
rocket), with the Rocket6DoFConfig defaults of rocket_6dof.py:36-89:

  state x = [m, r_I (3), v_I (3), q_BI = (w, x, y, z), omega_B (3)], control u =
  thrust in the body frame; m' = -alpha |u| (alpha = 1 / (I_sp g0));
  r' = v; v' = C_IB u / m + g_I; q' = 1/2 Omega(omega) q;
  omega' = J^-1 (r_T x u - omega x J omega).

``step`` is RK4 (discretization.py:229-252) + quaternion normalisation
(rocket_6dof.py:351-387); ``linearize(x, u, dt)`` returns I + A_c dt, B_c dt
(rocket_6dof.py:427-459) with the analytic Jacobians.  These are exactly the
formulas csrc/fleet6.hip evaluates on the device (the GPMPC 14-state path), and
oracle/sixdof_oracle.py restates them for the tests.  Host-side plumbing: one
state per call, the caller's plant -- the hot path never calls it.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np


@dataclass
class Rocket6DoFConfig:
    """rocket_6dof.py:36-89 (same fields and defaults)."""
    m_dry: float = 1.0
    m_wet: float = 2.0
    J_B: Optional[np.ndarray] = None
    I_sp: float = 30.0
    g0: float = 1.0
    T_min: float = 1.5
    T_max: float = 6.5
    r_T_B: Optional[np.ndarray] = None
    r_cp_B: Optional[np.ndarray] = None
    g_I: Optional[np.ndarray] = None
    delta_max: float = float(np.deg2rad(20.0))
    theta_max: float = float(np.deg2rad(90.0))
    gamma_gs: float = float(np.deg2rad(30.0))
    omega_max: float = float(np.deg2rad(60.0))
    enable_aero: bool = False
    C_A: Optional[np.ndarray] = None
    rho: float = 0.0
    S_ref: float = 1.0
    default_dt: float = 0.1
    use_rk4: bool = True

    def __post_init__(self):
        if self.J_B is None:
            self.J_B = np.diag([0.02, 1.0, 1.0]) * 0.168
        if self.r_T_B is None:
            self.r_T_B = np.array([-0.25, 0.0, 0.0])
        if self.r_cp_B is None:
            self.r_cp_B = np.array([0.05, 0.0, 0.0])
        if self.g_I is None:
            self.g_I = np.array([-1.0, 0.0, 0.0])

    @classmethod
    def szmuk_defaults(cls) -> "Rocket6DoFConfig":
        return cls()


@dataclass
class Rocket6DoFParams:
    """The ``dynamics.params`` fields (simdyn.Rocket6DoFParams as built at
    rocket_6dof.py:140-162); GPMPC reads ``g0`` (gp_mpc.py:275)."""
    m_dry: float
    m_wet: float
    J_B: np.ndarray
    I_sp: float
    g0: float
    g_I: np.ndarray
    r_T_B: np.ndarray
    r_cp_B: np.ndarray
    T_min: float
    T_max: float
    delta_max: float
    theta_max: float
    gamma_gs: float
    omega_max: float
    enable_aero: bool = False
    alpha: float = field(init=False)

    def __post_init__(self):
        self.alpha = 1.0 / (self.I_sp * self.g0)

    @property
    def g(self) -> float:
        return float(np.linalg.norm(self.g_I))


def dcm_ib(q) -> np.ndarray:
    """C_IB (body -> inertial) of q = (w, x, y, z), nominal_mpc.py:176-181."""
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _cross3(a, b) -> np.ndarray:
    """np.cross of two 3-vectors with its arithmetic (a1 b2 - a2 b1, ...: the same
    products and differences, so the same bits) without its general-axis overhead
    (~20 us a call, four per RK4 stage of ``step``)."""
    a0, a1, a2 = float(a[0]), float(a[1]), float(a[2])
    b0, b1, b2 = float(b[0]), float(b[1]), float(b[2])
    return np.array([a1 * b2 - a2 * b1, a2 * b0 - a0 * b2, a0 * b1 - a1 * b0])


def _skew(a) -> np.ndarray:
    return np.array([[0.0, -a[2], a[1]], [a[2], 0.0, -a[0]], [-a[1], a[0], 0.0]])


class Rocket6DoFDynamics:
    """rocket_6dof.py:92-738 (the members GPMPC, the uncertainty propagator and a
    Monte-Carlo caller use)."""
    IDX_MASS = 0
    IDX_POS = slice(1, 4)
    IDX_VEL = slice(4, 7)
    IDX_QUAT = slice(7, 11)
    IDX_OMEGA = slice(11, 14)
    N_STATE = 14
    N_CONTROL = 3

    def __init__(self, config: Optional[Rocket6DoFConfig] = None):
        self.config = config or Rocket6DoFConfig.szmuk_defaults()
        c = self.config
        self._params = Rocket6DoFParams(
            m_dry=c.m_dry, m_wet=c.m_wet, J_B=np.array(c.J_B, float), I_sp=c.I_sp, g0=c.g0,
            g_I=np.array(c.g_I, float), r_T_B=np.array(c.r_T_B, float), r_cp_B=np.array(c.r_cp_B, float),
            T_min=c.T_min, T_max=c.T_max, delta_max=c.delta_max, theta_max=c.theta_max,
            gamma_gs=c.gamma_gs, omega_max=c.omega_max, enable_aero=c.enable_aero)
        if c.enable_aero:
            raise NotImplementedError("aerodynamic moments are not part of the restated model "
                                      "(nominal_mpc.py:163-203 has none)")
        self._J = self._params.J_B
        self._Jinv = np.linalg.inv(self._J)
        diag = not np.any(self._J - np.diag(np.diag(self._J)))
        self._Jd = np.diag(self._J).copy() if diag else None  # divide, as nominal_mpc.py:197-203

    @property
    def params(self) -> Rocket6DoFParams:
        return self._params

    @property
    def n_state(self) -> int:
        return self.N_STATE

    @property
    def n_control(self) -> int:
        return self.N_CONTROL

    # ---- state packing and accessors (rocket_6dof.py:183-330) -------------
    def pack_state(self, mass, position, velocity, quaternion, omega) -> np.ndarray:
        return np.concatenate([[float(mass)], np.asarray(position, float), np.asarray(velocity, float),
                               np.asarray(quaternion, float), np.asarray(omega, float)])

    def create_initial_state(self, altitude: float = 10.0, downrange: float = 0.0, crossrange: float = 0.0,
                             velocity=None, tilt_angle: float = 0.0, tilt_axis=None, omega=None,
                             mass: Optional[float] = None) -> np.ndarray:
        """rocket_6dof.py:212-276."""
        position = np.array([altitude, crossrange, downrange])
        velocity = np.zeros(3) if velocity is None else np.asarray(velocity, float)
        if tilt_angle != 0.0:
            axis = np.array([0.0, 1.0, 0.0]) if tilt_axis is None else np.asarray(tilt_axis, float)
            axis = axis / np.linalg.norm(axis)
            h = tilt_angle / 2.0
            quaternion = np.array([np.cos(h), axis[0] * np.sin(h), axis[1] * np.sin(h), axis[2] * np.sin(h)])
        else:
            quaternion = np.array([1.0, 0.0, 0.0, 0.0])
        omega = np.zeros(3) if omega is None else np.asarray(omega, float)
        return self.pack_state(self.config.m_wet if mass is None else mass, position, velocity, quaternion, omega)

    def get_mass(self, x) -> float:
        return float(x[0])

    def get_position(self, x) -> np.ndarray:
        return np.asarray(x[1:4], float).copy()

    def get_velocity(self, x) -> np.ndarray:
        return np.asarray(x[4:7], float).copy()

    def get_quaternion(self, x) -> np.ndarray:
        return np.asarray(x[7:11], float).copy()

    def get_omega(self, x) -> np.ndarray:
        return np.asarray(x[11:14], float).copy()

    def get_altitude(self, x) -> float:
        return float(x[1])

    def get_speed(self, x) -> float:
        return float(np.linalg.norm(x[4:7]))

    def get_dcm(self, x) -> np.ndarray:
        """C_BI (body from inertial)."""
        return dcm_ib(np.asarray(x[7:11], float)).T

    def get_tilt_angle(self, x) -> float:
        """Angle between the body x (thrust) axis and the inertial vertical."""
        c = dcm_ib(np.asarray(x[7:11], float))[0, 0]
        return float(np.arccos(np.clip(c, -1.0, 1.0)))

    def get_gimbal_angle(self, u) -> float:
        u = np.asarray(u, float)
        t = np.linalg.norm(u)
        return 0.0 if t < 1e-10 else float(np.arccos(np.clip(u[0] / t, -1.0, 1.0)))

    def get_thrust_magnitude(self, u) -> float:
        return float(np.linalg.norm(u))

    def fuel_remaining(self, x) -> float:
        return float(x[0] - self._params.m_dry)

    def fuel_fraction(self, x) -> float:
        return self.fuel_remaining(x) / (self._params.m_wet - self._params.m_dry)

    # ---- dynamics (nominal_mpc.py:163-203; rocket_6dof.py:334-387) ----------
    def dynamics(self, x, u) -> np.ndarray:
        x = np.asarray(x, float); u = np.asarray(u, float)
        p = self._params
        m, v, q, w = x[0], x[4:7], x[7:11], x[11:14]
        out = np.empty(14)
        out[0] = -p.alpha * np.sqrt(u @ u)
        out[1:4] = v
        out[4:7] = dcm_ib(q) @ u / m + p.g_I
        qv = q[1:4]
        out[7] = 0.5 * -(w @ qv)
        out[8:11] = 0.5 * (q[0] * w + _cross3(w, qv))
        rhs = _cross3(p.r_T_B, u) - _cross3(w, self._J @ w)
        out[11:14] = rhs / self._Jd if self._Jd is not None else self._Jinv @ rhs
        return out

    def f(self, x, u) -> np.ndarray:
        return self.dynamics(x, u)

    def step(self, x, u, dt: Optional[float] = None) -> np.ndarray:
        """RK4 (discretization.py:229-252) + quaternion normalisation."""
        dt = self.config.default_dt if dt is None else dt
        x = np.asarray(x, float); u = np.asarray(u, float)
        k1 = self.dynamics(x, u)
        k2 = self.dynamics(x + dt * k1 / 2, u)
        k3 = self.dynamics(x + dt * k2 / 2, u)
        k4 = self.dynamics(x + dt * k3, u)
        xn = x + (dt / 6) * (k1 + 2 * k2 + 2 * k3 + k4)
        return self.normalize_state(xn)

    def f_discrete(self, x, u, dt: float) -> np.ndarray:
        return self.step(x, u, dt)

    def normalize_state(self, x) -> np.ndarray:
        x = np.array(x, float)
        x[7:11] = x[7:11] / np.sqrt(x[7:11] @ x[7:11])
        return x

    # ---- Jacobians (rocket_6dof.py:393-459) ---------------------------------
    def jacobian_x(self, x, u) -> np.ndarray:
        x = np.asarray(x, float); u = np.asarray(u, float)
        m, q, w = x[0], x[7:11], x[11:14]
        qw, qx, qy, qz = q
        u0, u1, u2 = u
        A = np.zeros((14, 14))
        A[1:4, 4:7] = np.eye(3)
        A[4:7, 0] = -(dcm_ib(q) @ u) / (m * m)
        dCu = np.array([  # d(C_IB u) / d(w, x, y, z)
            [-2 * qz * u1 + 2 * qy * u2, 2 * qy * u1 + 2 * qz * u2, -4 * qy * u0 + 2 * qx * u1 + 2 * qw * u2,
             -4 * qz * u0 - 2 * qw * u1 + 2 * qx * u2],
            [2 * qz * u0 - 2 * qx * u2, 2 * qy * u0 - 4 * qx * u1 - 2 * qw * u2, 2 * qx * u0 + 2 * qz * u2,
             2 * qw * u0 - 4 * qz * u1 + 2 * qy * u2],
            [-2 * qy * u0 + 2 * qx * u1, 2 * qz * u0 + 2 * qw * u1 - 4 * qx * u2,
             -2 * qw * u0 + 2 * qz * u1 - 4 * qy * u2, 2 * qx * u0 + 2 * qy * u1]])
        A[4:7, 7:11] = dCu / m
        wx, wy, wz = w
        A[7:11, 7:11] = 0.5 * np.array([[0, -wx, -wy, -wz], [wx, 0, -wz, wy], [wy, wz, 0, -wx],
                                        [wz, -wy, wx, 0]])
        A[7, 11:14] = -0.5 * q[1:4]
        A[8:11, 11:14] = 0.5 * np.array([[qw, qz, -qy], [-qz, qw, qx], [qy, -qx, qw]])
        # d/dw J^-1 (-w x J w) = J^-1 ([J w]x - [w]x J)
        A[11:14, 11:14] = self._Jinv @ (_skew(self._J @ w) - _skew(w) @ self._J)
        return A

    def jacobian_u(self, x, u) -> np.ndarray:
        x = np.asarray(x, float); u = np.asarray(u, float)
        p = self._params
        B = np.zeros((14, 3))
        B[0] = -p.alpha * u / np.sqrt(u @ u)
        B[4:7] = dcm_ib(x[7:11]) / x[0]
        B[11:14] = self._Jinv @ _skew(p.r_T_B)
        return B

    def A(self, x, u) -> np.ndarray:
        return self.jacobian_x(x, u)

    def B(self, x, u) -> np.ndarray:
        return self.jacobian_u(x, u)

    def linearize(self, x, u, dt: Optional[float] = None) -> Tuple[np.ndarray, np.ndarray]:
        """rocket_6dof.py:427-459: continuous Jacobians, or I + A_c dt, B_c dt."""
        A_c, B_c = self.jacobian_x(x, u), self.jacobian_u(x, u)
        if dt is not None:
            return np.eye(14) + A_c * dt, B_c * dt
        return A_c, B_c

    def linearize_discrete(self, x, u, dt: float):
        """rocket_6dof.py:461-488: A_d, B_d and c = F(x, u) - A_d x - B_d u."""
        A_d, B_d = self.linearize(x, u, dt)
        return A_d, B_d, self.step(x, u, dt) - A_d @ np.asarray(x, float) - B_d @ np.asarray(u, float)

    # ---- constraints and control utilities (rocket_6dof.py:492-669) ---------
    def thrust_constraint(self, u) -> Tuple[float, float]:
        t = self.get_thrust_magnitude(u)
        return self.config.T_min - t, t - self.config.T_max

    def glide_slope_constraint(self, x) -> float:
        """|r_yz| - tan(gamma_gs) r_x (negative = satisfied)."""
        return float(np.linalg.norm(x[2:4]) - np.tan(self.config.gamma_gs) * x[1])

    def gimbal_constraint(self, u) -> float:
        return self.get_gimbal_angle(u) - self.config.delta_max

    def tilt_constraint(self, x) -> float:
        return self.get_tilt_angle(x) - self.config.theta_max

    def angular_rate_constraint(self, x) -> float:
        return float(np.linalg.norm(x[11:14]) - self.config.omega_max)

    def hover_thrust(self, x) -> np.ndarray:
        """Body-frame thrust that cancels gravity: C_BI (-m g_I)."""
        x = np.asarray(x, float)
        return self.get_dcm(x) @ (-x[0] * self._params.g_I)

    def clamp_thrust(self, u) -> np.ndarray:
        """rocket_6dof.py:616-632."""
        u = np.asarray(u, float)
        t = np.linalg.norm(u)
        if t < 1e-10:
            return np.array([self.config.T_min, 0.0, 0.0])
        return u * (np.clip(t, self.config.T_min, self.config.T_max) / t)

    def matches_device_model(self) -> bool:
        """True when csrc/fleet6.hip's model can run this rocket: its J, r_T, g_I,
        alpha and g0 are runtime parameters (gpmpc_rollout6_config), the inertia
        tensor any invertible 3 x 3 matrix (rocket_J, ABI 4)."""
        J = np.asarray(self._params.J_B, float)
        return J.shape == (3, 3) and bool(np.all(np.isfinite(J))) and abs(np.linalg.det(J)) > 0.0

    def __repr__(self) -> str:
        return (f"Rocket6DoFDynamics(m_wet={self.config.m_wet}, m_dry={self.config.m_dry}, "
                f"T_range=[{self.config.T_min}, {self.config.T_max}])")


def create_szmuk_rocket() -> Rocket6DoFDynamics:
    return Rocket6DoFDynamics(Rocket6DoFConfig.szmuk_defaults())


def create_rocket_6dof(m_wet: float = 2.0, m_dry: float = 1.0, T_min: float = 1.5, T_max: float = 6.5,
                       I_sp: float = 30.0, **kwargs) -> Rocket6DoFDynamics:
    return Rocket6DoFDynamics(Rocket6DoFConfig(m_wet=m_wet, m_dry=m_dry, T_min=T_min, T_max=T_max,
                                               I_sp=I_sp, **kwargs))
