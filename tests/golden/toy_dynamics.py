"""Deterministic stand-in plants for the propagation fixtures (F9).

The reference's 6-DoF plant lives in the absent ``simdyn`` package, so the F9
fixture drives the reference UncertaintyPropagator with this 14-state model
(mass, position, velocity, attitude quaternion, body rates; explicit Euler,
central-difference Jacobians) and the tests drive the mirror with the same
one.  Test infrastructure only.
"""
from __future__ import annotations

import numpy as np


def _dcm(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


class ToyRocket14:
    n_state = 14
    n_control = 3

    def __init__(self):
        self.alpha = 0.05
        self.g = np.array([-1.0, 0.0, 0.0])
        self.J = np.array([0.2, 0.5, 0.5])
        self.r_T = np.array([-0.25, 0.0, 0.0])

    def f(self, x, u):
        x = np.asarray(x, float); u = np.asarray(u, float)
        m, v, q, w = x[0], x[4:7], x[7:11], x[11:14]
        out = np.empty(14)
        out[0] = -self.alpha * np.sqrt(u @ u + 1e-12)
        out[1:4] = v
        out[4:7] = _dcm(q) @ u / m + self.g
        wx, wy, wz = w
        Om = np.array([[0, -wx, -wy, -wz], [wx, 0, wz, -wy], [wy, -wz, 0, wx], [wz, wy, -wx, 0]])
        out[7:11] = 0.5 * Om @ q
        out[11:14] = (np.cross(self.r_T, u) - np.cross(w, self.J * w)) / self.J
        return out

    def step(self, x, u, dt=0.1):
        return np.asarray(x, float) + dt * self.f(x, u)

    def linearize(self, x, u, dt=0.1):
        x = np.asarray(x, float); u = np.asarray(u, float)
        A = np.empty((14, 14)); B = np.empty((14, 3))
        for i in range(14):
            h = 1e-6 * max(1.0, abs(x[i])); e = np.zeros(14); e[i] = h
            A[:, i] = (self.step(x + e, u, dt) - self.step(x - e, u, dt)) / (2 * h)
        for i in range(3):
            h = 1e-6 * max(1.0, abs(u[i])); e = np.zeros(3); e[i] = h
            B[:, i] = (self.step(x, u + e, dt) - self.step(x, u - e, dt)) / (2 * h)
        return A, B


def toy_case(seed=9, N=10):
    """x0 (14,), U (N, 3): a descending, slightly rotating vehicle."""
    rs = np.random.RandomState(seed)
    q = np.array([1.0, 0.02, -0.03, 0.01]); q /= np.linalg.norm(q)
    x0 = np.concatenate([[2.0], [20.0, 1.5, -1.0], [-2.0, 0.3, 0.1], q, [0.02, -0.01, 0.03]])
    U = np.array([2.2, 0.0, 0.0]) + 0.1 * rs.randn(N, 3)
    return x0, U


class _P3:
    g0 = 1.0
    alpha = 1.0 / 30.0
    g_vec = np.array([-1.0, 0.0, 0.0])


class DragRocket3DoF:
    """3-DoF Euler plant (nominal_mpc.py:585-605) plus the aero drag of
    experiments/dispersion.py:349-360 (rho 0.02, Cd = A = 1) -- a caller's
    plant whose step differs from the RTI's built-in model and whose
    Jacobian is not on the analytic Jacobian's pattern (drag couples every
    velocity component with mass and the other components).  F6b drives the
    reference OSQPRTIMPC / FastRTI3DoF with it; the tests drive the mirror."""
    n_state = 7
    n_control = 3
    params = _P3()

    def step(self, x, u, dt):
        x = np.asarray(x, float); u = np.asarray(u, float)
        out = np.empty(7)
        out[0] = x[0] - dt * self.params.alpha * np.sqrt(u @ u)
        out[1:4] = x[1:4] + dt * x[4:7]
        v = x[4:7]; s = np.sqrt(v @ v)
        drag = -(0.5 * 0.02 * s * s) / x[0] * (v / s) if s > 1.0 else np.zeros(3)
        out[4:7] = v + dt * (u / x[0] + self.params.g_vec + drag)
        return out
