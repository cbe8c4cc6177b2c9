"""NominalMPC3DoF surface of reference src/mpc/nominal_mpc.py:532-700.

The reference solves the 3-DoF NLP with CasADi/IPOPT (both absent here: no
reference output pins it).  This mirror solves the same problem
class by sequential quadratic programming on the device ADMM: linearise the
Euler model around the current trajectory (FastRTI3DoF Jacobians), solve the
RTI QP warm-started from the previous iterate, repeat until the trajectory
moves less than ``tol`` (or ``max_sqp_iter``).  The cost is the reference's
(Q = diag(0,10,10,10,1,1,1), R = 0.01 I, terminal 10 Q, nominal_mpc.py:619-631)
evaluated on the returned trajectory.  Difference from the NLP, stated: the
thrust set is the QP's box (osqp_rti.py:198-201) instead of |u| <= 5.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .. import _lib
from .qp_builder import Q_DIAG, R_DIAG, QF_SCALE, RTIQPBuilder, solution_to_vector, vector_to_solution


@dataclass
class MPCConfig:
    """nominal_mpc.py:41-64 (+ the SQP controls of this mirror)."""
    N: int = 20
    dt: float = 0.1
    integration_method: str = "euler"
    max_iter: int = 100
    tol: float = 1e-6
    warm_start: bool = True
    verbose: bool = False
    soft_constraints: bool = False
    constraint_slack_weight: float = 1e4
    use_reference: bool = False
    max_sqp_iter: int = 10
    sqp_tol: float = 1e-4
    qp_max_iter: int = 50
    qp_eps: float = 1e-4


@dataclass
class MPCSolution:
    """nominal_mpc.py:67-82."""
    success: bool
    X_opt: np.ndarray
    U_opt: np.ndarray
    cost: float
    solve_time: float
    iterations: int
    status: str

    @property
    def u0(self) -> np.ndarray:
        return self.U_opt[0]


def trajectory_cost(X, U, x_ref, u_ref=None) -> float:
    """nominal_mpc.py:619-631: sum (x-x_t)'Q(x-x_t) + u'Ru + 10 (x_N-x_t)'Q(x_N-x_t);
    x_ref may be a trajectory (N+1, 7) and u_ref (N, 3) a control reference
    (gp_mpc.py:442-453)."""
    e = np.asarray(X) - np.asarray(x_ref)
    du = np.asarray(U) - (0.0 if u_ref is None else np.asarray(u_ref))
    return float(np.sum(e[:-1] ** 2 * Q_DIAG) + np.sum(du ** 2 * R_DIAG)
                 + QF_SCALE * np.sum(e[-1] ** 2 * Q_DIAG))


class _SQPBase:
    n_x, n_u = 7, 3

    def __init__(self, dynamics, config, ctx=None):
        self.dynamics = dynamics
        self.config = config
        p = getattr(dynamics, "params", None)
        self._g0 = float(getattr(p, "g0", 1.0))
        self._qp = RTIQPBuilder(config.N, config.dt, alpha=getattr(p, "alpha", 1.0 / 30.0),
                                g_vec=getattr(p, "g_vec", np.array([-1.0, 0.0, 0.0])))
        self._ctx = ctx or _lib.default_context()
        self._ws = _lib.QPWorkspace(self._ctx, self._qp.n, self._qp.m, self._qp.rowptr, self._qp.colidx,
                                    settings=_lib.qp_default_settings(max_iter=int(config.qp_max_iter),
                                                                      eps_abs=float(config.qp_eps),
                                                                      eps_rel=float(config.qp_eps)))
        self._X_warm = self._U_warm = None
        self._is_setup = True

    def setup(self) -> None:
        self._is_setup = True

    def reset_warm_start(self) -> None:
        self._X_warm = self._U_warm = None
        self._ws.reset()

    def _gp_mean(self, X, U):
        return None

    def _sqp(self, x0, x_target, X, U, max_iter, sign, x_ref=None, u_ref=None):
        t0 = time.perf_counter()
        P, q = self._qp.cost(np.tile(x_target, (self.config.N + 1, 1)) if x_ref is None else x_ref, u_ref)
        converged, it, status = False, 0, -10
        for it in range(1, max_iter + 1):
            dv = self._gp_mean(X, U)
            Aval, l, u = self._qp.constraints(X, U, x0, gp_dv=dv, sign=sign)
            r = self._ws.solve(Aval, P, q, l, u, solution_to_vector(X, U))
            status = int(r["status"][0])
            if status not in (1, 2, -2):
                break
            Xn, Un = vector_to_solution(r["x"][0], self.config.N)
            dX, dU = np.max(np.abs(Xn - X)), np.max(np.abs(Un - U))
            X, U = Xn, Un
            if dX < self.config.sqp_tol and dU < self.config.sqp_tol:
                converged = True
                break
        return X, U, converged, it, status, time.perf_counter() - t0


class NominalMPC3DoF(_SQPBase):
    def __init__(self, dynamics, config: Optional[MPCConfig] = None, ctx=None):
        super().__init__(dynamics, config or MPCConfig(), ctx=ctx)

    def solve(self, x0, x_target) -> MPCSolution:
        """nominal_mpc.py:640-679: cold start (linspace X, hover U) every call."""
        x0 = np.asarray(x0, float); x_target = np.asarray(x_target, float)
        self._ws.reset()
        N = self.config.N
        X = np.linspace(x0, x_target, N + 1)
        U = np.zeros((N, self.n_u)); U[:, 0] = x0[0] * self._g0
        X, U, conv, it, st, dt = self._sqp(x0, x_target, X, U, self.config.max_sqp_iter, -1.0)
        self._X_warm, self._U_warm = X.copy(), U.copy()
        cost = trajectory_cost(X, U, x_target) if conv else np.inf
        return MPCSolution(success=conv, X_opt=X, U_opt=U, cost=cost, solve_time=dt,
                           iterations=it, status="Optimal" if conv else _lib.QP_STATUS_TEXT.get(st, str(st)))
