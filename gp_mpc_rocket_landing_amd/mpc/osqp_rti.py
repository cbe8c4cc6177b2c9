"""OSQP-RTI controller surfaces of reference src/mpc/osqp_rti.py; the QP solve
runs on the GPU.

OSQPRTIMPC / FastRTI3DoF keep the reference's real-time-iteration protocol
(osqp_rti.py:403-599): initialize -> linear-interpolation guess and hover
thrust, fresh solver workspace; prepare -> cost vector update; feedback ->
QP around the current linearisation with the measured state, warm start from
the shifted previous solution, solve, on "solved"/"solved inaccurate" take
X_opt as the next linearisation and shift it for the warm start, otherwise
fall back to the shifted previous plan.  The OSQP setup/update/warm_start/
solve calls are replaced by the batched device ADMM (gpmpc_qp_solve_batched,
OSQP-0.6 semantics, rho and scaled y carried between solves as OSQP's
workspace does).

c_k = f(x_k, u_k) - A_k x_k - B_k u_k evaluates f with the caller's plant,
``dynamics.step`` (osqp_rti.py:339).  OSQPRTIMPC linearises by forward
differences through that plant (osqp_rti.py:374-401, eps 1e-6) and keeps,
like the reference, the entries of A_k, B_k with |a| > 1e-10
(osqp_rti.py:299-312): the pattern is re-derived at every solve (the
reference's update(Ax=...) assumes it does not move).
FastRTI3DoF uses the analytic 3-DoF Jacobians (osqp_rti.py:656-710) on
their structural pattern, explicit zeros included.

``rhs_sign`` (default +1) reproduces the reference's equality right-hand side
l = u = +c_k; -1 gives x+ = A x + B u + c.  Structural zeros are
stored explicitly; polishing is not supported.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from .. import _lib
from .qp_builder import RTIQPBuilder, solution_to_vector, vector_to_solution


@dataclass
class OSQPRTIConfig:
    """osqp_rti.py:45-71."""
    N: int = 15
    dt: float = 0.1
    osqp_verbose: bool = False
    osqp_max_iter: int = 50
    osqp_eps_abs: float = 1e-4
    osqp_eps_rel: float = 1e-4
    osqp_polish: bool = False
    osqp_warm_start: bool = True
    osqp_scaling: int = 3
    max_rti_iter: int = 1
    trust_region: float = 10.0
    n_x: int = 7
    n_u: int = 3
    precompute_matrices: bool = True
    rhs_sign: float = 1.0


@dataclass
class OSQPRTISolution:
    """osqp_rti.py:74-86."""
    u0: np.ndarray
    X_opt: np.ndarray
    U_opt: np.ndarray
    cost: float
    prep_time_ms: float
    feedback_time_ms: float
    total_time_ms: float
    osqp_iterations: int
    success: bool


def qp_settings_from(cfg) -> "_lib.QPSettings":
    if getattr(cfg, "osqp_polish", False):
        raise NotImplementedError("solution polishing is not part of the device ADMM")
    return _lib.qp_default_settings(max_iter=int(cfg.osqp_max_iter), eps_abs=float(cfg.osqp_eps_abs),
                                    eps_rel=float(cfg.osqp_eps_rel), warm_start=int(cfg.osqp_warm_start),
                                    scaling=int(cfg.osqp_scaling))


class OSQPRTIMPC:
    """osqp_rti.py:89-639."""

    # finite-difference Jacobians: any entry may be non-zero.  The filtered
    # pattern must fit the device QP's caps (_lib.QP_NNZMAX = 896 non-zeros,
    # n <= 216, m <= 360): the drag Euler plant at N = 20 has 854; a plant whose
    # Jacobians are dense (e.g. an RK4 step, ~44 non-zeros per stage) exceeds the
    # cap from N ~ 16 on, and the first solve then raises ValueError.
    _DENSE_PATTERN = True

    def __init__(self, dynamics, config: Optional[OSQPRTIConfig] = None, ctx=None):
        self.dynamics = dynamics
        self.config = config or OSQPRTIConfig()
        if self.config.n_x != 7 or self.config.n_u != 3:
            raise NotImplementedError("the RTI QP is assembled for the 3-DoF model (n_x=7, n_u=3)")
        self.n_x, self.n_u, self.N = self.config.n_x, self.config.n_u, self.config.N
        self.n_vars = (self.N + 1) * self.n_x + self.N * self.n_u
        p = getattr(dynamics, "params", None)
        alpha = getattr(p, "alpha", 1.0 / 30.0)
        g_vec = getattr(p, "g_vec", np.array([-1.0, 0.0, 0.0]))
        self._qp = RTIQPBuilder(self.N, self.config.dt, alpha=alpha, g_vec=g_vec,
                                dense=self._DENSE_PATTERN)
        self._ctx = ctx or _lib.default_context()
        self._solver: Optional[_lib.QPWorkspace] = None
        self._x_ref = self._u_ref = None
        self._X_prev = self._U_prev = None
        self._X_lin = self._U_lin = None
        self._q = None
        self._pattern = None

    def initialize(self, x0, x_target, X_init=None, U_init=None) -> None:
        """osqp_rti.py:403-452."""
        N = self.N
        x0 = np.asarray(x0, float)
        self._x_ref = np.tile(np.asarray(x_target, float), (N + 1, 1))
        self._u_ref = np.zeros((N, self.n_u))
        if hasattr(self.dynamics, "params"):
            self._u_ref[:, 0] = x0[0] * getattr(self.dynamics.params, "g", 1.0)
        else:
            self._u_ref[:, 0] = x0[0] * 1.0
        if X_init is not None:
            self._X_lin = np.array(X_init, float)
        else:
            a = (np.arange(N + 1) / N)[:, None]
            self._X_lin = (1 - a) * x0 + a * np.asarray(x_target, float)
        self._U_lin = np.array(U_init, float) if U_init is not None else self._u_ref.copy()
        self._X_prev, self._U_prev = self._X_lin.copy(), self._U_lin.copy()
        self._setup_osqp(x0)

    def _setup_osqp(self, x_init) -> None:
        """osqp_rti.py:454-478: a fresh workspace (rho = settings.rho, y = 0)."""
        b = self._qp
        self._solver = _lib.QPWorkspace(self._ctx, b.n, b.m, b.rowptr, b.colidx, batch=1,
                                        settings=qp_settings_from(self.config))
        _, self._q = b.cost(self._x_ref)

    def _linearize(self, x, u, eps: float = 1e-6):
        """osqp_rti.py:374-401: forward differences through dynamics.step."""
        dt = self.config.dt
        x = np.asarray(x, float); u = np.asarray(u, float)
        A = np.zeros((self.n_x, self.n_x)); B = np.zeros((self.n_x, self.n_u))
        x_next_nom = np.asarray(self.dynamics.step(x, u, dt), float)
        for i in range(self.n_x):
            xp = x.copy(); xp[i] += eps
            A[:, i] = (np.asarray(self.dynamics.step(xp, u, dt), float) - x_next_nom) / eps
        for i in range(self.n_u):
            up = u.copy(); up[i] += eps
            B[:, i] = (np.asarray(self.dynamics.step(x, up, dt), float) - x_next_nom) / eps
        return A, B

    def _stage_jacobians(self):
        AB = [self._linearize(self._X_lin[k], self._U_lin[k]) for k in range(self.N)]
        return np.array([a for a, _ in AB]), np.array([b for _, b in AB])

    def _constraints(self, x_current) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """osqp_rti.py:260-372: Jacobians per stage, c_k from the caller's plant.
        Sets ``self._pattern`` (rowptr, colidx) of the returned A values."""
        dt = self.config.dt
        f_next = np.array([self.dynamics.step(self._X_lin[k], self._U_lin[k], dt) for k in range(self.N)],
                          dtype=float)
        Aval, l, u = self._qp.constraints(self._X_lin, self._U_lin, x_current, sign=self.config.rhs_sign,
                                          jac=self._stage_jacobians(), f_next=f_next)
        b = self._qp
        if not b.dense:
            self._pattern = (b.rowptr, b.colidx)
            return Aval, l, u
        # |a| > 1e-10 on the A_k / B_k entries (osqp_rti.py:299-312); the x0 and
        # bound identities and the -I of x_{k+1} always stay
        keep = np.ones(Aval.size, bool)
        dyn = slice(self.n_x, self.n_x + self.N * self.n_x * (self.n_x + self.n_u + 1))
        blk = keep[dyn].reshape(self.N, self.n_x, self.n_x + self.n_u + 1)
        blk[:, :, :-1] = np.abs(Aval[dyn].reshape(blk.shape)[:, :, :-1]) > 1e-10
        rows = np.repeat(np.arange(b.m), np.diff(b.rowptr))
        rowptr = np.concatenate([[0], np.cumsum(np.bincount(rows[keep], minlength=b.m))]).astype(np.int32)
        if int(rowptr[-1]) > _lib.QP_NNZMAX:
            raise ValueError(f"the plant's Jacobians give {int(rowptr[-1])} constraint non-zeros at N = {self.N}; "
                             f"the device QP holds at most {_lib.QP_NNZMAX} (QP_NNZMAX, csrc/qp.h)")
        self._pattern = (rowptr, b.colidx[keep])
        return Aval[keep], l, u

    def prepare(self) -> float:
        """osqp_rti.py:480-499."""
        t0 = time.perf_counter()
        if self._solver is None:
            return 0.0
        _, self._q = self._qp.cost(self._x_ref)
        return (time.perf_counter() - t0) * 1000

    def feedback(self, x_current) -> OSQPRTISolution:
        """osqp_rti.py:501-567."""
        t0 = time.perf_counter()
        Aval, l, u = self._constraints(np.asarray(x_current, float))
        t_update = time.perf_counter()
        xw = None
        if self._X_prev is not None and self.config.osqp_warm_start:
            xw = solution_to_vector(self._X_prev, self._U_prev)
        r = self._solver.solve(Aval, self._qp.P_diag, self._q, l, u, xw, pattern=self._pattern)
        t_solve = time.perf_counter()
        status = int(r["status"][0])
        if status in (1, 2):
            X_opt, U_opt = vector_to_solution(r["x"][0], self.N)
            u0, cost, success = U_opt[0], float(r["obj_val"][0]), True
            self._X_lin, self._U_lin = X_opt.copy(), U_opt.copy()
            self._X_prev = np.vstack([X_opt[1:], X_opt[-1:]])
            self._U_prev = np.vstack([U_opt[1:], U_opt[-1:]])
        else:
            X_opt = self._X_prev if self._X_prev is not None else self._X_lin
            U_opt = self._U_prev if self._U_prev is not None else self._U_lin
            u0, cost, success = U_opt[0], np.inf, False
        self.last_status = status
        return OSQPRTISolution(u0=u0, X_opt=X_opt, U_opt=U_opt, cost=cost, prep_time_ms=0.0,
                               feedback_time_ms=(t_solve - t_update) * 1000,
                               total_time_ms=(time.perf_counter() - t0) * 1000,
                               osqp_iterations=int(r["iter"][0]), success=success)

    def step(self, x_current) -> OSQPRTISolution:
        """osqp_rti.py:569-599."""
        t0 = time.perf_counter()
        prep = self.prepare()
        sol = self.feedback(x_current)
        return OSQPRTISolution(u0=sol.u0, X_opt=sol.X_opt, U_opt=sol.U_opt, cost=sol.cost,
                               prep_time_ms=prep, feedback_time_ms=sol.feedback_time_ms,
                               total_time_ms=(time.perf_counter() - t0) * 1000,
                               osqp_iterations=sol.osqp_iterations, success=sol.success)

    def update_reference(self, x_target) -> None:
        self._x_ref = np.tile(np.asarray(x_target, float), (self.N + 1, 1))

    def get_predicted_trajectory(self) -> Tuple[np.ndarray, np.ndarray]:
        return self._X_lin.copy(), self._U_lin.copy()


class FastRTI3DoF(OSQPRTIMPC):
    """osqp_rti.py:642-710: 3-DoF RTI with analytic Jacobians."""

    _DENSE_PATTERN = False

    def __init__(self, dynamics, config: Optional[OSQPRTIConfig] = None, ctx=None):
        config = config or OSQPRTIConfig()
        config.n_x = 7
        config.n_u = 3
        super().__init__(dynamics, config, ctx=ctx)

    def _linearize(self, x, u, eps: float = 1e-6):  # noqa: ARG002
        A, B = self._qp.jacobians(np.asarray(x, float)[None], np.asarray(u, float)[None])
        return A[0], B[0]

    def _stage_jacobians(self):
        return self._qp.jacobians(self._X_lin, self._U_lin)
