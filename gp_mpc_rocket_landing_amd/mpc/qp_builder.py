"""RTI QP data for the 3-DoF MPC, vectorised over the horizon.

Same QP as OSQPRTIMPC._build_cost_matrix / _build_constraint_matrix
(osqp_rti.py:168-372) with FastRTI3DoF's analytic Jacobians
(osqp_rti.py:656-710):

    z = [x_0, u_0, x_1, u_1, ..., x_{N-1}, u_{N-1}, x_N]
    P = blkdiag(Q, R, ..., Q, R, 10 Q),  q = -Q x_ref[k] (x-blocks)
    A = [ I_7 on x_0 ;  per k: A_k x_k + B_k u_k - x_{k+1} ;  I_n ]
    l = u = [x_init ; s c_k ; box bounds]

The sparsity pattern is the structural pattern of the analytic Jacobians
(26 entries per stage block) and is fixed for a given N, so one pattern serves
every solve and every landing; the reference filters |a| > 1e-10,
which stores the same QP with a value-dependent pattern.  ``dense=True``
stores every entry of A_k and B_k (77 per stage block) -- the pattern for
OSQPRTIMPC's finite-difference Jacobians of an arbitrary plant
(osqp_rti.py:374-401), whose non-zeros are not known in advance.

c_k = f(x_k, u_k) - A_k x_k - B_k u_k takes f from the caller's plant when
``f_next`` (the plant's dynamics.step at every stage, osqp_rti.py:339) is
given, else from the Euler 3-DoF model restated here (nominal_mpc.py:585-605).  s = +1 reproduces
the reference's right-hand side; the GP-MPC adapter uses s = -1
(x+ = A x + B u + c, gp_mpc.py:410-411) with the GP mean dt*d_v added to the
velocity rows of c_k (gp_mpc.py:309-314).
"""
from __future__ import annotations

import numpy as np

N_X, N_U = 7, 3
Q_DIAG = np.array([0.0, 10.0, 10.0, 10.0, 1.0, 1.0, 1.0])   # osqp_rti.py:171-182
R_DIAG = np.full(N_U, 0.01)
QF_SCALE = 10.0
X_MIN = np.array([-np.inf, -100.0, -100.0, -100.0, -50.0, -50.0, -50.0])  # osqp_rti.py:198-201
X_MAX = np.array([np.inf, 500.0, 100.0, 100.0, 50.0, 50.0, 50.0])
U_MIN = np.array([0.3, -5.0, -5.0])
U_MAX = np.array([5.0, 5.0, 5.0])

# (row i of a stage block) -> sorted columns relative to the stage start c0:
# A_k structure (I + dt dF/dx), B_k structure, then -I on x_{k+1}
_BLOCK_COLS = [
    [0, 7, 8, 9, 10],     # m:   A00, B00..B02, -1
    [1, 4, 11],           # r_x: A11, A14, -1
    [2, 5, 12],
    [3, 6, 13],
    [0, 4, 7, 14],        # v_x: A40, A44, B40, -1
    [0, 5, 8, 15],
    [0, 6, 9, 16],
]
DYN_NNZ = sum(len(c) for c in _BLOCK_COLS)  # 26


def n_vars(N: int) -> int:
    return (N + 1) * N_X + N * N_U


def solution_to_vector(X, U) -> np.ndarray:
    """osqp_rti.py:601-615."""
    N = U.shape[0]
    z = np.empty(n_vars(N))
    zz = z[:N * (N_X + N_U)].reshape(N, N_X + N_U)
    zz[:, :N_X] = X[:N]
    zz[:, N_X:] = U
    z[N * (N_X + N_U):] = X[N]
    return z


def vector_to_solution(z, N: int):
    """osqp_rti.py:616-631."""
    zz = np.asarray(z)[:N * (N_X + N_U)].reshape(N, N_X + N_U)
    X = np.empty((N + 1, N_X))
    X[:N] = zz[:, :N_X]
    X[N] = z[N * (N_X + N_U):]
    return X, zz[:, N_X:].copy()


class RTIQPBuilder:
    """Pattern + per-solve values of the RTI QP for horizon N."""

    def __init__(self, N: int, dt: float, alpha: float = 1.0 / 30.0,
                 g_vec=(-1.0, 0.0, 0.0), dense: bool = False):
        self.N, self.dt, self.alpha = int(N), float(dt), float(alpha)
        self.dense = bool(dense)
        block = ([list(range(N_X + N_U)) + [N_X + N_U + i] for i in range(N_X)] if self.dense
                 else _BLOCK_COLS)
        self.g_vec = np.asarray(g_vec, float)
        N = self.N
        self.n = n_vars(N)
        self.m = N_X * (N + 1) + self.n
        cols, rowlen = [], []
        for i in range(N_X):                      # x_0 identity rows
            cols.append([i]); rowlen.append(1)
        for k in range(N):
            c0 = k * (N_X + N_U)
            for i in range(N_X):
                cols.append([c0 + c for c in block[i]]); rowlen.append(len(block[i]))
        for j in range(self.n):                   # bound rows
            cols.append([j]); rowlen.append(1)
        self.rowptr = np.concatenate([[0], np.cumsum(rowlen)]).astype(np.int32)
        self.colidx = np.concatenate([np.asarray(c) for c in cols]).astype(np.int32)
        self.nnz = int(self.rowptr[-1])
        # cost diagonal and box bounds (constant)
        d = np.zeros(self.n)
        blk = d[:N * (N_X + N_U)].reshape(N, N_X + N_U)
        blk[:, :N_X] = Q_DIAG
        blk[:, N_X:] = R_DIAG
        d[N * (N_X + N_U):] = QF_SCALE * Q_DIAG
        self.P_diag = d
        lb = np.empty(self.n); ub = np.empty(self.n)
        lbb = lb[:N * (N_X + N_U)].reshape(N, N_X + N_U); ubb = ub[:N * (N_X + N_U)].reshape(N, N_X + N_U)
        lbb[:, :N_X] = X_MIN; lbb[:, N_X:] = U_MIN
        ubb[:, :N_X] = X_MAX; ubb[:, N_X:] = U_MAX
        lb[N * (N_X + N_U):] = X_MIN; ub[N * (N_X + N_U):] = X_MAX
        self._lb, self._ub = lb, ub

    # ------------------------------------------------------------------
    def cost(self, x_ref, u_ref=None):
        """(P diagonal, q) for the reference trajectory x_ref (N+1, 7) and, when
        given, the control reference u_ref (N, 3): sum |x_k - x_ref[k]|_Q^2 +
        |u_k - u_ref[k]|_R^2 (gp_mpc.py:442-453; osqp_rti.py's cost has u_ref = 0)."""
        N = self.N
        x_ref = np.asarray(x_ref, float)
        q = np.zeros(self.n)
        qq = q[:N * (N_X + N_U)].reshape(N, N_X + N_U)
        qq[:, :N_X] = -Q_DIAG * x_ref[:N]
        if u_ref is not None:
            qq[:, N_X:] = -R_DIAG * np.asarray(u_ref, float)[:N]
        q[N * (N_X + N_U):] = -QF_SCALE * Q_DIAG * x_ref[N]
        return self.P_diag, q

    def jacobians(self, X_lin, U_lin):
        """FastRTI3DoF._linearize (osqp_rti.py:656-710) for all stages: A (N,7,7), B (N,7,3)."""
        N, dt = self.N, self.dt
        X = np.asarray(X_lin, float)[:N]; U = np.asarray(U_lin, float)[:N]
        m = X[:, 0]
        tm = np.sqrt(np.sum(U * U, axis=1)) + 1e-10
        A = np.tile(np.eye(N_X), (N, 1, 1))
        A[:, 1, 4] = A[:, 2, 5] = A[:, 3, 6] = dt
        A[:, 4:7, 0] = -U / (m * m)[:, None] * dt
        B = np.zeros((N, N_X, N_U))
        B[:, 0, :] = -self.alpha * U / tm[:, None] * dt
        B[:, 4, 0] = B[:, 5, 1] = B[:, 6, 2] = dt / m
        return A, B

    def constraints(self, X_lin, U_lin, x_init, gp_dv=None, sign: float = 1.0, jac=None,
                    f_next=None):
        """(A values in pattern order, l, u) around the linearisation (X_lin, U_lin).

        ``jac`` = (A (N,7,7), B (N,7,3)) overrides the analytic Jacobians; with
        the structural pattern it must keep that pattern's zeros.  ``f_next``
        (N,7) = the plant's step at (X_lin[k], U_lin[k]) for c_k."""
        N, dt = self.N, self.dt
        X = np.asarray(X_lin, float); U = np.asarray(U_lin, float)
        A, B = self.jacobians(X, U) if jac is None else (np.asarray(jac[0], float), np.asarray(jac[1], float))
        if self.dense:
            v = np.concatenate([A, B, np.broadcast_to(-1.0, (N, N_X, 1))], axis=2)
        else:
            v = np.empty((N, DYN_NNZ))
            v[:, 0] = A[:, 0, 0]; v[:, 1:4] = B[:, 0, :]; v[:, 4] = -1.0
            for i in range(1, 4):
                o = 5 + 3 * (i - 1)
                v[:, o] = A[:, i, i]; v[:, o + 1] = A[:, i, i + 3]; v[:, o + 2] = -1.0
            for i in range(4, 7):
                o = 14 + 4 * (i - 4)
                v[:, o] = A[:, i, 0]; v[:, o + 1] = A[:, i, i]; v[:, o + 2] = B[:, i, i - 4]; v[:, o + 3] = -1.0
        Aval = np.concatenate([np.ones(N_X), v.reshape(-1), np.ones(self.n)])
        # c_k = f(x_k, u_k) - A_k x_k - B_k u_k   (+ dt d_v on the velocity rows)
        Xk, Uk = X[:N], U[:N]
        if f_next is not None:
            f = np.asarray(f_next, float).reshape(N, N_X)
        else:
            f = np.empty((N, N_X))
            f[:, 0] = Xk[:, 0] - dt * self.alpha * np.sqrt(np.sum(Uk * Uk, axis=1))
            f[:, 1:4] = Xk[:, 1:4] + dt * Xk[:, 4:7]
            f[:, 4:7] = Xk[:, 4:7] + dt * (Uk / Xk[:, :1] + self.g_vec)
        c = f - np.einsum("kij,kj->ki", A, Xk) - np.einsum("kij,kj->ki", B, Uk)
        if gp_dv is not None:
            c[:, 4:7] += np.asarray(gp_dv, float)[:N] * dt
        leq = np.concatenate([np.asarray(x_init, float), sign * c.reshape(-1)])
        return Aval, np.concatenate([leq, self._lb]), np.concatenate([leq, self._ub])

    def initial_guess(self, x0, x_target, g: float = 1.0):
        """OSQPRTIMPC.initialize (osqp_rti.py:403-452): linear interpolation X, hover U."""
        N = self.N
        a = (np.arange(N + 1) / N)[:, None]
        X = (1.0 - a) * np.asarray(x0, float) + a * np.asarray(x_target, float)
        U = np.zeros((N, N_U)); U[:, 0] = float(x0[0]) * g
        return X, U
