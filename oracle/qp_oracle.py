"""numpy restatement of the 3-DoF plant, analytic linearisation and the OSQP-RTI
QP data assembly (TEST INFRASTRUCTURE ONLY).

Reference: src/mpc/osqp_rti.py (OSQPRTIMPC / FastRTI3DoF) and the 3-DoF Euler
model of src/mpc/nominal_mpc.py:585-605.  ``simdyn`` (the reference's plant
package) is absent and undeclared, so the plant is restated from those formulas
with alpha = 1/(I_sp*g0) = 1/30, g = [-1, 0, 0] (rocket_3dof.py:33-64).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

N_X, N_U = 7, 3
ALPHA = 1.0 / 30.0          # 1/(I_sp*g0), rocket_3dof.py:40-41
G_VEC = np.array([-1.0, 0.0, 0.0])  # rocket_3dof.py:63-64
G_RTI = 1.0                 # osqp_rti.py:428,676 getattr(params, "g", 1.0)

Q_DIAG = np.array([0.0, 10.0, 10.0, 10.0, 1.0, 1.0, 1.0])  # osqp_rti.py:171-182
R_DIAG = np.full(3, 0.01)
QF_DIAG = 10.0 * Q_DIAG
X_MIN = np.array([-np.inf, -100, -100, -100, -50, -50, -50.0])  # osqp_rti.py:198-201
X_MAX = np.array([np.inf, 500, 100, 100, 50, 50, 50.0])
U_MIN = np.array([0.3, -5, -5.0])
U_MAX = np.array([5.0, 5, 5])


def plant_step(x, u, dt):
    """3-DoF Euler step (nominal_mpc.py:585-605): m+ = m - dt*alpha*|u|, r+ = r + dt v,
    v+ = v + dt (u/m + g)."""
    x = np.asarray(x, float); u = np.asarray(u, float)
    out = np.empty(7)
    out[0] = x[0] - dt * ALPHA * np.sqrt(u @ u)
    out[1:4] = x[1:4] + dt * x[4:7]
    out[4:7] = x[4:7] + dt * (u / x[0] + G_VEC)
    return out


def drag_residual(x):
    """Aero residual of experiments/dispersion.py:349-360 (rho=0.02, Cd=A=1) as an
    acceleration: -0.5 rho Cd A |v|^2 / m * v/|v| when |v| > 1, else 0."""
    v = x[4:7]; s = np.sqrt(v @ v)
    if s > 1.0:
        return -(0.5 * 0.02 * s * s) / x[0] * (v / s)
    return np.zeros(3)


def linearize(x, u, dt):
    """FastRTI3DoF._linearize (osqp_rti.py:656-710)."""
    m = x[0]; T = np.asarray(u, float)
    tm = np.sqrt(T @ T) + 1e-10
    A = np.eye(7)
    A[1, 4] = A[2, 5] = A[3, 6] = dt
    A[4:7, 0] = -T / m ** 2 * dt
    B = np.zeros((7, 3))
    B[0, :] = -ALPHA * T / tm * dt
    B[4, 0] = B[5, 1] = B[6, 2] = dt / m
    return A, B


def n_vars(N):
    return (N + 1) * N_X + N * N_U


def cost(N, x_ref):
    """_build_cost_matrix (osqp_rti.py:203-258): P (CSC) and q."""
    n = n_vars(N)
    d = np.zeros(n); q = np.zeros(n)
    for k in range(N):
        o = k * (N_X + N_U)
        d[o:o + N_X] = Q_DIAG; d[o + N_X:o + N_X + N_U] = R_DIAG
        q[o:o + N_X] = -Q_DIAG * x_ref[k]
    o = N * (N_X + N_U)
    d[o:o + N_X] = QF_DIAG
    q[o:o + N_X] = -QF_DIAG * x_ref[N]
    nz = d != 0
    P = sp.csc_matrix((d[nz], (np.nonzero(nz)[0], np.nonzero(nz)[0])), shape=(n, n))
    return P, q


# structural non-zeros of the analytic 3-DoF Jacobians (osqp_rti.py:682-708)
A_STRUCT = np.eye(7, dtype=bool)
A_STRUCT[1, 4] = A_STRUCT[2, 5] = A_STRUCT[3, 6] = True
A_STRUCT[4:7, 0] = True
B_STRUCT = np.zeros((7, 3), dtype=bool)
B_STRUCT[0, :] = True
B_STRUCT[4, 0] = B_STRUCT[5, 1] = B_STRUCT[6, 2] = True


def constraints(X_lin, U_lin, x_init, dt, gp_dv=None, sign=+1.0, filter_small=True):
    """_build_constraint_matrix (osqp_rti.py:260-372).

    Rows: [x0 identity (7); per k: A_k x_k + B_k u_k - x_{k+1} (7); bounds identity (n)].
    l = u = [x_init; sign*c_k; ...].  The reference sets +c_k (sign=+1);
    the GP-MPC adapter uses sign=-1 (x+ = A x + B u + c) and adds the GP mean
    dt*d_v on the velocity rows of c_k (gp_mpc.py:309-314, 410-411).
    ``filter_small`` keeps the |a| > 1e-10 value filter; False keeps
    the structural pattern of the analytic Jacobians (zeros stored explicitly), the
    fixed pattern the batched HIP solver shares across landings.
    """
    N = U_lin.shape[0]; n = n_vars(N)
    rows, cols, vals = [], [], []
    for i in range(N_X):
        rows.append(i); cols.append(i); vals.append(1.0)
    neq = N_X * (N + 1)
    leq = np.zeros(neq)
    leq[:N_X] = x_init
    for k in range(N):
        r0 = N_X * (k + 1); c0 = k * (N_X + N_U)
        Ak, Bk = linearize(X_lin[k], U_lin[k], dt)
        for i in range(N_X):
            for j in range(N_X):
                if (A_STRUCT[i, j] if not filter_small else abs(Ak[i, j]) > 1e-10):
                    rows.append(r0 + i); cols.append(c0 + j); vals.append(Ak[i, j])
            for j in range(N_U):
                if (B_STRUCT[i, j] if not filter_small else abs(Bk[i, j]) > 1e-10):
                    rows.append(r0 + i); cols.append(c0 + N_X + j); vals.append(Bk[i, j])
            rows.append(r0 + i); cols.append(c0 + N_X + N_U + i); vals.append(-1.0)
        xn = plant_step(X_lin[k], U_lin[k], dt)
        ck = xn - Ak @ X_lin[k] - Bk @ U_lin[k]
        if gp_dv is not None:
            ck[4:7] += gp_dv[k] * dt
        leq[r0:r0 + N_X] = sign * ck
    Aeq = sp.csc_matrix((vals, (rows, cols)), shape=(neq, n))
    lb = np.zeros(n); ub = np.zeros(n)
    for k in range(N):
        o = k * (N_X + N_U)
        lb[o:o + N_X] = X_MIN; ub[o:o + N_X] = X_MAX
        lb[o + N_X:o + N_X + N_U] = U_MIN; ub[o + N_X:o + N_X + N_U] = U_MAX
    o = N * (N_X + N_U)
    lb[o:] = X_MIN; ub[o:] = X_MAX
    A = sp.vstack([Aeq, sp.eye(n, format="csc")], format="csc")
    return A, np.concatenate([leq, lb]), np.concatenate([leq, ub])


def to_vector(X, U):
    """_solution_to_vector (osqp_rti.py:601-615)."""
    N = U.shape[0]
    z = np.empty(n_vars(N))
    for k in range(N):
        o = k * (N_X + N_U)
        z[o:o + N_X] = X[k]; z[o + N_X:o + N_X + N_U] = U[k]
    z[N * (N_X + N_U):] = X[N]
    return z


def from_vector(z, N):
    """_vector_to_solution (osqp_rti.py:617-631)."""
    X = np.empty((N + 1, N_X)); U = np.empty((N, N_U))
    for k in range(N):
        o = k * (N_X + N_U)
        X[k] = z[o:o + N_X]; U[k] = z[o + N_X:o + N_X + N_U]
    X[N] = z[N * (N_X + N_U):]
    return X, U


def initial_guess(x0, x_target, N):
    """OSQPRTIMPC.initialize (osqp_rti.py:403-452): linear interpolation X, hover U."""
    X = np.array([(1 - k / N) * x0 + (k / N) * x_target for k in range(N + 1)])
    U = np.zeros((N, N_U)); U[:, 0] = x0[0] * G_RTI
    return X, U
