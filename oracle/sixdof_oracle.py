"""6-DoF GP-MPC rollout restatement (TEST INFRASTRUCTURE ONLY) -- BASELINE configs[4].

The reference's 6-DoF closed loop is ``GPMPC.solve`` (src/mpc/gp_mpc.py:229-369)
over the 14-state rocket of src/dynamics/rocket_6dof.py, whose physics lives in
the absent ``simdyn``.  This module restates what the reference spells out and
pins the rest as documented choices:

* dynamics f(x, u): nominal_mpc.py:163-203 (state [m, r_I, v_I, q_BI (w,x,y,z),
  w_B]; C_IB of :176-181; m' = -alpha |u|; v' = C_IB u / m + g_I; q' =
  0.5 Omega(w) q; w' = J^-1 (r_T x u - w x J w)), parameters of
  Rocket6DoFConfig (rocket_6dof.py:36-84: J = diag(0.02, 1, 1) 0.168,
  r_T = (-0.25, 0, 0), g_I = (-1, 0, 0), alpha = 1 / (I_sp g0) = 1/30);
* plant step: RK4 (discretization.py:229-252) + quaternion normalisation
  (rocket_6dof.py:371-387); linearisation A_d = I + A_c dt, B_d = B_c dt with
  the analytic continuous Jacobians (rocket_6dof.py:427-459);
* truth = plant + the aero-drag dispersion on the velocity
  (dispersion.py:349-360) and a -0.05 w rate damping (the residuals of the
  config-5 training generator), evaluated at the pre-step state;
* GP means: the FITC posterior mean K*u L_uu^-T alpha by default; the
  reference's as-written K*u alpha (sparse_gp.py:280-283) is the
  ``corrected=False`` flag -- its magnitudes off the training data (|d_w| ~ 10
  at the hover guess) make the first QP primal infeasible for most rollouts;
* one control step = one pass of GPMPC.solve: forward simulation of the
  warm-start controls with the GP mean (gp_mpc.py:258-281, hover guess
  [0, 0, m g0] of :271-275 on the first call), linearisation and
  c_k = [.., d_v dt, .., d_w dt] at the simulated points (:299-320), the QP
  subproblem in deviation variables (:394-460) with its QCQP constraints made
  linear -- thrust ball -> box [-T_max, T_max]^3, |u| >= T_min linearised at
  U_nom, glideslope cone -> 4 half-planes (stages 1..N-1), trust balls -> boxes
  sqrt(10) / sqrt(5) -- solved by the OSQP-0.6 restatement (admm_ref) with
  osqp_rti.py's settings, warm start dz = 0 with OSQP's persistent rho / y;
  X_pred + dX, U_pred + dU returned; the plan is kept unshifted as the next
  warm start (:358-359); a solve without a solution -> DIVERGENCE.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

NX, NU = 14, 3
ALPHA = 1.0 / 30.0
J_DIAG = np.array([0.02, 1.0, 1.0]) * 0.168
R_T = np.array([-0.25, 0.0, 0.0])
G_I = np.array([-1.0, 0.0, 0.0])
G0 = 1.0
# Rocket6DoFConfig defaults as one parameter set; every dynamics function takes an
# optional ``rk`` of this shape (rocket_6dof.py:36-84)
DEFAULT_ROCKET = dict(J=J_DIAG, r_T=R_T, g_I=G_I, alpha=ALPHA, g0=G0)


def rocket_params(J=None, r_T=None, g_I=None, I_sp=30.0, g0=1.0):
    """A parameter set for a Rocket6DoFConfig.  J: the diagonal of a diagonal J_B, or
    the 3 x 3 tensor (rocket_6dof.py:44, 77-78: any matrix).  A full tensor adds
    ``Jf`` and its inverse ``Ji``: w' = Ji (r_T x u - w x Jf w), nominal_mpc.py:196-199's
    ca.solve(J, .) as the host mirror (dynamics/rocket_6dof.py) states it; a diagonal
    3 x 3 tensor is its diagonal."""
    J = np.asarray(J_DIAG if J is None else J, float)
    rk = dict(r_T=np.asarray(R_T if r_T is None else r_T, float),
              g_I=np.asarray(G_I if g_I is None else g_I, float), alpha=1.0 / (I_sp * g0), g0=float(g0))
    if J.ndim == 2 and np.any(J - np.diag(np.diag(J))):
        rk.update(J=np.diag(J).copy(), Jf=J.copy(), Ji=np.linalg.inv(J))
    else:
        rk["J"] = np.diag(J).copy() if J.ndim == 2 else J
    return rk
T_MIN, T_MAX = 0.5, 5.0                 # ConstraintParams (constraints.py:35-50)
TAN_GS = np.tan(np.deg2rad(30.0))       # gamma_gs 30 deg
TRUST_X, TRUST_U = np.sqrt(10.0), np.sqrt(5.0)   # gp_mpc.py:432-435
Q_DIAG = np.array([0.0, 10, 10, 10, 1, 1, 1, 0, 5, 5, 0, 0.1, 0.1, 0.1])  # CostWeights (cost_functions.py:75-98)
R_DIAG = np.full(3, 0.01)
P_SCALE = 10.0


def dcm_ib(q):
    """C_IB of nominal_mpc.py:176-181 (body -> inertial)."""
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def f(x, u, rk=None):
    """nominal_mpc.py:163-203."""
    rk = rk or DEFAULT_ROCKET
    m, v, q, w = x[0], x[4:7], x[7:11], x[11:14]
    tm = np.sqrt(u @ u)
    out = np.empty(NX)
    out[0] = -rk["alpha"] * tm
    out[1:4] = v
    out[4:7] = dcm_ib(q) @ u / m + rk["g_I"]
    qv = q[1:4]
    out[7] = 0.5 * -(w @ qv)
    out[8:11] = 0.5 * (q[0] * w + np.cross(w, qv))
    torque = np.cross(rk["r_T"], u)
    if "Jf" in rk:   # a full inertia tensor
        out[11:14] = rk["Ji"] @ (torque - np.cross(w, rk["Jf"] @ w))
        return out
    jw = rk["J"] * w
    out[11:14] = (torque - np.cross(w, jw)) / rk["J"]
    return out


def step(x, u, dt, rk=None):
    """RK4 (discretization.py:229-252) + quaternion normalisation (rocket_6dof.py:371-387)."""
    k1 = f(x, u, rk)
    k2 = f(x + dt * k1 / 2, u, rk)
    k3 = f(x + dt * k2 / 2, u, rk)
    k4 = f(x + dt * k3, u, rk)
    xn = x + (dt / 6) * (k1 + 2 * k2 + 2 * k3 + k4)
    xn[7:11] = xn[7:11] / np.sqrt(xn[7:11] @ xn[7:11])
    return xn


def jacobians(x, u, rk=None):
    """Analytic A_c = df/dx (14 x 14), B_c = df/du (14 x 3) of f."""
    rk = rk or DEFAULT_ROCKET
    m, q, w = x[0], x[7:11], x[11:14]
    qw, qx, qy, qz = q
    u0, u1, u2 = u
    A = np.zeros((NX, NX)); B = np.zeros((NX, NU))
    tm = np.sqrt(u @ u)
    B[0] = -rk["alpha"] * u / tm
    A[1:4, 4:7] = np.eye(3)
    C = dcm_ib(q)
    A[4:7, 0] = -(C @ u) / (m * m)
    dCu = np.array([  # d(C u)/d(w, x, y, z)
        [-2 * qz * u1 + 2 * qy * u2, 2 * qy * u1 + 2 * qz * u2, -4 * qy * u0 + 2 * qx * u1 + 2 * qw * u2,
         -4 * qz * u0 - 2 * qw * u1 + 2 * qx * u2],
        [2 * qz * u0 - 2 * qx * u2, 2 * qy * u0 - 4 * qx * u1 - 2 * qw * u2, 2 * qx * u0 + 2 * qz * u2,
         2 * qw * u0 - 4 * qz * u1 + 2 * qy * u2],
        [-2 * qy * u0 + 2 * qx * u1, 2 * qz * u0 + 2 * qw * u1 - 4 * qx * u2, -2 * qw * u0 + 2 * qz * u1 - 4 * qy * u2,
         2 * qx * u0 + 2 * qy * u1]])
    A[4:7, 7:11] = dCu / m
    B[4:7] = C / m
    wx, wy, wz = w
    A[7:11, 7:11] = 0.5 * np.array([[0, -wx, -wy, -wz], [wx, 0, -wz, wy], [wy, wz, 0, -wx], [wz, -wy, wx, 0]])
    A[7, 11:14] = -0.5 * q[1:4]
    A[8:11, 11:14] = 0.5 * np.array([[qw, qz, -qy], [-qz, qw, qx], [qy, -qx, qw]])
    rx, ry, rz = rk["r_T"]
    Rx = np.array([[0, -rz, ry], [rz, 0, -rx], [-ry, rx, 0]])
    if "Jf" in rk:   # d/dw Ji (-w x Jf w) = Ji ([Jf w]x - [w]x Jf); B: Ji [r_T]x
        def skew(a):
            return np.array([[0.0, -a[2], a[1]], [a[2], 0.0, -a[0]], [-a[1], a[0], 0.0]])
        A[11:14, 11:14] = rk["Ji"] @ (skew(rk["Jf"] @ w) - skew(w) @ rk["Jf"])
        B[11:14] = rk["Ji"] @ Rx
        return A, B
    j1, j2, j3 = rk["J"]
    A[11, 11:14] = -(j3 - j2) / j1 * np.array([0, wz, wy])
    A[12, 11:14] = -(j1 - j3) / j2 * np.array([wz, 0, wx])
    A[13, 11:14] = -(j2 - j1) / j3 * np.array([wy, wx, 0])
    B[11:14] = Rx / rk["J"][:, None]
    return A, B


def linearize(x, u, dt, rk=None):
    """rocket_6dof.py:451-457."""
    A, B = jacobians(x, u, rk)
    return np.eye(NX) + A * dt, B * dt


def drag(x):
    """dispersion.py:349-360: rho 0.02, Cd = A = 1, applied when |v| > 1."""
    v = x[4:7]
    sp_ = np.sqrt(v @ v)
    if sp_ > 1.0:
        return -(0.5 * 0.02 * sp_ ** 2) / x[0] * (v / sp_)
    return np.zeros(3)


def truth_step(x, u, dt, rk=None):
    """The rollout plant: nominal step + the residual the config-5 GP is trained on
    (data.synthetic_6dof_training_data): the drag dispersion on v and a rate
    damping -0.05 w on w-dot, both at the pre-step state."""
    xn = step(x, u, dt, rk)
    xn[4:7] += drag(x) * dt
    xn[11:14] += -0.05 * x[11:14] * dt
    return xn


def fitc_mean(st, Zq, corrected=True):
    """FITC predictive mean.  As written (sparse_gp.py:280-283) it is
    K*u alpha; the FITC posterior mean is K*u L_uu^-T alpha (alpha = L_B^-T L_B^-1
    A Lambda^-1 y in the whitened basis of sparse_gp.py:200-210)."""
    from scipy.linalg import solve_triangular
    from . import gp_oracle
    Ksu = gp_oracle.gram("se_ard", np.atleast_2d(Zq), st["Zi"], st["sigma2"], st["ls"])
    if corrected:
        if "beta" not in st:
            st["beta"] = solve_triangular(st["Luu"].T, st["alpha"], lower=False)
        a = st["beta"]
    else:
        a = st["alpha"]
    return (Ksu @ a) * st["y_std"] + st["y_mean"]


def gp_mean(gpv, gpw, x, u, corrected=True):
    """StructuredRocketGP.predict means (structured_gp.py:225-268) of the FITC pair."""
    from . import gp_oracle
    mv = fitc_mean(gpv, gp_oracle.features_translational(x[None], u[None]), corrected)
    mw = fitc_mean(gpw, gp_oracle.features_rotational(x[None], u[None]), corrected)
    return mv[0], mw[0]


def qp_pattern(N):
    """CSR pattern of the 6-DoF QP (row order: x0, dynamics, bounds, thrust, glideslope)."""
    n = N * (NX + NU) + NX
    rows = []
    for i in range(NX):
        rows.append([i])
    for k in range(N):
        o, on = k * (NX + NU), (k + 1) * (NX + NU)
        for i in range(NX):
            rows.append(list(range(o, o + NX + NU)) + [on + i])
    for j in range(n):
        rows.append([j])
    for k in range(N):
        o = k * (NX + NU) + NX
        rows.append([o, o + 1, o + 2])
    for k in range(1, N):
        o = k * (NX + NU)
        for c in (2, 3):
            rows.append([o + 1, o + c])
            rows.append([o + 1, o + c])
    rp = np.cumsum([0] + [len(r) for r in rows])
    ci = np.concatenate(rows)
    return n, len(rows), rp.astype(np.int32), ci.astype(np.int32)


def default_problem():
    """GPMPC's problem data with the reference defaults: CostWeights Q / R / P
    (cost_functions.py:39-105), ConstraintParams T_min, T_max, gamma_gs
    (constraints.py:35-50), trust radii^2 10 / 5 (gp_mpc.py:432-435)."""
    return dict(Q=Q_DIAG.copy(), P=Q_DIAG * P_SCALE, R=R_DIAG.copy(), t_min=T_MIN, t_max=T_MAX,
                tan_gs=TAN_GS, trust_x2=10.0, trust_u2=5.0)


def build_qp(Xn, Un, gm, x_ref, dt, x0=None, prob=None, rk=None, u_ref=None):
    """QP of gp_mpc.py:394-460 around (Xn, Un) with c_k = GP mean dt (gp_mpc.py:309-314)
    in deviation variables z = [dx_0, du_0, ..., dx_N]; the cost's X_ref is x_ref
    (one state for every stage, or (N+1, 14)), its U_ref u_ref (N, 3; None = 0)
    (gp_mpc.py:442-453).  x0 rows: dx_0 = x0 - X_nom[0] (gp_mpc.py:402; 0 when
    X_nom[0] = x0).  Returns Pdiag, q, A (CSR), l, u."""
    pr = prob or default_problem()
    N = Un.shape[0]
    x_ref = np.asarray(x_ref, float)
    Xr = np.broadcast_to(x_ref, (N + 1, NX)) if x_ref.ndim == 1 else x_ref
    Ur = np.zeros((N, NU)) if u_ref is None else np.asarray(u_ref, float)
    n, m, rp, ci = qp_pattern(N)
    val = np.zeros(rp[-1]); l = np.zeros(m); u = np.zeros(m)
    Pd = np.zeros(n); q = np.zeros(n)
    tr_x, tr_u = np.sqrt(pr["trust_x2"]), np.sqrt(pr["trust_u2"])
    for k in range(N + 1):
        o = k * (NX + NU)
        w = pr["P"] if k == N else pr["Q"]
        Pd[o:o + NX] = w
        q[o:o + NX] = w * (Xn[k] - Xr[k])
        if k < N:
            Pd[o + NX:o + NX + NU] = pr["R"]
            q[o + NX:o + NX + NU] = pr["R"] * (Un[k] - Ur[k])
    r = 0
    for i in range(NX):
        val[rp[r]] = 1.0
        l[r] = u[r] = 0.0 if x0 is None else x0[i] - Xn[0, i]
        r += 1
    for k in range(N):
        Ad, Bd = linearize(Xn[k], Un[k], dt, rk)
        c = np.zeros(NX)
        c[4:7] = gm[k, :3] * dt
        c[11:14] = gm[k, 3:] * dt
        for i in range(NX):
            a = rp[r]
            val[a:a + NX] = -Ad[i]
            val[a + NX:a + NX + NU] = -Bd[i]
            val[a + NX + NU] = 1.0
            l[r] = u[r] = c[i]
            r += 1
    for j in range(n):
        k, i = divmod(j, NX + NU)
        val[rp[r]] = 1.0
        if i < NX:
            l[r], u[r] = -tr_x, tr_x
        else:
            ub = Un[k, i - NX]
            l[r] = max(-tr_u, -pr["t_max"] - ub)
            u[r] = min(tr_u, pr["t_max"] - ub)
        r += 1
    for k in range(N):
        ub = Un[k]
        tm = np.sqrt(ub @ ub)
        val[rp[r]:rp[r] + 3] = ub / tm
        l[r], u[r] = pr["t_min"] - tm, np.inf
        r += 1
    tg = pr["tan_gs"]
    for k in range(1, N):
        rx, ry, rz = Xn[k, 1:4]
        for c, rc in ((2, ry), (3, rz)):
            a = rp[r]
            val[a:a + 2] = (tg, -1.0); l[r], u[r] = -(tg * rx - rc), np.inf; r += 1
            a = rp[r]
            val[a:a + 2] = (tg, 1.0); l[r], u[r] = -(tg * rx + rc), np.inf; r += 1
    A = sp.csr_matrix((val, ci, rp), shape=(m, n))
    return Pd, q, A, l, u


def incremental_target(x, upright=False):
    """monte_carlo.py:497-500 on the 14-state layout: x copied (attitude and rates
    kept), v = 0, altitude - 2 m with a 0.5 m floor; ``upright`` also sets
    q = (1, 0, 0, 0), omega = 0 (the fleet6 ``upright_target`` option)."""
    t = x.copy()
    t[4:7] = 0.0
    t[1] = max(0.5, x[1] - 2.0)
    if upright:
        t[7:11] = (1.0, 0.0, 0.0, 0.0)
        t[11:14] = 0.0
    return t


def hover_guess(x, N, g0=G0):
    """gp_mpc.py:271-275: [0, 0, m g0] (thrust on the body z axis, as written) at
    every stage.  As written the loop reads X_pred[k, 0] before the forward
    simulation has filled it, so stages k >= 1 get zero thrust; zero thrust has
    no linearisation of the thrust-magnitude rows (u / |u|), so the evident
    intent m0 g0 is used at every stage."""
    U = np.zeros((N, NU))
    U[:, 2] = x[0] * g0
    return U


def new_rollout(x0, N=30):
    from . import admm_ref
    n, m, _, _ = qp_pattern(N)
    rec = np.zeros(16)
    rec[4:11] = x0[:7]
    rec[13] = x0[0]
    return dict(x=np.array(x0, float), U=hover_guess(x0, N), y=np.zeros(m),
                rho=admm_ref.default_settings().rho, rec=rec, X=None)


def rollout_step(gpv, gpw, S, dt=0.1, max_steps=300, qp_settings=None, corrected=True, upright=False, rk=None):
    """One control step of the 6-DoF rollout (monte_carlo.py:455-537 termination
    rules on the first seven states; one GPMPC.solve pass as the module header)."""
    from . import admm_ref, mc_oracle
    x = S["x"].copy(); U = S["U"].copy(); rec = S["rec"].copy()
    N = U.shape[0]
    out = dict(S, x=x, U=U, rec=rec, y=S["y"].copy())
    if rec[0] != 0:
        return out, None
    m0 = rec[13]
    o = mc_oracle.TIMEOUT if rec[1] >= max_steps else mc_oracle.pre_step_outcome(x[:7], m0)
    if o == 0 and (np.any(np.abs(x) > 1e6) or np.any(np.isnan(x))):
        o = mc_oracle.DIVERGENCE
    if o:
        rec[0] = o; rec[2] = m0 - x[0]; rec[4:11] = x[:7]
        return out, None
    # forward simulation with the GP mean (gp_mpc.py:258-281)
    X = np.zeros((N + 1, NX)); X[0] = x
    gm = np.zeros((N, 6))
    for k in range(N):
        dv, dw = gp_mean(gpv, gpw, X[k], U[k], corrected)
        gm[k, :3], gm[k, 3:] = dv, dw
        X[k + 1] = step(X[k], U[k], dt, rk)
        X[k + 1, 4:7] += dv * dt
        X[k + 1, 11:14] += dw * dt
    Pd, q, A, l, u = build_qp(X, U, gm, incremental_target(x, upright), dt, rk=rk)
    qp = admm_ref.RefQP(len(out["y"]), settings=qp_settings)
    qp.y = out["y"]; qp.rho = np.array([out["rho"]])
    try:
        r = qp.solve(Pd, q, A, l, u, np.zeros(Pd.size))
    except RuntimeError:
        rec[0] = mc_oracle.DIVERGENCE; rec[14] = -100; rec[2] = m0 - x[0]; rec[4:11] = x[:7]
        return out, (0, -100)
    if r["status"] not in (1, 2, -2):
        rec[0] = mc_oracle.DIVERGENCE; rec[14] = r["status"]; rec[2] = m0 - x[0]; rec[4:11] = x[:7]
        return out, (r["iter"], r["status"])
    z = r["x"]
    Xo = X + np.array([z[k * (NX + NU):k * (NX + NU) + NX] for k in range(N + 1)])
    Uo = U + np.array([z[k * (NX + NU) + NX:(k + 1) * (NX + NU)] for k in range(N)])
    xn = truth_step(x, Uo[0], dt, rk)
    out.update(x=xn, U=Uo, X=Xo, X_pred=X, y=qp.y, rho=float(qp.rho[0]), gm=gm)
    rec[1] += 1; rec[2] = m0 - xn[0]; rec[3] = rec[1] * dt; rec[4:11] = xn[:7]
    rec[11] += r["iter"]; rec[12] += r["status"] == 1; rec[14] = r["status"]; rec[15] = qp.rho[0]
    return out, (r["iter"], r["status"])


def initial_condition(seed):
    """6-DoF rollout start: the run_experiments 3-DoF draw (mc_oracle) for
    [m, r, v], then a tilt of N(0, 5 deg) about a random horizontal body axis,
    at rest in rotation."""
    from . import mc_oracle
    x7 = mc_oracle.sample_initial_condition(seed)
    rs = np.random.RandomState(seed + 7919)
    ang = np.deg2rad(5.0) * rs.randn()
    phi = 2 * np.pi * rs.rand()
    ax = np.array([0.0, np.cos(phi), np.sin(phi)])
    x = np.zeros(NX)
    x[:7] = x7
    x[7] = np.cos(ang / 2); x[8:11] = ax * np.sin(ang / 2)
    return x


def gpmpc_solve(gpv, gpw, S, x0, x_target, max_sqp_iter=10, sqp_tol=1e-4, dt=0.1, qp_settings=None,
                corrected=True, use_gp=True, prob=None, rk=None, X_ref=None, U_ref=None):
    """GPMPC.solve (gp_mpc.py:229-369) on the 14-state rocket with the QP made
    linear as in build_qp and solved by the OSQP-0.6 restatement:

    * X_pred[0] = x0; the controls are the warm start S["U"] (the previous
      plan, unshifted, :266-267 / :358-359; the caller puts hover_guess there on
      the first call); forward simulation with the GP mean (:277-281);
    * up to max_sqp_iter passes (:299-353): GP means and Jacobians at
      (X_pred[k], U_pred[k]) (the first pass reuses the simulation's means,
      which are the same calls), QP around (X_pred, U_pred), plan = X_pred +
      dX, U_pred + dU; a QP without a solution returns the nominal (:478-482),
      so that pass changes nothing and the loop stops as converged; stop when
      max|X_new - X_pred| and max|U_new - U_pred| are both < sqp_tol;
    * the ADMM keeps OSQP's persistent rho / scaled y across passes and calls;
      a failed pass leaves them as they were (the device writes them back only
      with a solution).

    * the QP cost tracks X_ref ((N+1, 14), default x_target on every stage) and
      U_ref ((N, 3), default 0) (:442-453); ``rk``: the rocket (rocket_params).

    S: dict(U (N, 3), y (m,), rho).  Returns dict(X, U, y, rho, passes,
    converged, qp_status, qp_iters, n_solved, X_pred (of the first pass), gm)."""
    from . import admm_ref
    U = np.array(S["U"], float)
    N = U.shape[0]
    x0 = np.asarray(x0, float)
    X = np.zeros((N + 1, NX)); X[0] = x0
    gm = np.zeros((N, 6))
    for k in range(N):
        if use_gp:
            dv, dw = gp_mean(gpv, gpw, X[k], U[k], corrected)
            gm[k, :3], gm[k, 3:] = dv, dw
        X[k + 1] = step(X[k], U[k], dt, rk)
        X[k + 1, 4:7] += gm[k, :3] * dt
        X[k + 1, 11:14] += gm[k, 3:] * dt
    X_first = X.copy()
    x_ref = x_target if X_ref is None else np.asarray(X_ref, float)
    n, m, _, _ = qp_pattern(N)
    qp = admm_ref.RefQP(m, settings=qp_settings)
    qp.y = np.array(S["y"], float); qp.rho = np.array([float(S["rho"])])
    passes, qit, qst, conv, nsolved = 0, 0, -10, False, 0
    for it in range(max_sqp_iter):
        if it > 0:
            gm = np.zeros((N, 6))
            if use_gp:
                for k in range(N):
                    dv, dw = gp_mean(gpv, gpw, X[k], U[k], corrected)
                    gm[k, :3], gm[k, 3:] = dv, dw
        Pd, q, A, l, u = build_qp(X, U, gm, x_ref, dt, x0=x0, prob=prob, rk=rk, u_ref=U_ref)
        y_keep, rho_keep = qp.y.copy(), qp.rho.copy()
        try:
            r = qp.solve(Pd, q, A, l, u, np.zeros(Pd.size))
            st, nit = r["status"], r["iter"]
        except RuntimeError:
            r, st, nit = None, -100, 0
        passes += 1; qit += nit; qst = st
        nsolved += st == 1
        if st in (1, 2, -2):
            z = r["x"]
            Xn = X + np.array([z[k * (NX + NU):k * (NX + NU) + NX] for k in range(N + 1)])
            Un = U + np.array([z[k * (NX + NU) + NX:(k + 1) * (NX + NU)] for k in range(N)])
        else:
            qp.y, qp.rho = y_keep, rho_keep
            Xn, Un = X, U
        dx, du = np.max(np.abs(Xn - X)), np.max(np.abs(Un - U))
        X, U = Xn, Un
        if dx < sqp_tol and du < sqp_tol:
            conv = True
            break
    return dict(X=X, U=U, y=qp.y, rho=float(qp.rho[0]), passes=passes, converged=conv, qp_status=qst,
                qp_iters=qit, n_solved=nsolved, X_pred=X_first, gm=gm)


def solution_cost(X, U, x_target, prob=None, U_ref=None):
    """The QP subproblem's objective at the returned plan (gp_mpc.py:447-458;
    x_target: one state or the (N+1, 14) X_ref; U_ref None = 0)."""
    pr = prob or default_problem()
    e = np.asarray(X) - np.asarray(x_target)
    du = np.asarray(U) - (0.0 if U_ref is None else np.asarray(U_ref))
    return float(np.sum(e[:-1] ** 2 * pr["Q"]) + np.sum(du ** 2 * pr["R"])
                 + np.sum(e[-1] ** 2 * pr["P"]))
