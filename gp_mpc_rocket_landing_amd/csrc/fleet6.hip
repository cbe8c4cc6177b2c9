// fleet6.hip -- BASELINE configs[4]: a batch of closed-loop 6-DoF GP-MPC rollouts
// (N = 30, 14 states, the StructuredRocketGP FITC residuals), device-resident.
//
// One control step of rollout b (oracle/sixdof_oracle.py restates it):
//   1. k_r6_predict  (256 threads / rollout): Monte-Carlo termination rules
//      (monte_carlo.py:455-488 on the first seven states), then GPMPC.solve's
//      forward simulation (gp_mpc.py:258-281): X[k+1] = RK4(X[k], U[k])
//      (discretization.py:229-252, quaternion normalised, rocket_6dof.py:371-387)
//      + [.., d_v dt, .., d_w dt] with the FITC means of the two GPs at
//      (X[k], U[k]) (structured_gp.py:225-268; sparse_gp.py:255-305 mean as
//      written, K*u alpha) -- the 2 x M kernel rows of a point are spread over
//      the workgroup and reduced; the 30 points are sequential.  The mean is the
//      FITC posterior mean K*u L_uu^-T alpha (SURVEY D1 fixed; the reference's
//      K*u alpha behind fitc_mean_as_written).
//   2. k_r6_control  (512 threads / rollout): the QP subproblem of
//      gp_mpc.py:394-460 in deviation variables z = [dx_0, du_0, .., dx_30]
//      (n = 524): x0 + dynamics equalities with A_d = I + A_c dt, B_d = B_c dt
//      (rocket_6dof.py:427-459, analytic Jacobians) and c_k = GP mean dt; the
//      QCQP rows made linear (thrust box, |u| >= T_min at U_nom, glideslope
//      half-planes, trust-region boxes; m = 1104); OSQP-0.6 ADMM (Ruiz scaling,
//      rho vector, adaptive rho, termination every 25) on the reduced KKT
//      matrix, which is block tridiagonal in the 31 stage blocks [x_k, u_k]:
//      S_0 = D_0, S_k+1 = D_k+1 - C_k S_k^-1 C_k^T with S_k^-1 formed by
//      Gauss-Jordan in LDS; each iteration's solve is a forward chain
//      (y_k+1 -= G_k y_k, G_k = C_k S_k^-1, one DPP row), the 31 diagonal
//      products u_k = S_k^-1 y_k in parallel, and a backward chain (x_k = u_k -
//      G_k^T x_k+1, two DPP rows); the chains keep their vector in registers
//      (r6_solve).  Then the plan X + dX, U + dU (kept unshifted
//      as the next warm start, gp_mpc.py:358-359), the truth plant step (RK4
//      + the drag dispersion of dispersion.py:349-360 and the -0.05 w rate
//      damping the config-5 GP is trained on) and the records.
// Ownership: item j = tid + 512 h (h = 0, 1) of thread tid: variable j < 524
// (+ its bound row; general row tid < 146 rides on slot 0), else equality row
// j - 524 < 434.  At 1024 threads (one item each) a lane had 128 VGPRs and the
// ADMM loop reloaded 222 spilled registers from scratch; two items per lane at
// 256 VGPRs is the same register file without them.  The 14 x 17 dynamics
// block of each equality row lives in its owner's registers, a column copy in
// the variable owner's; only the factor and the cross-thread vectors are LDS.
#include "internal.h"
#include "gemm.h"
#include "qp.h"
#include <vector>

#define R6_NX 14
#define R6_NU 3
#define R6_SZ 17
// the horizon N is a compile-time constant of the kernels (fully unrolled chains,
// LDS layout): fleet6_n.h is compiled once per supported horizon, in namespaces
// r6n20 (GPMPCConfig's N = 20, gp_mpc.py:110 / nominal_mpc.py:47) and r6n30
// (BASELINE configs[4]); the C-ABI dispatches on the config's horizon
#define R6_T 512                              // two items (variables / rows) per thread
#define R6_TRI 153                            // packed lower 17 x 17
#define R6_PT 512                             // predict threads (7 kernel-row waves + the RK4 wave)
#define R6_FOR_H _Pragma("unroll") for (int h = 0; h < 2; ++h)

// ConstraintParams (constraints.py:35-50), CostWeights (cost_functions.py:39-98),
// gp_mpc.py trust regions (:432-435)
#define R6_T_MIN 0.5
#define R6_T_MAX 5.0

// the rocket (Rocket6DoFConfig, rocket_6dof.py:36-84): diagonal J_B, thrust point
// r_T_B, gravity g_I, alpha = 1 / (I_sp g0), g0 -- kernel arguments (uniform values)
struct R6Rocket {
  double J[3], rT[3], gI[3], alpha, g0;
};

struct R6Impl;  // the kernels of one horizon (fleet6_n.h), below
struct gpmpc_rollout6 {
  gpmpc_ctx *ctx = nullptr;
  GpView gv{}, gw{};
  bool exact = false;  // the GP pair is exact (mean K* alpha over the training rows)
  gpmpc_rollout6_config cfg{};
  const R6Impl *impl = nullptr;
  int B = 0, N = 0, M = 0;  // batch, horizon, QP rows
  DevBuf x, U, Xp, gm, Xo, ysc, rho, rec, lin, pending;
  DevBuf betav, betaw;  // (L_uu^-T alpha)^T of each GP, 3 x M
  DevBuf prm;           // problem data (R6_PRM doubles, r6_prm layout)
  DevBuf xt, ut, done, passes, qit, qst, xin;  // GPMPC.solve mode: X_ref (B x (N+1) x 14), U_ref (B x N x 3)
};

// problem data in device memory (read per thread with a dynamic index, so not a
// by-value kernel argument): Q (14), P (14), R (3), T_min, T_max, tan gamma_gs,
// trust x / u radii
#define R6_PQ 0
#define R6_PP 14
#define R6_PR 28
#define R6_PTMIN 31
#define R6_PTMAX 32
#define R6_PTAN 33
#define R6_PTRX 34
#define R6_PTRU 35
#define R6_PRM 36

extern "C" void gpmpc_rollout6_default_config(gpmpc_rollout6_config *c) {
  c->horizon = 30;     // BASELINE configs[4]: N = 30
  c->dt = 0.1;
  c->max_steps = 300;
  gpmpc_qp_default_settings(&c->qp);   // osqp_rti.py:54-60 settings, as the 3-DoF path
  c->fitc_mean_as_written = 0;         // FITC posterior mean (SURVEY D1 fixed, flag 1 = as written)
  // CostWeights (cost_functions.py:39-98): Q = diag(w_mass, w_pos x3, w_vel x3, 0, w_att x2, 0,
  // w_omega x3), R = w_thrust I, P = terminal_weight Q
  const double q[R6_NX] = {0.0, 10, 10, 10, 1, 1, 1, 0, 5, 5, 0, 0.1, 0.1, 0.1};
  for (int i = 0; i < R6_NX; ++i) { c->q_diag[i] = q[i]; c->p_diag[i] = 10.0 * q[i]; }
  for (int i = 0; i < R6_NU; ++i) c->r_diag[i] = 0.01;
  c->t_min = R6_T_MIN;                 // ConstraintParams (constraints.py:35-50)
  c->t_max = R6_T_MAX;
  c->tan_gamma_gs = 0.5773502691896257;  // np.tan(np.deg2rad(30.0))
  c->trust_x2 = 10.0;                  // gp_mpc.py:432-435
  c->trust_u2 = 5.0;
  c->use_gp_mean = 1;
  c->upright_target = 0;
  // Rocket6DoFConfig defaults (rocket_6dof.py:36-84)
  c->rocket_j[0] = 0.02 * 0.168; c->rocket_j[1] = 1.0 * 0.168; c->rocket_j[2] = 1.0 * 0.168;
  c->rocket_r_t[0] = -0.25; c->rocket_r_t[1] = 0.0; c->rocket_r_t[2] = 0.0;
  c->rocket_g_i[0] = -1.0; c->rocket_g_i[1] = 0.0; c->rocket_g_i[2] = 0.0;
  c->rocket_alpha = 1.0 / (30.0 * 1.0);  // I_sp 30, g0 1
  c->rocket_g0 = 1.0;
}

// beta^T = alpha^T L_uu^-1 (3 x M): the FITC posterior mean is K*u beta.
// W = L_uu^-1 (lower, row-major, ld M) is the fit's first M rows of core.W; the
// product is one FP64-MFMA NN GEMM (a thread-per-column loop took 614 us at M = 2000)

// ---------------------------------------------------------------------------
// dynamics (nominal_mpc.py:163-203)
__device__ __forceinline__ void r6_dcm(const double *q, double C[3][3]) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  C[0][0] = 1 - 2 * (y * y + z * z); C[0][1] = 2 * (x * y - w * z); C[0][2] = 2 * (x * z + w * y);
  C[1][0] = 2 * (x * y + w * z); C[1][1] = 1 - 2 * (x * x + z * z); C[1][2] = 2 * (y * z - w * x);
  C[2][0] = 2 * (x * z - w * y); C[2][1] = 2 * (y * z + w * x); C[2][2] = 1 - 2 * (x * x + y * y);
}

__device__ void r6_f(const R6Rocket &rk, const double *x, const double *u, double *o) {
  const double m = x[0];
  const double tm = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
  double C[3][3];
  r6_dcm(x + 7, C);
  o[0] = -rk.alpha * tm;
  o[1] = x[4]; o[2] = x[5]; o[3] = x[6];
  for (int i = 0; i < 3; ++i) o[4 + i] = (C[i][0] * u[0] + C[i][1] * u[1] + C[i][2] * u[2]) / m + rk.gI[i];
  const double qw = x[7], qx = x[8], qy = x[9], qz = x[10], wx = x[11], wy = x[12], wz = x[13];
  o[7] = 0.5 * -((wx * qx + wy * qy) + wz * qz);
  o[8] = 0.5 * (qw * wx + (wy * qz - wz * qy));
  o[9] = 0.5 * (qw * wy + (wz * qx - wx * qz));
  o[10] = 0.5 * (qw * wz + (wx * qy - wy * qx));
  // r_T x u; w x J w
  const double *rT = rk.rT, *J = rk.J;
  const double tq[3] = {rT[1] * u[2] - rT[2] * u[1], rT[2] * u[0] - rT[0] * u[2], rT[0] * u[1] - rT[1] * u[0]};
  const double jw[3] = {J[0] * wx, J[1] * wy, J[2] * wz};
  const double cx[3] = {wy * jw[2] - wz * jw[1], wz * jw[0] - wx * jw[2], wx * jw[1] - wy * jw[0]};
  for (int i = 0; i < 3; ++i) o[11 + i] = (tq[i] - cx[i]) / J[i];
}

// RK4 (discretization.py:229-252) + quaternion normalisation (rocket_6dof.py:371-387)
__device__ void r6_step(const R6Rocket &rk, const double *x, const double *u, double dt, double *xn) {
  double k1[R6_NX], k2[R6_NX], k3[R6_NX], k4[R6_NX], t[R6_NX];
  r6_f(rk, x, u, k1);
  for (int i = 0; i < R6_NX; ++i) t[i] = x[i] + dt * k1[i] / 2;
  r6_f(rk, t, u, k2);
  for (int i = 0; i < R6_NX; ++i) t[i] = x[i] + dt * k2[i] / 2;
  r6_f(rk, t, u, k3);
  for (int i = 0; i < R6_NX; ++i) t[i] = x[i] + dt * k3[i];
  r6_f(rk, t, u, k4);
  for (int i = 0; i < R6_NX; ++i) xn[i] = x[i] + (dt / 6) * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
  const double nq = sqrt(xn[7] * xn[7] + xn[8] * xn[8] + xn[9] * xn[9] + xn[10] * xn[10]);
  for (int i = 7; i < 11; ++i) xn[i] = xn[i] / nq;
}

// -[A_d | B_d] (A_d = I + A_c dt, B_d = B_c dt) into a zeroed 14 x 17 row-major block
__device__ void r6_neg_lin(const R6Rocket &rk, const double *x, const double *u, double dt, double *blk) {
  auto set = [&](int i, int j, double v) { blk[i * R6_SZ + j] = v; };
  const double m = x[0], qw = x[7], qx = x[8], qy = x[9], qz = x[10], wx = x[11], wy = x[12], wz = x[13];
  const double u0 = u[0], u1 = u[1], u2 = u[2];
  const double tm = sqrt(u0 * u0 + u1 * u1 + u2 * u2);
  double C[3][3];
  r6_dcm(x + 7, C);
  for (int i = 0; i < R6_NX; ++i) set(i, i, -(1.0 + 0.0 * dt));
  set(0, 14, -(-rk.alpha * u0 / tm * dt)); set(0, 15, -(-rk.alpha * u1 / tm * dt));
  set(0, 16, -(-rk.alpha * u2 / tm * dt));
  for (int i = 0; i < 3; ++i) set(1 + i, 4 + i, -(1.0 * dt));
  for (int i = 0; i < 3; ++i) {
    const double cu = C[i][0] * u0 + C[i][1] * u1 + C[i][2] * u2;
    set(4 + i, 0, -(-cu / (m * m) * dt));
    for (int j = 0; j < 3; ++j) set(4 + i, 14 + j, -(C[i][j] / m * dt));
  }
  const double dCu[3][4] = {
      {-2 * qz * u1 + 2 * qy * u2, 2 * qy * u1 + 2 * qz * u2, -4 * qy * u0 + 2 * qx * u1 + 2 * qw * u2,
       -4 * qz * u0 - 2 * qw * u1 + 2 * qx * u2},
      {2 * qz * u0 - 2 * qx * u2, 2 * qy * u0 - 4 * qx * u1 - 2 * qw * u2, 2 * qx * u0 + 2 * qz * u2,
       2 * qw * u0 - 4 * qz * u1 + 2 * qy * u2},
      {-2 * qy * u0 + 2 * qx * u1, 2 * qz * u0 + 2 * qw * u1 - 4 * qx * u2,
       -2 * qw * u0 + 2 * qz * u1 - 4 * qy * u2, 2 * qx * u0 + 2 * qy * u1}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) set(4 + i, 7 + j, -(dCu[i][j] / m * dt));
  const double Om[4][4] = {{0, -wx, -wy, -wz}, {wx, 0, -wz, wy}, {wy, wz, 0, -wx}, {wz, -wy, wx, 0}};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) set(7 + i, 7 + j, -((i == j ? 1.0 : 0.0) + 0.5 * Om[i][j] * dt));
  const double Qw[4][3] = {{-qx, -qy, -qz}, {qw, qz, -qy}, {-qz, qw, qx}, {qy, -qx, qw}};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 3; ++j) set(7 + i, 11 + j, -(0.5 * Qw[i][j] * dt));
  const double j1 = rk.J[0], j2 = rk.J[1], j3 = rk.J[2];
  const double Aw[3][3] = {{0, wz, wy}, {wz, 0, wx}, {wy, wx, 0}};
  const double cw[3] = {-(j3 - j2) / j1, -(j1 - j3) / j2, -(j2 - j1) / j3};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) set(11 + i, 11 + j, -((i == j ? 1.0 : 0.0) + cw[i] * Aw[i][j] * dt));
  // B_c omega rows: J^-1 [r_T]x
  const double rx = rk.rT[0], ry = rk.rT[1], rz = rk.rT[2];
  const double Rx[3][3] = {{0, -rz, ry}, {rz, 0, -rx}, {-ry, rx, 0}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) set(11 + i, 14 + j, -(Rx[i][j] / rk.J[i] * dt));
}

// ---------------------------------------------------------------------------
// StructuredRocketGP features (features.py:196-263, :304-356), scaled by the GP's
// lengthscales (the k_scale_rows arithmetic).  The formulas are split over six
// wave-uniform roles, one lane each, so the transcendental chains of a point run
// side by side instead of one after another on one lane:
//   0: v 0-2, 7-11 (velocity, thrust, altitude)    1: v 3, w 0-6, 10 (speeds, rates, thrust)
//   2: v 4, 12, w 11 (density: exp)                3: v 5 (angle of attack: atan2)
//   4: v 6 (sideslip: asin)                        5: w 7-9 (body-frame velocity)
// Each role evaluates its features with the same expressions as the whole set
// would, so the scaled features are the same bits.
#define R6_FEAT_ROLES 6
__device__ __forceinline__ double r6_speed(const double *x) {
  const double vx = x[4], vy = x[5], vz = x[6];
  return sqrt((vx * vx + vy * vy) + vz * vz);
}
__device__ __forceinline__ void r6_body_velocity(const double *x, double *vb) {
  const double vx = x[4], vy = x[5], vz = x[6];
  // body-from-inertial DCM (features.py:265-270)
  const double w = x[7], qx = x[8], qy = x[9], qz = x[10];
  const double Cb[3][3] = {{1 - 2 * (qy * qy + qz * qz), 2 * (qx * qy + w * qz), 2 * (qx * qz - w * qy)},
                           {2 * (qx * qy - w * qz), 1 - 2 * (qx * qx + qz * qz), 2 * (qy * qz + w * qx)},
                           {2 * (qx * qz + w * qy), 2 * (qy * qz - w * qx), 1 - 2 * (qx * qx + qy * qy)}};
  for (int i = 0; i < 3; ++i) vb[i] = (Cb[i][0] * vx + Cb[i][1] * vy) + Cb[i][2] * vz;
}

__device__ void r6_features_role(int role, const double *x, const double *u, const double *lsv,
                                 const double *lsw, double *zv, double *zw) {
  const double qn = 0.5 * 1.225 * 100.0;
  switch (role) {
    case 0: {
      const double tm = sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
      zv[0] = (x[4] / 10.0) / lsv[0]; zv[1] = (x[5] / 10.0) / lsv[1]; zv[2] = (x[6] / 10.0) / lsv[2];
      zv[7] = (u[0] / 10.0) / lsv[7]; zv[8] = (u[1] / 10.0) / lsv[8]; zv[9] = (u[2] / 10.0) / lsv[9];
      zv[10] = (tm / 10.0) / lsv[10]; zv[11] = (x[1] / 100.0) / lsv[11];
      break;
    }
    case 1: {
      const double speed = r6_speed(x);
      const double wxx = x[11], wyy = x[12], wzz = x[13];
      const double wm = sqrt((wxx * wxx + wyy * wyy) + wzz * wzz);
      zv[3] = (speed / 10.0) / lsv[3];
      zw[0] = wxx / lsw[0]; zw[1] = wyy / lsw[1]; zw[2] = wzz / lsw[2]; zw[3] = wm / lsw[3];
      zw[4] = (u[0] / 10.0) / lsw[4]; zw[5] = (u[1] / 10.0) / lsw[5]; zw[6] = (u[2] / 10.0) / lsw[6];
      zw[10] = (speed / 10.0) / lsw[10];
      break;
    }
    case 2: {
      const double speed = r6_speed(x);
      const double rho = 1.225 * exp(-x[1] / 8500.0);
      const double qd = 0.5 * rho * speed * speed;
      zv[4] = (qd / qn) / lsv[4]; zv[12] = (rho / 1.225) / lsv[12];
      zw[11] = (qd / qn) / lsw[11];
      break;
    }
    case 3: {
      const double speed = r6_speed(x);
      double vb[3];
      r6_body_velocity(x, vb);
      zv[5] = (speed > 1e-3 ? atan2(-vb[2], vb[0]) : 0.0) / lsv[5];
      break;
    }
    case 4: {
      const double speed = r6_speed(x);
      double vb[3];
      r6_body_velocity(x, vb);
      const bool moving = speed > 1e-3;
      double sb = vb[1] / (moving ? speed : 1.0);
      sb = fmin(fmax(sb, -1.0), 1.0);
      zv[6] = (moving ? asin(sb) : 0.0) / lsv[6];
      break;
    }
    default: {
      double vb[3];
      r6_body_velocity(x, vb);
      zw[7] = (vb[0] / 10.0) / lsw[7]; zw[8] = (vb[1] / 10.0) / lsw[8]; zw[9] = (vb[2] / 10.0) / lsw[9];
      break;
    }
  }
}

__device__ __forceinline__ bool r6_landing_ok(const double *x, double m0) {
  // LandingConstraints.check_landing (monte_carlo.py:54-104), run_experiments tolerances
  if (fabs(x[1]) > 1.0) return false;
  if (fabs(x[2]) > 5.0 || fabs(x[3]) > 5.0) return false;
  if (fabs(x[4]) > 3.0) return false;
  if (fabs(x[5]) > 1.0 || fabs(x[6]) > 1.0) return false;
  if (1.0 - x[0] / m0 > 1.0 - 0.05) return false;
  return true;
}

struct R6Args {
  QPSettingsDev st;
  double dt;
  int max_steps;
  double *x, *U, *Xp, *gm, *Xo, *ysc, *rho, *rec;
  double *lin;   // per rollout and stage: -[A_d | B_d] (14 x 17), from k_r6_predict
  int *pending;  // the control kernel solved: k_r6_plant applies U[0]
  // the two FITC GPs (d_v: 13 features, d_w: 12)
  GpView gv, gw;
  int Mv, Mw;
  const double *cv, *cw;  // mean coefficients (3 x M): beta^T, or alpha^T as written
  const double *prm;      // problem data (R6_PRM, r6 layout above)
  int use_gp, upright;
  // GPMPC.solve mode (gpmpc_rollout6_solve): 0 = Monte-Carlo rollout step; 1 = first
  // pass (forward simulation of U); 2 = later pass (GP means and Jacobians at the plan)
  int mode;
  double sqp_tol;
  const double *xt;       // GPMPC.solve: per-rollout X_ref (B x (N+1) x 14)
  const double *ut;       // GPMPC.solve: per-rollout U_ref (B x N x 3)
  R6Rocket rk;
  int *done, *passes, *qit, *qst;
};

// ---------------------------------------------------------------------------
// 1. termination rules + forward simulation with the GP mean
// sum over the inducing rows i = t0, t0 + stride, .. of k(z, x_i) coef[c][i] (c < 3),
// two rows per trip with all their loads issued before either is used
template <int D>
__device__ __forceinline__ void r6_kernel_rows(const GpView &v, int M, const double *__restrict__ cf,
                                               const double *zs, int t0, int stride, double *acc) {
  double z[D], zn = 0.0;
#pragma unroll
  for (int f = 0; f < D; ++f) { z[f] = zs[f]; zn += z[f] * z[f]; }  // |z|^2 in the feature order
  const double *__restrict__ Xs = v.Xs;
  const double *__restrict__ Xn = v.Xn;
  int i = t0;
  for (; i + stride < M; i += 2 * stride) {
    const int j = i + stride;
    double xa[D], xb[D], ca[3], cb[3];
#pragma unroll
    for (int f = 0; f < D; ++f) { xa[f] = Xs[(int64_t)i * D + f]; xb[f] = Xs[(int64_t)j * D + f]; }
    const double na = Xn[i], nb = Xn[j];
#pragma unroll
    for (int c = 0; c < 3; ++c) { ca[c] = cf[(int64_t)c * M + i]; cb[c] = cf[(int64_t)c * M + j]; }
    double da = 0.0, db = 0.0;
#pragma unroll
    for (int f = 0; f < D; ++f) { da = fma(z[f], xa[f], da); db = fma(z[f], xb[f], db); }
    const double ka = kernel_epilogue(GPMPC_SE_ARD, (zn + na) - 2.0 * da, v.sigma2, 0.0);
    const double kb = kernel_epilogue(GPMPC_SE_ARD, (zn + nb) - 2.0 * db, v.sigma2, 0.0);
#pragma unroll
    for (int c = 0; c < 3; ++c) { acc[c] += ka * ca[c]; acc[c] += kb * cb[c]; }
  }
  if (i < M) {
    double dot = 0.0;
#pragma unroll
    for (int f = 0; f < D; ++f) dot = fma(z[f], Xs[(int64_t)i * D + f], dot);
    const double kv = kernel_epilogue(GPMPC_SE_ARD, (zn + Xn[i]) - 2.0 * dot, v.sigma2, 0.0);
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += kv * cf[(int64_t)c * M + i];
  }
}


// the kernels of one horizon, compiled per supported N (fleet6_n.h)
struct R6Impl {
  int N, M;
  size_t smem;
  hipError_t (*init)();
  void (*predict)(hipStream_t, int B, const R6Args &, bool stamps);
  void (*control)(hipStream_t, int B, const R6Args &, bool stamps);
  void (*plant)(hipStream_t, int B, const R6Args &);
  void (*reset)(hipStream_t, int first, int count, const double *x0, const R6Args &, double rho0);
  void (*solve_begin)(hipStream_t, int B, const R6Args &, int cold, double rho0);
  void (*print_stamps)();
};

namespace r6n20 {
#define R6_N 20
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n20
namespace r6n30 {
#define R6_N 30
#include "fleet6_n.h"
#undef R6_N
}  // namespace r6n30

static const R6Impl *r6_impl(int N) {
  switch (N) {
    case 20: return &r6n20::impl;
    case 30: return &r6n30::impl;
    default: return nullptr;
  }
}
// ---------------------------------------------------------------------------
static int r6_create(gpmpc_ctx *ctx, const GpView &gv, const GpView &gw, bool exact,
                     const gpmpc_rollout6_config *cfg, int batch, gpmpc_rollout6 **out) {
  GPMPC_CHECK_ARG(ctx && cfg && out && batch > 0);
  if (gv.d != 13 || gw.d != 12 || gv.n_out != 3 || gw.n_out != 3 || gv.kind != GPMPC_SE_ARD ||
      gw.kind != GPMPC_SE_ARD) {
    gpmpc_set_error("rollout6: expects the StructuredRocketGP pair (13 / 12 features, 3 outputs, SE-ARD)");
    return -2;
  }
  const R6Impl *impl = r6_impl(cfg->horizon);
  if (!impl) {
    gpmpc_set_error("rollout6: horizon %d not compiled (20: GPMPCConfig's N, 30: BASELINE configs[4])",
                    cfg->horizon);
    return -2;
  }
  for (int i = 0; i < R6_NX; ++i)
    if (!(cfg->q_diag[i] >= 0.0) || !(cfg->p_diag[i] >= 0.0)) {
      gpmpc_set_error("rollout6: cost weights must be non-negative");
      return -2;
    }
  if (!(cfg->t_max > 0.0) || !(cfg->trust_x2 > 0.0) || !(cfg->trust_u2 > 0.0)) {
    gpmpc_set_error("rollout6: t_max and the trust radii must be positive");
    return -2;
  }
  for (int i = 0; i < 3; ++i)
    if (!(cfg->rocket_j[i] > 0.0)) {
      gpmpc_set_error("rollout6: the rocket's J_B diagonal must be positive");
      return -2;
    }
  if (!(cfg->rocket_alpha >= 0.0) || !(cfg->rocket_g0 > 0.0)) {
    gpmpc_set_error("rollout6: rocket alpha must be >= 0 and g0 > 0");
    return -2;
  }
  GPMPC_HIP(hipSetDevice(ctx->device));
  auto *r = new gpmpc_rollout6();
  r->ctx = ctx; r->gv = gv; r->gw = gw; r->exact = exact; r->cfg = *cfg; r->B = batch;
  r->impl = impl; r->N = impl->N; r->M = impl->M;
  const size_t B = batch, N = r->N;
  if (r->x.alloc(sizeof(double) * B * R6_NX) || r->U.alloc(sizeof(double) * B * N * R6_NU) ||
      r->Xp.alloc(sizeof(double) * B * (N + 1) * R6_NX) || r->gm.alloc(sizeof(double) * B * N * 6) ||
      r->Xo.alloc(sizeof(double) * B * (N + 1) * R6_NX) || r->ysc.alloc(sizeof(double) * B * r->M) ||
      r->rho.alloc(sizeof(double) * B) || r->rec.alloc(sizeof(double) * B * GPMPC_REC_LEN) ||
      r->lin.alloc(sizeof(double) * B * N * R6_NX * R6_SZ) || r->pending.alloc(sizeof(int) * B) ||
      r->betav.alloc(sizeof(double) * 3 * gv.n) || r->betaw.alloc(sizeof(double) * 3 * gw.n) ||
      r->prm.alloc(sizeof(double) * R6_PRM) || r->xt.alloc(sizeof(double) * B * (N + 1) * R6_NX) ||
      r->ut.alloc(sizeof(double) * B * N * R6_NU) ||
      r->xin.alloc(sizeof(double) * B * R6_NX) || r->done.alloc(sizeof(int) * B) ||
      r->passes.alloc(sizeof(int) * B) || r->qit.alloc(sizeof(int) * B) || r->qst.alloc(sizeof(int) * B)) {
    delete r;
    gpmpc_set_error("rollout6: out of device memory");
    return -1;
  }
  double prm[R6_PRM];
  for (int i = 0; i < R6_NX; ++i) { prm[R6_PQ + i] = cfg->q_diag[i]; prm[R6_PP + i] = cfg->p_diag[i]; }
  for (int i = 0; i < R6_NU; ++i) prm[R6_PR + i] = cfg->r_diag[i];
  prm[R6_PTMIN] = cfg->t_min; prm[R6_PTMAX] = cfg->t_max; prm[R6_PTAN] = cfg->tan_gamma_gs;
  prm[R6_PTRX] = cfg->trust_x2; prm[R6_PTRU] = cfg->trust_u2;
  hipMemcpyAsync(r->prm.p, prm, sizeof(prm), hipMemcpyHostToDevice, ctx->stream);
  std::vector<double> rc(B * GPMPC_REC_LEN, 0.0);
  for (size_t i = 0; i < B; ++i) rc[i * GPMPC_REC_LEN] = -1.0;  // not started until reset
  hipMemcpyAsync(r->rec.p, rc.data(), sizeof(double) * rc.size(), hipMemcpyHostToDevice, ctx->stream);
  hipMemsetAsync(r->Xo.p, 0, sizeof(double) * B * (N + 1) * R6_NX, ctx->stream);
  hipMemsetAsync(r->ut.p, 0, sizeof(double) * B * N * R6_NU, ctx->stream);
  hipMemsetAsync(r->pending.p, 0, sizeof(int) * B, ctx->stream);
  hipMemsetAsync(r->done.p, 0, sizeof(int) * B, ctx->stream);
  if (!exact) {  // beta^T = alpha^T L_uu^-1: the FITC posterior mean's coefficients
    if (launch_gemm_nn(ctx->stream, 3, gv.n, gv.n, gv.alphaT, gv.n, gv.W, gv.n, r->betav.as<double>(), gv.n, 1.0,
                       0.0) != hipSuccess ||
        launch_gemm_nn(ctx->stream, 3, gw.n, gw.n, gw.alphaT, gw.n, gw.W, gw.n, r->betaw.as<double>(), gw.n, 1.0,
                       0.0) != hipSuccess) {
      delete r;
      gpmpc_set_error("rollout6: beta GEMM launch failed");
      return -1;
    }
  }
  if (impl->init() != hipSuccess) {
    delete r;
    gpmpc_set_error("rollout6: %zu B of LDS not available", impl->smem);
    return -1;
  }
  GPMPC_HIP(hipStreamSynchronize(ctx->stream));
  *out = r;
  return 0;
}

extern "C" int gpmpc_rollout6_create(gpmpc_ctx *ctx, gpmpc_fitc *gp_v, gpmpc_fitc *gp_w,
                                     const gpmpc_rollout6_config *cfg, int batch, gpmpc_rollout6 **out) {
  GPMPC_CHECK_ARG(gp_v && gp_w);
  return r6_create(ctx, fitc_view(gp_v), fitc_view(gp_w), false, cfg, batch, out);
}

extern "C" int gpmpc_rollout6_create_exact(gpmpc_ctx *ctx, gpmpc_gp *gp_v, gpmpc_gp *gp_w,
                                           const gpmpc_rollout6_config *cfg, int batch, gpmpc_rollout6 **out) {
  GPMPC_CHECK_ARG(gp_v && gp_w);
  return r6_create(ctx, gp_view(gp_v), gp_view(gp_w), true, cfg, batch, out);
}

static R6Args r6_args(gpmpc_rollout6 *r) {
  R6Args a;
  a.st = to_dev(r->cfg.qp);
  a.dt = r->cfg.dt;
  a.max_steps = r->cfg.max_steps;
  a.x = r->x.as<double>(); a.U = r->U.as<double>(); a.Xp = r->Xp.as<double>();
  a.gm = r->gm.as<double>(); a.Xo = r->Xo.as<double>(); a.ysc = r->ysc.as<double>();
  a.rho = r->rho.as<double>(); a.rec = r->rec.as<double>();
  a.lin = r->lin.as<double>(); a.pending = r->pending.as<int>();
  a.gv = r->gv; a.gw = r->gw;
  a.Mv = a.gv.n; a.Mw = a.gw.n;
  const bool as_written = r->exact || r->cfg.fitc_mean_as_written;
  a.cv = as_written ? a.gv.alphaT : r->betav.as<double>();
  a.cw = as_written ? a.gw.alphaT : r->betaw.as<double>();
  a.prm = r->prm.as<double>();
  a.use_gp = r->cfg.use_gp_mean != 0;
  a.upright = r->cfg.upright_target != 0;
  a.mode = 0;
  a.sqp_tol = 0.0;
  a.xt = r->xt.as<double>();
  a.ut = r->ut.as<double>();
  a.done = r->done.as<int>(); a.passes = r->passes.as<int>();
  a.qit = r->qit.as<int>(); a.qst = r->qst.as<int>();
  const gpmpc_rollout6_config &c = r->cfg;
  for (int i = 0; i < 3; ++i) { a.rk.J[i] = c.rocket_j[i]; a.rk.rT[i] = c.rocket_r_t[i]; a.rk.gI[i] = c.rocket_g_i[i]; }
  a.rk.alpha = c.rocket_alpha;
  a.rk.g0 = c.rocket_g0;
  return a;
}

extern "C" int gpmpc_rollout6_reset(gpmpc_rollout6 *r, int first, int count, const double *x0) {
  GPMPC_CHECK_ARG(r && x0 && first >= 0 && count >= 0 && first + count <= r->B);
  if (count == 0) return 0;
  hipStream_t s = r->ctx->stream;
  DevBuf d;
  GPMPC_HIP(d.alloc(s, sizeof(double) * count * R6_NX));
  GPMPC_HIP(hipMemcpyAsync(d.p, x0, sizeof(double) * count * R6_NX, hipMemcpyHostToDevice, s));
  r->impl->reset(s, first, count, d.as<double>(), r6_args(r), r->cfg.qp.rho);
  GPMPC_HIP(hipGetLastError());
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

static bool r6_stamps_on() {
  static const bool on = [] {
    const char *e = getenv("GPMPC_R6_STAMPS");
    return e && atoi(e) > 0;
  }();
  return on;
}

extern "C" int gpmpc_rollout6_step_phases(gpmpc_rollout6 *r, int mask) {
  GPMPC_CHECK_ARG(r);
  GPMPC_HIP(hipSetDevice(r->ctx->device));
  hipStream_t s = r->ctx->stream;
  const R6Args a = r6_args(r);
  if (mask & 1) r->impl->predict(s, r->B, a, r6_stamps_on());
  if (mask & 2) r->impl->control(s, r->B, a, r6_stamps_on());
  if (mask & 4) r->impl->plant(s, r->B, a);
  GPMPC_HIP(hipGetLastError());
  return 0;
}

extern "C" int gpmpc_rollout6_step(gpmpc_rollout6 *r, int nsteps) {
  GPMPC_CHECK_ARG(r && nsteps >= 0);
  for (int it = 0; it < nsteps; ++it) {
    const int rc = gpmpc_rollout6_step_phases(r, 7);
    if (rc) return rc;
  }
  return 0;
}

extern "C" int gpmpc_rollout6_solve_ref(gpmpc_rollout6 *r, const double *x0, const double *x_target,
                                        const double *X_ref, const double *U_ref, int cold, int max_sqp_iter,
                                        double sqp_tol, double *X, double *U, int *passes, int *converged,
                                        int *qp_status, int *qp_iters) {
  GPMPC_CHECK_ARG(r && x0 && x_target && max_sqp_iter >= 1 && sqp_tol >= 0.0 && cold >= 0 && cold <= 2);
  GPMPC_HIP(hipSetDevice(r->ctx->device));
  hipStream_t s = r->ctx->stream;
  const size_t B = r->B, N = r->N;
  GPMPC_HIP(hipMemcpyAsync(r->x.p, x0, sizeof(double) * B * R6_NX, hipMemcpyHostToDevice, s));
  // the QP cost's references (gp_mpc.py:442-445): X_ref = x_target on every stage unless given,
  // U_ref = 0 unless given
  std::vector<double> xr;
  if (!X_ref) {
    xr.resize(B * (N + 1) * R6_NX);
    for (size_t b = 0; b < B; ++b)
      for (size_t k = 0; k <= N; ++k)
        for (int i = 0; i < R6_NX; ++i) xr[(b * (N + 1) + k) * R6_NX + i] = x_target[b * R6_NX + i];
    X_ref = xr.data();
  }
  GPMPC_HIP(hipMemcpyAsync(r->xt.p, X_ref, sizeof(double) * B * (N + 1) * R6_NX, hipMemcpyHostToDevice, s));
  if (U_ref) GPMPC_HIP(hipMemcpyAsync(r->ut.p, U_ref, sizeof(double) * B * N * R6_NU, hipMemcpyHostToDevice, s));
  else GPMPC_HIP(hipMemsetAsync(r->ut.p, 0, sizeof(double) * B * N * R6_NU, s));
  R6Args a = r6_args(r);
  a.sqp_tol = sqp_tol;
  r->impl->solve_begin(s, r->B, a, cold, r->cfg.qp.rho);
  for (int p = 1; p <= max_sqp_iter; ++p) {  // passes of converged rollouts exit at once
    a.mode = p == 1 ? 1 : 2;
    r->impl->predict(s, r->B, a, false);
    r->impl->control(s, r->B, a, false);
  }
  GPMPC_HIP(hipGetLastError());
  if (X) GPMPC_HIP(hipMemcpyAsync(X, r->Xo.p, sizeof(double) * B * (N + 1) * R6_NX, hipMemcpyDeviceToHost, s));
  if (U) GPMPC_HIP(hipMemcpyAsync(U, r->U.p, sizeof(double) * B * N * R6_NU, hipMemcpyDeviceToHost, s));
  if (passes) GPMPC_HIP(hipMemcpyAsync(passes, r->passes.p, sizeof(int) * B, hipMemcpyDeviceToHost, s));
  if (converged) GPMPC_HIP(hipMemcpyAsync(converged, r->done.p, sizeof(int) * B, hipMemcpyDeviceToHost, s));
  if (qp_status) GPMPC_HIP(hipMemcpyAsync(qp_status, r->qst.p, sizeof(int) * B, hipMemcpyDeviceToHost, s));
  if (qp_iters) GPMPC_HIP(hipMemcpyAsync(qp_iters, r->qit.p, sizeof(int) * B, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

extern "C" int gpmpc_rollout6_solve(gpmpc_rollout6 *r, const double *x0, const double *x_target, int cold,
                                    int max_sqp_iter, double sqp_tol, double *X, double *U, int *passes,
                                    int *converged, int *qp_status, int *qp_iters) {
  return gpmpc_rollout6_solve_ref(r, x0, x_target, nullptr, nullptr, cold, max_sqp_iter, sqp_tol, X, U, passes,
                                  converged, qp_status, qp_iters);
}

extern "C" int gpmpc_rollout6_read(gpmpc_rollout6 *r, double *records, double *x) {
  GPMPC_CHECK_ARG(r);
  hipStream_t s = r->ctx->stream;
  if (records)
    GPMPC_HIP(hipMemcpyAsync(records, r->rec.p, sizeof(double) * r->B * GPMPC_REC_LEN,
                             hipMemcpyDeviceToHost, s));
  if (x) GPMPC_HIP(hipMemcpyAsync(x, r->x.p, sizeof(double) * r->B * R6_NX, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

extern "C" int gpmpc_rollout6_get_state(gpmpc_rollout6 *r, double *U, double *X_plan, double *X_pred,
                                        double *gp_mean, double *y_scaled, double *rho) {
  GPMPC_CHECK_ARG(r);
  hipStream_t s = r->ctx->stream;
  const size_t B = r->B, N = r->N;
  if (U) GPMPC_HIP(hipMemcpyAsync(U, r->U.p, sizeof(double) * B * N * R6_NU, hipMemcpyDeviceToHost, s));
  if (X_plan)
    GPMPC_HIP(hipMemcpyAsync(X_plan, r->Xo.p, sizeof(double) * B * (N + 1) * R6_NX, hipMemcpyDeviceToHost, s));
  if (X_pred)
    GPMPC_HIP(hipMemcpyAsync(X_pred, r->Xp.p, sizeof(double) * B * (N + 1) * R6_NX, hipMemcpyDeviceToHost, s));
  if (gp_mean) GPMPC_HIP(hipMemcpyAsync(gp_mean, r->gm.p, sizeof(double) * B * N * 6, hipMemcpyDeviceToHost, s));
  if (y_scaled) GPMPC_HIP(hipMemcpyAsync(y_scaled, r->ysc.p, sizeof(double) * B * r->M, hipMemcpyDeviceToHost, s));
  if (rho) GPMPC_HIP(hipMemcpyAsync(rho, r->rho.p, sizeof(double) * B, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

extern "C" double *gpmpc_rollout6_records_dev(gpmpc_rollout6 *r) { return r ? r->rec.as<double>() : nullptr; }

extern "C" int gpmpc_rollout6_set_state(gpmpc_rollout6 *r, const double *U, const double *y_scaled,
                                        const double *rho) {
  GPMPC_CHECK_ARG(r);
  hipStream_t s = r->ctx->stream;
  const size_t B = r->B, N = r->N;
  if (U) GPMPC_HIP(hipMemcpyAsync(r->U.p, U, sizeof(double) * B * N * R6_NU, hipMemcpyHostToDevice, s));
  if (y_scaled) GPMPC_HIP(hipMemcpyAsync(r->ysc.p, y_scaled, sizeof(double) * B * r->M, hipMemcpyHostToDevice, s));
  if (rho) GPMPC_HIP(hipMemcpyAsync(r->rho.p, rho, sizeof(double) * B, hipMemcpyHostToDevice, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

extern "C" int gpmpc_rollout6_destroy(gpmpc_rollout6 *r) {
  if (r && r->ctx) (void)hipStreamSynchronize(r->ctx->stream);
  if (r && r6_stamps_on() && r->impl) r->impl->print_stamps();
  delete r;
  return 0;
}
