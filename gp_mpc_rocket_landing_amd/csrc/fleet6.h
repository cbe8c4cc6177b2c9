// fleet6.h -- what the 6-DoF rollout kernels of every horizon share (fleet6.hip: the
// C-ABI; fleet6_n.h: the kernels of one horizon, instantiated by fleet6_h*.hip).
#pragma once
#include "internal.h"
#include "gemm.h"
#include "qp.h"
#include <vector>

#define R6_NX 14
#define R6_NU 3
#define R6_SZ 17
// the horizon N is a compile-time constant of the kernels (fully unrolled chains,
// LDS layout): fleet6_n.h is compiled once per horizon N = R6_NMIN .. R6_NMAX, in
// namespaces r6n2 .. r6n30 (fleet6_h*.hip); the C-ABI dispatches on the config's
// horizon (GPMPCConfig N = 20, gp_mpc.py:110 / nominal_mpc.py:47; configs[4] N = 30)
#define R6_NMIN 2
#define R6_NMAX 30
#define R6_T 512                              // two items (variables / rows) per thread
#define R6_TRI 153                            // packed lower 17 x 17
#define R6_PT 512                             // predict threads (7 kernel-row waves + the RK4 wave)
#define R6_FOR_H _Pragma("unroll") for (int h = 0; h < 2; ++h)
// 1: the control kernel's item indices and thread index are made opaque once per ADMM
// iteration (fleet6_n.h r6_launder / r6_tid), so the addresses derived from them are
// not hoisted out of the loop into spilled registers (N = 30: scratch 360 -> 112 B/lane)
#ifndef R6_LAUNDER
#define R6_LAUNDER 1
#endif
// block steps per chain-loop trip (the whole chain since the spills went: 64 rollouts
// 0.881-0.888 -> 0.869-0.870 ms per step against 3, profiles/r5_r6_unroll_ab.log) and
// diagonal-product operands in flight per chunk (6, 9, 17 measured level)
#ifndef R6_CHAIN_UNROLL
#define R6_CHAIN_UNROLL 15
#endif
#ifndef R6_DIAG_CHUNK
#define R6_DIAG_CHUNK 6
#endif
#define R6_STR_(x) #x
#define R6_STR(x) R6_STR_(x)

// ConstraintParams (constraints.py:35-50), CostWeights (cost_functions.py:39-98),
// gp_mpc.py trust regions (:432-435)
#define R6_T_MIN 0.5
#define R6_T_MAX 5.0

// the rocket (Rocket6DoFConfig, rocket_6dof.py:36-84): J_B, thrust point r_T_B, gravity
// g_I, alpha = 1 / (I_sp g0), g0 -- kernel arguments (uniform values).  A diagonal J_B
// runs as its diagonal J (divisions, the arithmetic of round 5); any other (full = 1)
// as the row-major tensor Jf and its inverse Ji: w' = Ji (r_T x u - w x Jf w), the
// ca.solve(J, .) of nominal_mpc.py:196-199 with the inverse formed once on the host
struct R6Rocket {
  double J[3], rT[3], gI[3], alpha, g0;
  double Jf[9], Ji[9];
  int full;
};

__device__ __forceinline__ void r6_mat3(const double *M, const double *v, double *o) {
  for (int i = 0; i < 3; ++i) o[i] = (M[3 * i] * v[0] + M[3 * i + 1] * v[1]) + M[3 * i + 2] * v[2];
}


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

static __device__ void r6_f(const R6Rocket &rk, const double *x, const double *u, double *o) {
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
  if (rk.full) {
    const double w[3] = {wx, wy, wz};
    double jw[3];
    r6_mat3(rk.Jf, w, jw);
    const double r[3] = {tq[0] - (wy * jw[2] - wz * jw[1]), tq[1] - (wz * jw[0] - wx * jw[2]),
                         tq[2] - (wx * jw[1] - wy * jw[0])};
    r6_mat3(rk.Ji, r, o + 11);
    return;
  }
  const double jw[3] = {J[0] * wx, J[1] * wy, J[2] * wz};
  const double cx[3] = {wy * jw[2] - wz * jw[1], wz * jw[0] - wx * jw[2], wx * jw[1] - wy * jw[0]};
  for (int i = 0; i < 3; ++i) o[11 + i] = (tq[i] - cx[i]) / J[i];
}

// RK4 (discretization.py:229-252) + quaternion normalisation (rocket_6dof.py:371-387)
static __device__ void r6_step(const R6Rocket &rk, const double *x, const double *u, double dt, double *xn) {
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
static __device__ void r6_neg_lin(const R6Rocket &rk, const double *x, const double *u, double dt, double *blk) {
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
  const double rx = rk.rT[0], ry = rk.rT[1], rz = rk.rT[2];
  const double Rx[3][3] = {{0, -rz, ry}, {rz, 0, -rx}, {-ry, rx, 0}};
  if (rk.full) {
    // d/dw Ji (-w x Jf w) = Ji ([Jf w]x - [w]x Jf);  B_c omega rows: Ji [r_T]x
    const double w[3] = {wx, wy, wz};
    double jw[3];
    r6_mat3(rk.Jf, w, jw);
    const double Wx[3][3] = {{0, -wz, wy}, {wz, 0, -wx}, {-wy, wx, 0}};
    const double JWx[3][3] = {{0, -jw[2], jw[1]}, {jw[2], 0, -jw[0]}, {-jw[1], jw[0], 0}};
    double D[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        D[i][j] = JWx[i][j] - ((Wx[i][0] * rk.Jf[j] + Wx[i][1] * rk.Jf[3 + j]) + Wx[i][2] * rk.Jf[6 + j]);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        const double a = (rk.Ji[3 * i] * D[0][j] + rk.Ji[3 * i + 1] * D[1][j]) + rk.Ji[3 * i + 2] * D[2][j];
        const double bu = (rk.Ji[3 * i] * Rx[0][j] + rk.Ji[3 * i + 1] * Rx[1][j]) + rk.Ji[3 * i + 2] * Rx[2][j];
        set(11 + i, 11 + j, -((i == j ? 1.0 : 0.0) + a * dt));
        set(11 + i, 14 + j, -(bu * dt));
      }
    return;
  }
  const double j1 = rk.J[0], j2 = rk.J[1], j3 = rk.J[2];
  const double Aw[3][3] = {{0, wz, wy}, {wz, 0, wx}, {wy, wx, 0}};
  const double cw[3] = {-(j3 - j2) / j1, -(j1 - j3) / j2, -(j2 - j1) / j3};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) set(11 + i, 11 + j, -((i == j ? 1.0 : 0.0) + cw[i] * Aw[i][j] * dt));
  // B_c omega rows: J^-1 [r_T]x
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

static __device__ void r6_features_role(int role, const double *x, const double *u, const double *lsv,
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
  int mcv, mcw;  // inducing rows of each GP the predict kernel keeps in LDS (r6_pcache_rows)
  // the split predict (r6_predict_parts): each rollout's kernel rows over `parts`
  // co-resident workgroups, their per-wave sums exchanged as tagged 8-byte granules
  // (R6_GRAN per point, two point parities per rollout, zeroed before every launch)
  int parts, nb;  // workgroups per rollout; the batch (the split's grid covers it in eights)
  unsigned long long *gran;
  unsigned *tmo;  // a bounded spin that gave up (nonzero: the results are unreliable)
};
// per rollout and point parity: 7 kernel-row waves x 6 sums x 2 granules (hi, lo words)
#define R6_GRAN 84
// rows of each GP the predict kernel caches in LDS, feature-major: 720 x (13 + 12) doubles =
// 141 KB beside its ~4 KB of static LDS (GPMPC_R6_PCACHE rows; 0 = none)
#define R6_PCACHE_ROWS 720

// ---------------------------------------------------------------------------
// 1. termination rules + forward simulation with the GP mean
// The kernel rows K*u . coefficients of one GP for this thread's inducing rows t0, t0 +
// stride, ...: rows below Mc come from the feature-major LDS copy sx (sx[f Mc + i], loaded
// once per launch), the rest from the row-major global Xs.  Same rows, same order, same
// fma sequence either way (identical bits); the LDS rows spare the texture path the
// lane-strided 8-byte loads that bound the phase.
template <int D>
__device__ __forceinline__ void r6_kernel_rows(const GpView &v, int M, const double *__restrict__ cf,
                                               const double *zs, int t0, int stride, double *acc,
                                               const double *sx = nullptr, int Mc = 0) {
  double z[D], zn = 0.0;
#pragma unroll
  for (int f = 0; f < D; ++f) { z[f] = zs[f]; zn += z[f] * z[f]; }  // |z|^2 in the feature order
  const double *__restrict__ Xs = v.Xs;
  const double *__restrict__ Xn = v.Xn;
  auto row2 = [&](int i, int j, const double (&xa)[D], const double (&xb)[D]) {
    const double na = Xn[i], nb = Xn[j];
    double ca[3], cb[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { ca[c] = cf[(int64_t)c * M + i]; cb[c] = cf[(int64_t)c * M + j]; }
    double da = 0.0, db = 0.0;
#pragma unroll
    for (int f = 0; f < D; ++f) { da = fma(z[f], xa[f], da); db = fma(z[f], xb[f], db); }
    const double ka = kernel_epilogue(GPMPC_SE_ARD, (zn + na) - 2.0 * da, v.sigma2, 0.0);
    const double kb = kernel_epilogue(GPMPC_SE_ARD, (zn + nb) - 2.0 * db, v.sigma2, 0.0);
#pragma unroll
    for (int c = 0; c < 3; ++c) { acc[c] += ka * ca[c]; acc[c] += kb * cb[c]; }
  };
  auto row1 = [&](int i, const double (&x)[D]) {
    double dot = 0.0;
#pragma unroll
    for (int f = 0; f < D; ++f) dot = fma(z[f], x[f], dot);
    const double kv = kernel_epilogue(GPMPC_SE_ARD, (zn + Xn[i]) - 2.0 * dot, v.sigma2, 0.0);
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += kv * cf[(int64_t)c * M + i];
  };
  int i = t0;
  if (Mc > 0) {  // the LDS rows (feature-major: a wave's 64 rows are 64 consecutive doubles)
    for (; i + stride < Mc; i += 2 * stride) {
      double xa[D], xb[D];
#pragma unroll
      for (int f = 0; f < D; ++f) { xa[f] = sx[f * Mc + i]; xb[f] = sx[f * Mc + i + stride]; }
      row2(i, i + stride, xa, xb);
    }
    if (i < Mc) {
      double xa[D];
#pragma unroll
      for (int f = 0; f < D; ++f) xa[f] = sx[f * Mc + i];
      if (i + stride < M) {  // pair it with the first global row (keeps two rows in flight)
        double xb[D];
#pragma unroll
        for (int f = 0; f < D; ++f) xb[f] = Xs[(int64_t)(i + stride) * D + f];
        row2(i, i + stride, xa, xb);
        i += 2 * stride;
      } else {
        row1(i, xa);
        i += stride;
      }
    }
  }
  for (; i + stride < M; i += 2 * stride) {
    const int j = i + stride;
    double xa[D], xb[D];
#pragma unroll
    for (int f = 0; f < D; ++f) { xa[f] = Xs[(int64_t)i * D + f]; xb[f] = Xs[(int64_t)j * D + f]; }
    row2(i, j, xa, xb);
  }
  if (i < M) {
    double x[D];
#pragma unroll
    for (int f = 0; f < D; ++f) x[f] = Xs[(int64_t)i * D + f];
    row1(i, x);
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
