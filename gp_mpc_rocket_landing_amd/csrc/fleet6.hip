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
#include "fleet6.h"
#include <algorithm>
#include <cmath>
#include <vector>

struct R6Impl;  // the kernels of one horizon (fleet6_n.h), below
struct gpmpc_rollout6 {
  gpmpc_ctx *ctx = nullptr;
  GpView gv{}, gw{};
  bool exact = false;  // the GP pair is exact (mean K* alpha over the training rows)
  gpmpc_rollout6_config cfg{};
  const R6Impl *impl = nullptr;
  double Jd[3] = {}, Jf[9] = {}, Ji[9] = {};  // the rocket's inertia: diagonal, or full + inverse
  int jfull = 0;
  int B = 0, N = 0, M = 0;  // batch, horizon, QP rows
  DevBuf x, U, Xp, gm, Xo, ysc, rho, rec, lin, pending;
  DevBuf betav, betaw;  // (L_uu^-T alpha)^T of each GP, 3 x M
  DevBuf prm;           // problem data (R6_PRM doubles, r6_prm layout)
  DevBuf xt, ut, done, passes, qit, qst, xin;  // GPMPC.solve mode: X_ref (B x (N+1) x 14), U_ref (B x N x 3)
  DevBuf gran;          // the split predict's granules (B x 2 x R6_GRAN) and timeout word, one block
  int cus = 0;          // compute units of the device (the split predict needs parts x B of them)
};

extern "C" void gpmpc_rollout6_default_config(gpmpc_rollout6_config *c) {
  c->horizon = 30;     // BASELINE configs[4]: N = 30
  c->dt = 0.1;
  c->max_steps = 300;
  gpmpc_qp_default_settings(&c->qp);   // osqp_rti.py:54-60 settings, as the 3-DoF path
  // the reference's FITC mean as written, K*u alpha (sparse_gp.py:280-283): compat by
  // default, as the GPMPC surface (D1 kept, the fix behind a flag); 0 = the
  // FITC posterior mean K*u L_uu^-T alpha (SURVEY D1 fixed)
  c->fitc_mean_as_written = 1;
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
  for (int i = 0; i < 9; ++i) c->rocket_J[i] = 0.0;  // unset: diag(rocket_j)
}

// the kernels of every horizon (fleet6_h*.hip instantiate fleet6_n.h per N)
#define R6_DECL(N) namespace r6n##N { const R6Impl *impl(); }
R6_DECL(2) R6_DECL(3) R6_DECL(4) R6_DECL(5) R6_DECL(6) R6_DECL(7) R6_DECL(8) R6_DECL(9) R6_DECL(10)
R6_DECL(11) R6_DECL(12) R6_DECL(13) R6_DECL(14) R6_DECL(15) R6_DECL(16) R6_DECL(17) R6_DECL(18) R6_DECL(19)
R6_DECL(20) R6_DECL(21) R6_DECL(22) R6_DECL(23) R6_DECL(24) R6_DECL(25) R6_DECL(26) R6_DECL(27) R6_DECL(28)
R6_DECL(29) R6_DECL(30)
#undef R6_DECL

static const R6Impl *r6_impl(int N) {
  using F = const R6Impl *(*)();
  static const F tab[R6_NMAX + 1] = {
      nullptr, nullptr, r6n2::impl, r6n3::impl, r6n4::impl, r6n5::impl, r6n6::impl, r6n7::impl,
      r6n8::impl, r6n9::impl, r6n10::impl, r6n11::impl, r6n12::impl, r6n13::impl, r6n14::impl,
      r6n15::impl, r6n16::impl, r6n17::impl, r6n18::impl, r6n19::impl, r6n20::impl, r6n21::impl,
      r6n22::impl, r6n23::impl, r6n24::impl, r6n25::impl, r6n26::impl, r6n27::impl, r6n28::impl,
      r6n29::impl, r6n30::impl};
  return N >= R6_NMIN && N <= R6_NMAX ? tab[N]() : nullptr;
}
// ---------------------------------------------------------------------------
// the inertia tensor: rocket_J (ABI 4, row-major) when it is set, else diag(rocket_j).
// A diagonal tensor runs as its diagonal (the divisions of the diagonal model); any
// other as J and J^-1, which is formed here once (adjugate / determinant).  0, or -2
// with the error set.
static int r6_inertia(const double *rocket_J, const double *rocket_j, double Jd[3], double Jf[9], double Ji[9],
                      bool &joff) {
  bool jset = false;
  joff = false;
  for (int i = 0; i < 9; ++i) jset = jset || rocket_J[i] != 0.0;
  for (int i = 0; i < 9; ++i) joff = joff || (i % 4 != 0 && rocket_J[i] != 0.0);
  for (int i = 0; i < 3; ++i) Jd[i] = jset ? rocket_J[4 * i] : rocket_j[i];
  if (!joff) {
    for (int i = 0; i < 3; ++i)
      if (!(Jd[i] > 0.0)) {
        gpmpc_set_error("rollout6: the rocket's J_B diagonal must be positive");
        return -2;
      }
    return 0;
  }
  for (int i = 0; i < 9; ++i) Jf[i] = rocket_J[i];
  const double c00 = Jf[4] * Jf[8] - Jf[5] * Jf[7], c01 = Jf[5] * Jf[6] - Jf[3] * Jf[8],
               c02 = Jf[3] * Jf[7] - Jf[4] * Jf[6];
  const double det = Jf[0] * c00 + Jf[1] * c01 + Jf[2] * c02;
  bool fin = std::isfinite(det);
  for (int i = 0; i < 9; ++i) fin = fin && std::isfinite(Jf[i]);
  double scale = 0.0;
  for (int i = 0; i < 9; ++i) scale = std::max(scale, std::fabs(Jf[i]));
  if (!fin || !(std::fabs(det) > 1e-14 * scale * scale * scale)) {
    gpmpc_set_error("rollout6: the rocket's J_B must be finite and invertible");
    return -2;
  }
  const double adj[9] = {c00, Jf[2] * Jf[7] - Jf[1] * Jf[8], Jf[1] * Jf[5] - Jf[2] * Jf[4],
                         c01, Jf[0] * Jf[8] - Jf[2] * Jf[6], Jf[2] * Jf[3] - Jf[0] * Jf[5],
                         c02, Jf[1] * Jf[6] - Jf[0] * Jf[7], Jf[0] * Jf[4] - Jf[1] * Jf[3]};
  for (int i = 0; i < 9; ++i) Ji[i] = adj[i] / det;
  return 0;
}

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
  if (cfg->qp.max_iter < 1) {  // OSQP's validate_settings: "max_iter must be positive"
    gpmpc_set_error("rollout6: qp.max_iter must be positive");
    return -2;
  }
  if (!(cfg->t_max > 0.0) || !(cfg->trust_x2 > 0.0) || !(cfg->trust_u2 > 0.0)) {
    gpmpc_set_error("rollout6: t_max and the trust radii must be positive");
    return -2;
  }
  double Jd[3], Jf[9], Ji[9];
  bool joff = false;
  if (r6_inertia(cfg->rocket_J, cfg->rocket_j, Jd, Jf, Ji, joff)) return -2;
  if (!(cfg->rocket_alpha >= 0.0) || !(cfg->rocket_g0 > 0.0)) {
    gpmpc_set_error("rollout6: rocket alpha must be >= 0 and g0 > 0");
    return -2;
  }
  GPMPC_HIP(hipSetDevice(ctx->device));
  auto *r = new gpmpc_rollout6();
  r->ctx = ctx; r->gv = gv; r->gw = gw; r->exact = exact; r->cfg = *cfg; r->B = batch;
  r->jfull = joff;
  for (int i = 0; i < 3; ++i) r->Jd[i] = Jd[i];
  if (joff)
    for (int i = 0; i < 9; ++i) { r->Jf[i] = Jf[i]; r->Ji[i] = Ji[i]; }
  r->impl = impl; r->N = impl->N; r->M = impl->M;
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) == hipSuccess) r->cus = cus;
  }
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
      r->passes.alloc(sizeof(int) * B) || r->qit.alloc(sizeof(int) * B) || r->qst.alloc(sizeof(int) * B) ||
      r->gran.alloc(sizeof(unsigned long long) * (B * 2 * R6_GRAN + 2))) {
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
  hipMemsetAsync(r->gran.p, 0, sizeof(unsigned long long) * (B * 2 * R6_GRAN + 2), ctx->stream);
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

// Workgroups per rollout for the predict kernel: 4 when four per rollout fit the device
// at once (one per CU: each needs a CU's whole register file), else 1.  The kernel rows
// of a point are split by whole waves, so every split gives the same bits.
// GPMPC_R6_SPLIT=0 keeps one workgroup per rollout (read at every step).
static int r6_predict_parts(int B, int cus) {
  const char *e = getenv("GPMPC_R6_SPLIT");
  if (e && atoi(e) == 0) return 1;
  return (cus > 0 && 4 * ((B + 7) / 8) * 8 <= cus) ? 4 : 1;
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
  for (int i = 0; i < 3; ++i) { a.rk.J[i] = r->Jd[i]; a.rk.rT[i] = c.rocket_r_t[i]; a.rk.gI[i] = c.rocket_g_i[i]; }
  for (int i = 0; i < 9; ++i) { a.rk.Jf[i] = r->Jf[i]; a.rk.Ji[i] = r->Ji[i]; }
  a.rk.full = r->jfull;
  a.rk.alpha = c.rocket_alpha;
  a.rk.g0 = c.rocket_g0;
  a.parts = r6_predict_parts(r->B, r->cus);
  a.gran = r->gran.as<unsigned long long>();
  a.tmo = (unsigned *)(a.gran + (size_t)r->B * 2 * R6_GRAN);
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

static int r6_check_timeout(gpmpc_rollout6 *r) {
  unsigned t = 0;
  GPMPC_HIP(hipMemcpy(&t, r->gran.as<unsigned long long>() + (size_t)r->B * 2 * R6_GRAN, sizeof(t),
                      hipMemcpyDeviceToHost));
  if (t) {
    gpmpc_set_error("rollout6: the split predict timed out waiting for its co-resident workgroups "
                    "(set GPMPC_R6_SPLIT=0)");
    return -1;
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
  return r6_check_timeout(r);
}

extern "C" int gpmpc_rollout6_solve(gpmpc_rollout6 *r, const double *x0, const double *x_target, int cold,
                                    int max_sqp_iter, double sqp_tol, double *X, double *U, int *passes,
                                    int *converged, int *qp_status, int *qp_iters) {
  return gpmpc_rollout6_solve_ref(r, x0, x_target, nullptr, nullptr, cold, max_sqp_iter, sqp_tol, X, U, passes,
                                  converged, qp_status, qp_iters);
}

// the split predict's sticky timeout word: a part that gave up waiting for its siblings
// (they were not co-resident) leaves results that cannot be trusted
extern "C" int gpmpc_rollout6_read(gpmpc_rollout6 *r, double *records, double *x) {
  GPMPC_CHECK_ARG(r);
  hipStream_t s = r->ctx->stream;
  if (records)
    GPMPC_HIP(hipMemcpyAsync(records, r->rec.p, sizeof(double) * r->B * GPMPC_REC_LEN,
                             hipMemcpyDeviceToHost, s));
  if (x) GPMPC_HIP(hipMemcpyAsync(x, r->x.p, sizeof(double) * r->B * R6_NX, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return r6_check_timeout(r);
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

// ---------------------------------------------------------------------------
// UncertaintyPropagator._propagate_linear (uncertainty_prop.py:117-177) for the 14-state
// model over a StructuredRocketGP pair, batch trajectories at once (gpmpc_uprop6_linear).
// One workgroup per trajectory walks the N steps: the raw features of (x_k, u_k) (six
// roles on six lanes, r6_features_role with unit length-scales) and -[A_d | B_d] at
// (x_k, u_k) (r6_neg_lin, one lane of wave 1) side by side; then the features scaled by
// each GP's length-scales (the k_scale_rows arithmetic), both GPs' means over their rows
// (all threads, a fixed-order reduction), and on thread 0 the RK4 step with quaternion
// normalisation (rocket_6dof.py step) plus dt d_v / dt d_w on the velocity / rate rows.
// The variances of all B N queries then come from each GP's batched posterior, and one
// launch propagates every covariance (k_cov_propagate).
#define U6_NCAP 256  // horizon steps whose controls k_uprop6_means stages in LDS
__global__ __launch_bounds__(256) void k_uprop6_means(GpView gv, GpView gw, R6Rocket rk, int N, double dt,
                                                      const double *__restrict__ x0, const double *__restrict__ U,
                                                      double *__restrict__ Qv, double *__restrict__ Qw,
                                                      double *__restrict__ A, double *__restrict__ means) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ double sx[R6_NX], sxn[R6_NX], sug[R6_NU], qv[13], qw[12], zv[13], zw[12], red[4][6];
  __shared__ double blk[R6_NX * R6_SZ];
  // this thread's rows of each GP (row tid), held in registers for the N steps when both
  // GPs have at most 256 rows (FITC inducing sets); else read per step
  const bool reg = gv.n <= 256 && gw.n <= 256;
  double xv[13], xw[12], nv = 0.0, nw = 0.0, av[3] = {0.0, 0.0, 0.0}, aw[3] = {0.0, 0.0, 0.0};
  const bool okv = reg && tid < gv.n, okw = reg && tid < gw.n;
#pragma unroll
  for (int f = 0; f < 13; ++f) xv[f] = okv ? gv.Xs[(int64_t)tid * 13 + f] : 0.0;
#pragma unroll
  for (int f = 0; f < 12; ++f) xw[f] = okw ? gw.Xs[(int64_t)tid * 12 + f] : 0.0;
  if (okv) {
    nv = gv.Xn[tid];
    for (int c = 0; c < 3; ++c) av[c] = gv.alphaT[(int64_t)c * gv.n + tid];
  }
  if (okw) {
    nw = gw.Xn[tid];
    for (int c = 0; c < 3; ++c) aw[c] = gw.alphaT[(int64_t)c * gw.n + tid];
  }
  // the trajectory's controls staged in LDS once (up to U6_NCAP steps): no global round
  // trip on the step chain
  __shared__ double sU[U6_NCAP * R6_NU];
  const bool uc = N <= U6_NCAP;
  for (int e = tid; uc && e < N * R6_NU; e += 256) sU[e] = U[(int64_t)b * N * R6_NU + e];
  if (tid < R6_NX) {
    sx[tid] = x0[(int64_t)b * R6_NX + tid];
    means[(int64_t)b * (N + 1) * R6_NX + tid] = sx[tid];
  }
  if (!uc && tid < R6_NU && N > 0) sug[tid] = U[(int64_t)b * N * R6_NU + tid];
  __syncthreads();
  for (int k = 0; k < N; ++k) {
    const int64_t pk = (int64_t)b * N + k;
    const double *su = uc ? sU + k * R6_NU : sug;
    // the raw features (six roles, six lanes), -[A_d | B_d] and the nominal RK4 step, side by side
    if (tid < R6_FEAT_ROLES) {
      const double one[13] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
      r6_features_role(tid, sx, su, one, one, qv, qw);
    } else if (tid == 64) {
      for (int e = 0; e < R6_NX * R6_SZ; ++e) blk[e] = 0.0;
      r6_neg_lin(rk, sx, su, dt, blk);
    } else if (tid == 255) {
      r6_step(rk, sx, su, dt, sxn);
    }
    __syncthreads();
    if (tid < 13) {
      zv[tid] = gv.kind == GPMPC_SE_ISO ? qv[tid] : qv[tid] / gv.ls[tid];
      Qv[pk * 13 + tid] = qv[tid];
    } else if (tid >= 64 && tid < 76) {
      const int f = tid - 64;
      zw[f] = gw.kind == GPMPC_SE_ISO ? qw[f] : qw[f] / gw.ls[f];
      Qw[pk * 12 + f] = qw[f];
    } else if (tid >= 128 && tid < 128 + 98) {  // A_k = I + A_c dt = -(the block's first 14 columns)
      for (int e = tid - 128; e < R6_NX * R6_NX; e += 98) {
        const int r = e / R6_NX, c = e - r * R6_NX;
        A[pk * R6_NX * R6_NX + e] = -blk[r * R6_SZ + c];
      }
    }
    __syncthreads();
    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    {
      double z[13], zn = 0.0;
#pragma unroll
      for (int f = 0; f < 13; ++f) { z[f] = zv[f]; zn += z[f] * z[f]; }
      if (reg) {
        if (okv) {
          double dot = 0.0;
#pragma unroll
          for (int f = 0; f < 13; ++f) dot = fma(z[f], xv[f], dot);
          const double kv = kernel_epilogue(gv.kind, (zn + nv) - 2.0 * dot, gv.sigma2, gv.iso_scale);
#pragma unroll
          for (int c = 0; c < 3; ++c) acc[c] = fma(kv, av[c], acc[c]);
        }
      } else {
        for (int j = tid; j < gv.n; j += 256) {
          double dot = 0.0;
#pragma unroll
          for (int f = 0; f < 13; ++f) dot = fma(z[f], gv.Xs[(int64_t)j * 13 + f], dot);
          const double kv = kernel_epilogue(gv.kind, (zn + gv.Xn[j]) - 2.0 * dot, gv.sigma2, gv.iso_scale);
#pragma unroll
          for (int c = 0; c < 3; ++c) acc[c] = fma(kv, gv.alphaT[(int64_t)c * gv.n + j], acc[c]);
        }
      }
    }
    {
      double z[12], zn = 0.0;
#pragma unroll
      for (int f = 0; f < 12; ++f) { z[f] = zw[f]; zn += z[f] * z[f]; }
      if (reg) {
        if (okw) {
          double dot = 0.0;
#pragma unroll
          for (int f = 0; f < 12; ++f) dot = fma(z[f], xw[f], dot);
          const double kv = kernel_epilogue(gw.kind, (zn + nw) - 2.0 * dot, gw.sigma2, gw.iso_scale);
#pragma unroll
          for (int c = 0; c < 3; ++c) acc[3 + c] = fma(kv, aw[c], acc[3 + c]);
        }
      } else {
        for (int j = tid; j < gw.n; j += 256) {
          double dot = 0.0;
#pragma unroll
          for (int f = 0; f < 12; ++f) dot = fma(z[f], gw.Xs[(int64_t)j * 12 + f], dot);
          const double kv = kernel_epilogue(gw.kind, (zn + gw.Xn[j]) - 2.0 * dot, gw.sigma2, gw.iso_scale);
#pragma unroll
          for (int c = 0; c < 3; ++c) acc[3 + c] = fma(kv, gw.alphaT[(int64_t)c * gw.n + j], acc[3 + c]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 6; ++c)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc[c] += __shfl_xor(acc[c], o);
    if (lane == 0)
      for (int c = 0; c < 6; ++c) red[wave][c] = acc[c];
    __syncthreads();
    if (tid == 0) {
      double d[6];
      for (int c = 0; c < 6; ++c) {
        const double m = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
        const GpView &g = c < 3 ? gv : gw;
        d[c] = m * g.ystd[c % 3] + g.ymean[c % 3];
      }
      double xn[R6_NX];
      for (int i = 0; i < R6_NX; ++i) xn[i] = sxn[i];
      for (int c = 0; c < 3; ++c) {
        xn[4 + c] = xn[4 + c] + d[c] * dt;
        xn[11 + c] = xn[11 + c] + d[3 + c] * dt;
      }
      for (int i = 0; i < R6_NX; ++i) {
        sx[i] = xn[i];
        means[((int64_t)b * (N + 1) + k + 1) * R6_NX + i] = xn[i];
      }
    } else if (!uc && tid >= 1 && tid <= R6_NU && k + 1 < N) {
      sug[tid - 1] = U[(pk + 1) * R6_NU + tid - 1];  // the next step's controls (long horizons)
    }
    __syncthreads();
  }
}

// q_k = var dt^2 on the velocity rows 4-6 (d_v) and the rate rows 11-13 (d_omega)
__global__ void k_uprop6_q(int P, double dt2, const double *__restrict__ vv, const double *__restrict__ vw,
                           double *__restrict__ q) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= P) return;
  for (int i = 0; i < R6_NX; ++i) {
    double v = 0.0;
    if (i >= 4 && i < 7) v = vv[(int64_t)j * 3 + i - 4] * dt2;
    if (i >= 11) v = vw[(int64_t)j * 3 + i - 11] * dt2;
    q[(int64_t)j * R6_NX + i] = v;
  }
}

extern "C" int gpmpc_uprop6_linear(gpmpc_ctx *ctx, void *gp_v, void *gp_w, int exact, const double *rocket,
                                   int batch, int N, double dt, const double *x0, const double *U,
                                   const double *S0, double s0_diag, double *means, double *covs) {
  GPMPC_CHECK_ARG(ctx && gp_v && gp_w && rocket && x0 && U && means && covs && batch >= 0 && N >= 0);
  const GpView gv = exact ? gp_view((gpmpc_gp *)gp_v) : fitc_view((gpmpc_fitc *)gp_v);
  const GpView gw = exact ? gp_view((gpmpc_gp *)gp_w) : fitc_view((gpmpc_fitc *)gp_w);
  if (gv.d != 13 || gw.d != 12 || gv.n_out != 3 || gw.n_out != 3 || gv.kind == GPMPC_KPROG ||
      gw.kind == GPMPC_KPROG) {
    gpmpc_set_error("uprop6_linear: needs the StructuredRocketGP pair (13 / 12 features, 3 outputs, leaf kernels)");
    return -2;
  }
  // rocket: J_B (9, row-major), r_T_B (3), g_I (3), alpha, g0
  R6Rocket rk{};
  double Jd[3], Jf[9] = {}, Ji[9] = {};
  bool joff = false;
  const double jdiag[3] = {rocket[0], rocket[4], rocket[8]};
  if (r6_inertia(rocket, jdiag, Jd, Jf, Ji, joff)) return -2;
  for (int i = 0; i < 3; ++i) { rk.J[i] = Jd[i]; rk.rT[i] = rocket[9 + i]; rk.gI[i] = rocket[12 + i]; }
  for (int i = 0; i < 9; ++i) { rk.Jf[i] = Jf[i]; rk.Ji[i] = Ji[i]; }
  rk.full = joff;
  rk.alpha = rocket[15];
  rk.g0 = rocket[16];
  if (batch == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const size_t B = batch, P = B * N;
  DevBuf dQv, dQw, dA, dq, mv, vv, mw, vw;
  GPMPC_HIP(dQv.alloc(s, sizeof(double) * (P * 13 + 1)));
  GPMPC_HIP(dQw.alloc(s, sizeof(double) * (P * 12 + 1)));
  GPMPC_HIP(dA.alloc(s, sizeof(double) * (P * R6_NX * R6_NX + 1)));
  GPMPC_HIP(dq.alloc(s, sizeof(double) * (P * R6_NX + 1)));
  // inputs in one pinned upload, means and covariances in one read-back
  const size_t bytes = Stage::pad(8 * B * R6_NX) + Stage::pad(8 * P * R6_NU) +
                       (S0 ? Stage::pad(8 * B * R6_NX * R6_NX) : 0) + Stage::pad(8 * B * (N + 1) * R6_NX) +
                       Stage::pad(8 * B * (N + 1) * R6_NX * R6_NX);
  Stage sg(s, bytes);
  if (!sg.ok()) {
    gpmpc_set_error("uprop6_linear: staging buffers: out of memory");
    return -1;
  }
  const double *dx0 = sg.in(x0, B * R6_NX), *dU = sg.in(U, P * R6_NU);
  const double *dS0 = S0 ? sg.in(S0, B * R6_NX * R6_NX) : nullptr;
  double *dmeans = sg.out(means, B * (N + 1) * R6_NX), *dcov = sg.out(covs, B * (N + 1) * R6_NX * R6_NX);
  GPMPC_HIP(sg.upload());
  hipLaunchKernelGGL(k_uprop6_means, dim3(batch), dim3(256), 0, s, gv, gw, rk, N, dt, dx0, dU, dQv.as<double>(),
                     dQw.as<double>(), dA.as<double>(), dmeans);
  GPMPC_HIP(hipGetLastError());
  if (P) {
    for (DevBuf *d : {&mv, &vv, &mw, &vw}) GPMPC_HIP(d->alloc(s, sizeof(double) * P * 3));
    int rc = exact ? gp_posterior_dev(ctx, (gpmpc_gp *)gp_v, dQv.as<double>(), (int)P, mv.as<double>(), vv.as<double>())
                   : fitc_posterior_dev(ctx, (gpmpc_fitc *)gp_v, dQv.as<double>(), (int)P, mv.as<double>(),
                                        vv.as<double>());
    if (rc) return rc;
    rc = exact ? gp_posterior_dev(ctx, (gpmpc_gp *)gp_w, dQw.as<double>(), (int)P, mw.as<double>(), vw.as<double>())
               : fitc_posterior_dev(ctx, (gpmpc_fitc *)gp_w, dQw.as<double>(), (int)P, mw.as<double>(), vw.as<double>());
    if (rc) return rc;
    hipLaunchKernelGGL(k_uprop6_q, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, (int)P, dt * dt,
                       vv.as<double>(), vw.as<double>(), dq.as<double>());
    GPMPC_HIP(hipGetLastError());
  }
  const int rc = gpmpc_cov_propagate_dev(ctx, batch, N, R6_NX, dA.as<double>(), dq.as<double>(), dS0, s0_diag, dcov);
  if (rc) return rc;
  GPMPC_HIP(sg.download());
  return 0;
}
