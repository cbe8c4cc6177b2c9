// fleet.hip -- a batch of closed-loop 3-DoF GP-MPC landings, device-resident.
//
// One control step for every landing b:
//   1. k_fleet_queries   Simple3DoF features (features.py:403-444) of the N
//                        horizon points of b's linearisation trajectory
//                        (X_lin, U_lin = shifted previous solution: RTI), scaled
//                        by the kernel lengthscales;
//   2. GP posterior      K* = k(Z*, X) (gram kernel), mean = K* alpha and
//                        var = sigma2 - |L^-1 K*^T|^2 on the FP64-MFMA GEMM with
//                        fused sum-of-squares epilogue (gemm.hip) -- all B*N
//                        queries in one batched pass over one shared factor;
//   3. k_fleet_control   one workgroup per landing: Monte-Carlo termination
//                        checks (monte_carlo.py:455-488), target (monte_carlo.py
//                        :497-500 or fixed), RTI QP assembly with analytic
//                        Jacobians (osqp_rti.py:656-710) and the GP mean on the
//                        velocity rows of c_k with the correct sign (gp_mpc.py
//                        :309-314, 410-411), the OSQP-style ADMM of
//                        qp_device.h, the plant step (nominal Euler + the aero
//                        residual the GP learns) and the warm-start shift.
#include "internal.h"
#include "gemm.h"
#include "qp.h"
#include "fleet_qp.h"
#include <mutex>
#include <vector>
#include <algorithm>

#ifndef FQ_KNS
#define FQ_KNS fq_narrow
#endif
#define NX 7
#define NU 3
#define NFEAT 11
#define DYN_NNZ 26

#ifndef FLEET_WIDE_TU  // (fleet_wide.hip compiles only the control kernel below)
struct gpmpc_fleet {
  gpmpc_ctx *ctx = nullptr;
  gpmpc_gp *gp = nullptr;
  gpmpc_fleet_config cfg{};
  int B = 0, N = 0, n = 0, m = 0;
  int gp_n = 0;  // training rows of the GP when the GP scratch was sized
  // upper bound on the running landings, refreshed whenever the host reads the
  // records (landings only terminate between resets): with the dispatch order
  // putting running landings first, the GP posterior and the control launch
  // cover only the first n_active slots
  int n_active = 0;
  QPPatternHost pat;
  DevBuf x, Xw, Uw, ysc, rho, rec, xt;      // landing state
  DevBuf Q, Qn, Ks, part, meanT, mean, var;  // GP scratch
  DevBuf order, lastit;                      // dispatch order: longest predicted solve first
  unsigned long long *stamps = nullptr;      // diagnostic (gpmpc_fleet_set_stamps)
  unsigned long long *trace = nullptr;       // diagnostic (gpmpc_fleet_set_trace)
  bool use_order = true;                     // GPMPC_FLEET_ORDER=0 launches in landing order
  bool use_fq = true;                        // fleet-specialised solver (GPMPC_FLEET_SOLVER=0: generic)
  bool wide = false;                         // its 256-thread build (fleet_wide.hip): fleets of <= 1 landing per CU
  int alt_wave = 0;                          // GPMPC_FLEET_ALTWAVE=1: alternate the chain wave
  DevBuf claims;                             // per-CU chain-SIMD claims (k_fleet_control2)
  DevBuf sqp_done;                           // SQP mode: landing converged this control step
  int sqp_it = 0;                            // SQP mode: pass of the current control step
  unsigned epoch = 0;                        // control launches so far (claim generation)
  bool simd_pick = true;                     // GPMPC_FLEET_SIMD=0: chain on wave 0 always
  bool fuse_post = true;                     // GPMPC_FLEET_FUSE_POST=0: separate k_post_finish
  int64_t post_P = 0;                        // query rows / partial row tiles of the last
  int post_nrt = 0;                          //   posterior GEMM (fused finish reads them)
  // Every size-dependent path choice is made once, at creation, for plan_B landings (the
  // fleet's own size, or the whole Monte-Carlo fleet this one is a shard of): the kernels
  // differ in summation order, so choosing them from the running count or the shard size
  // would make a landing's bits depend on how many others fly beside it
  int plan_B = 0;
  int post_kind = 0;                         // posterior GEMM kernel (gemm_sumsq_kind at plan_B N)
  bool post_few = false;                     // queries + K* in one launch (<= 64 planned query rows)
  // a sparse GP (FITC or VFE, gpmpc_fleet_create_fitc) instead of the exact one: the
  // posterior is K*u against the inducing rows, mean K*u alpha as the reference writes it
  // (sparse_gp.py:280-283), variance sigma2 - |L_uu^-1 k*|^2 + |W2 k*|^2
  gpmpc_fitc *fitc = nullptr;
  DevBuf part2;                              // |W2 k*|^2 partials
  int post_kind2 = 0, post_nrt2 = 0;
};

// the GP the fleet reads: its exact GP, or the sparse one's inducing-point view
static GpView fleet_view(const gpmpc_fleet *f) { return f->fitc ? fitc_view(f->fitc) : gp_view(f->gp); }

extern "C" int gpmpc_fleet_set_stamps(gpmpc_fleet *f, void *dev_u64x16) {
  GPMPC_CHECK_ARG(f);
  f->stamps = (unsigned long long *)dev_u64x16;
  return 0;
}

extern "C" int gpmpc_fleet_set_trace(gpmpc_fleet *f, void *dev_u64xbx4) {
  GPMPC_CHECK_ARG(f);
  f->trace = (unsigned long long *)dev_u64xbx4;
  return 0;
}

extern "C" void gpmpc_fleet_default_config(gpmpc_fleet_config *c) {
  c->horizon = 20;           // BASELINE config: N = 20
  c->dt = 0.1;               // MPCConfig.dt / SimulationConfig.dt
  c->target_mode = 1;        // solve protocol of MonteCarloSimulator (GPMPC surface)
  c->use_gp = 1;
  c->residual_model = 1;
  c->max_steps = 300;        // run_experiments.py SimulationConfig max_time 30 s / dt
  gpmpc_qp_default_settings(&c->qp);
  c->sqp_iters = 1;          // RTI; > 1: GPMPC.solve's loop (gp_mpc.py:296-345)
  c->sqp_tol = 1e-4;         // gp_mpc.py:343
  c->sqp_qp = c->qp;         // the SQP passes' QP settings: max_iter 0 = "the same as qp",
  c->sqp_qp.max_iter = 0;    // resolved at launch, so later edits of qp reach the passes too
}

// ---------------------------------------------------------------------------
// structural CSR of the 3-DoF MPC QP (unfiltered: SURVEY D3 zeros kept)
static void mpc_pattern(int N, std::vector<int> &rp, std::vector<int> &ci) {
  const int n = (N + 1) * NX + N * NU, m = NX * (N + 1) + n;
  rp.assign(1, 0);
  ci.clear();
  auto row = [&](std::initializer_list<int> cols) {
    for (int c : cols) ci.push_back(c);
    rp.push_back((int)ci.size());
  };
  for (int i = 0; i < NX; ++i) row({i});
  for (int k = 0; k < N; ++k) {
    const int o = k * (NX + NU), on = (k + 1) * (NX + NU);
    row({o + 0, o + 7, o + 8, o + 9, on + 0});  // mass: A00, B0j, -1
    row({o + 1, o + 4, on + 1});                // r: A_ii, dt, -1
    row({o + 2, o + 5, on + 2});
    row({o + 3, o + 6, on + 3});
    row({o + 0, o + 4, o + 7, on + 4});         // v: A_i0, A_ii, B, -1
    row({o + 0, o + 5, o + 8, on + 5});
    row({o + 0, o + 6, o + 9, on + 6});
  }
  for (int j = 0; j < n; ++j) row({j});
  (void)m;
}

#endif  // FLEET_WIDE_TU
__device__ __forceinline__ void features3(const double *x, const double *u, double *z) {
  // Simple3DoFFeatureExtractor.extract (features.py:403-444)
  const double vx = x[4], vy = x[5], vz = x[6], alt = x[1];
  const double speed = sqrt(vx * vx + vy * vy + vz * vz);
  const double rho = 1.225 * exp(-alt / 8500.0);
  const double qd = 0.5 * rho * speed * speed;
  const double tm = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
  z[0] = vx / 10.0; z[1] = vy / 10.0; z[2] = vz / 10.0; z[3] = speed / 10.0;
  z[4] = qd / (0.5 * 1.225 * 100.0);
  z[5] = u[0] / 10.0; z[6] = u[1] / 10.0; z[7] = u[2] / 10.0; z[8] = tm / 10.0;
  z[9] = alt / 100.0; z[10] = rho / 1.225;
}

// GPMPC.solve's loop: X_pred[0] = x0 (gp_mpc.py:263) -- before the first pass of
// a control step the unshifted plan's first point becomes the current state
#ifndef FLEET_WIDE_TU
__global__ void k_fleet_x0_to_plan(int B, int N, const double *__restrict__ x, const double *__restrict__ rec,
                                   double *__restrict__ Xw) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= B * NX) return;
  const int b = g / NX, i = g - b * NX;
  if (rec[(int64_t)b * GPMPC_REC_LEN] != 0.0) return;
  Xw[(int64_t)b * (N + 1) * NX + i] = x[g];
}

__global__ void k_fleet_queries(int B, int N, const double *__restrict__ Xw,
                                const double *__restrict__ Uw, const double *__restrict__ ls,
                                int iso, const int *__restrict__ order, double *__restrict__ Q,
                                double *__restrict__ Qn) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;  // = slot*N + k
  if (g >= B * N) return;
  const int sl = g / N, k = g - sl * N;
  const int b = order ? order[sl] : sl;
  double z[NFEAT];
  features3(Xw + ((int64_t)b * (N + 1) + k) * NX, Uw + ((int64_t)b * N + k) * NU, z);
  double s = 0.0;
#pragma unroll
  for (int f = 0; f < NFEAT; ++f) {
    const double v = iso ? z[f] : z[f] / ls[f];
    Q[(int64_t)g * NFEAT + f] = v;
    s += v * v;
  }
  Qn[g] = s;
}

// The queries and K* in one launch for a fleet of at most 64 query rows (one to three
// landings: the single-landing step): every workgroup forms all the rows' features in LDS
// (k_fleet_queries' arithmetic) and its 64 training columns of K* as k_gram does (same
// fma order, same kernel_epilogue: the same bits as the two-launch path).
__global__ __launch_bounds__(256) void k_fleet_queries_gram(int B, int N, const double *__restrict__ Xw,
                                                            const double *__restrict__ Uw,
                                                            const double *__restrict__ ls, int iso,
                                                            const int *__restrict__ order, int kind,
                                                            const double *__restrict__ Xs,
                                                            const double *__restrict__ Xn, int n, double sigma2,
                                                            double iso_scale, double *__restrict__ Ks) {
  __shared__ double sq[64][NFEAT + 1];
  __shared__ double sqn[64];
  const int P = B * N, tid = threadIdx.x;
  if (tid < P) {
    const int sl = tid / N, k = tid - sl * N;
    const int b = order ? order[sl] : sl;
    double z[NFEAT];
    features3(Xw + ((int64_t)b * (N + 1) + k) * NX, Uw + ((int64_t)b * N + k) * NU, z);
    double sn = 0.0;
#pragma unroll
    for (int f = 0; f < NFEAT; ++f) {
      const double v = iso ? z[f] : z[f] / ls[f];
      sq[tid][f] = v;
      sn += v * v;
    }
    sqn[tid] = sn;
  }
  __syncthreads();
  const int col = blockIdx.x * 64 + (tid & 63), rg = tid >> 6;
  if (col >= n) return;
  double bj[NFEAT];
#pragma unroll
  for (int k = 0; k < NFEAT; ++k) bj[k] = Xs[(int64_t)col * NFEAT + k];
  const double nbj = Xn[col];
  for (int rr = 0; rr < 16; ++rr) {
    const int row = rg * 16 + rr;
    if (row >= P) break;
    double dot = 0.0;
#pragma unroll
    for (int k = 0; k < NFEAT; ++k) dot = fma(sq[row][k], bj[k], dot);
    const double d2 = (sqn[row] + nbj) - 2.0 * dot;
    Ks[(int64_t)row * n + col] = kernel_epilogue(kind, d2, sigma2, iso_scale);
  }
}

#endif  // FLEET_WIDE_TU
// ---------------------------------------------------------------------------
__device__ __forceinline__ void plant_euler(const double *x, const double *u, double dt,
                                            double *o) {
  // nominal_mpc.py:585-605 (alpha = 1/(I_sp g0) = 1/30, g = [-1, 0, 0])
  const double tm = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
  o[0] = x[0] - dt * (1.0 / 30.0) * tm;
  o[1] = x[1] + dt * x[4];
  o[2] = x[2] + dt * x[5];
  o[3] = x[3] + dt * x[6];
  o[4] = x[4] + dt * (u[0] / x[0] + -1.0);
  o[5] = x[5] + dt * (u[1] / x[0] + 0.0);
  o[6] = x[6] + dt * (u[2] / x[0] + 0.0);
}

__device__ __forceinline__ void drag_residual(const double *x, double *d) {
  // experiments/dispersion.py:349-360: rho 0.02, Cd = A = 1, |v| > 1
  const double vx = x[4], vy = x[5], vz = x[6];
  const double sp = sqrt(vx * vx + vy * vy + vz * vz);
  if (sp > 1.0) {
    const double a = (0.5 * 0.02 * 1.0 * 1.0 * sp * sp) / x[0];
    d[0] = -a * (vx / sp); d[1] = -a * (vy / sp); d[2] = -a * (vz / sp);
  } else {
    d[0] = d[1] = d[2] = 0.0;
  }
}

__device__ __forceinline__ bool landing_ok(const double *x, double m0) {
  // LandingConstraints.check_landing (monte_carlo.py:54-104), run_experiments.py tolerances
  if (fabs(x[1]) > 1.0) return false;
  if (fabs(x[2]) > 5.0 || fabs(x[3]) > 5.0) return false;
  if (fabs(x[4]) > 3.0) return false;
  if (fabs(x[5]) > 1.0 || fabs(x[6]) > 1.0) return false;
  if (1.0 - x[0] / m0 > 1.0 - 0.05) return false;
  return true;
}

struct FleetArgs {
  QPPattern pt;
  QPSettingsDev st;
  int N, target_mode, use_gp, residual_model, max_steps;
  double dt;
  double *x, *Xw, *Uw, *ysc, *rho, *rec, *xt;
  const double *gmean;  // (B*N) x 3, row (slot or landing)*N + k
  int gp_by_slot;       // gmean rows follow the dispatch slot (order[]) instead of the landing
  const int *order;     // workgroup -> landing (longest predicted first), or null
  int alt_wave;         // fleet solver: odd workgroups run the KKT chain on wave 1
  // fused posterior finish (k_fleet_control2 only; null part: k_post_finish ran)
  const double *part, *meanT, *ymean, *ystd;
  double *mean_out, *var_out;
  double sigma2;
  int nrt;
  int64_t pld;          // leading dimension of part / meanT (P)
  const double *part2;  // a sparse GP's second partials |W2 k*|^2 (or null: exact GP)
  int nrt2;
  unsigned *claims;     // per-CU claimed chain SIMDs, (epoch << 8) | 4-bit mask (or null)
  unsigned epoch;       // this launch's claim generation (never 0)
  int *lastit;          // ADMM iterations of each landing's last solve
  unsigned long long *stamps;  // diagnostic phase cycles of block 0 (or null)
  unsigned long long *trace;   // diagnostic per-landing placement/timing (or null)
  // SQP pass of GPMPC.solve's loop (gp_mpc.py:296-345; sqp = 0: RTI)
  int sqp, sqp_first, sqp_last;
  double sqp_tol;
  int *sqp_done;               // landing converged in an earlier pass of this control step
};

// The latent variance of query row q from the SUMSQ partials (k_post_finish / k_fitc_finish
// arithmetic): exact GP sigma2 - |L^-1 k*|^2 (exact_gp.py:256-266); a sparse GP (FITC / VFE,
// one predict body, sparse_gp.py:285-301) sigma2 - |L_uu^-1 k*|^2 + |L_B^-1 L_uu^-1 k*|^2
__device__ __forceinline__ double fleet_latent_var(const FleetArgs &a, int64_t q) {
  double ss = 0.0;
  for (int t = 0; t < a.nrt; ++t) ss += a.part[(int64_t)t * a.pld + q];
  double lat;
  if (a.part2) {
    double sw = 0.0;
    for (int t = 0; t < a.nrt2; ++t) sw += a.part2[(int64_t)t * a.pld + q];
    lat = a.sigma2 - ss + sw;
  } else {
    lat = a.sigma2 - ss;
  }
  return lat > 1e-10 ? lat : 1e-10;
}

// the 256-thread build of k_fleet_control2 (fleet_wide.hip)
hipError_t launch_fleet_control_wide(hipStream_t s, int nb, const FleetArgs &a, bool stamps);

#ifndef FLEET_WIDE_TU
__global__ __launch_bounds__(256) void k_fleet_control(FleetArgs a) {
  __shared__ QPSmemStd s;
  __shared__ double sx[NX], st_tgt[NX];
  __shared__ int s_out;
  const int b = a.order ? a.order[blockIdx.x] : (int)blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int N = a.N, n = a.pt.n, m = a.pt.m;
  const double dt = a.dt;
  double *rec = a.rec + (int64_t)b * GPMPC_REC_LEN;
  if (rec[0] != 0.0) return;  // terminated landing
  if (a.sqp && !a.sqp_first && a.sqp_done[b]) return;  // converged in an earlier SQP pass
  QPStamps T;
  T.out = (b == 0) ? a.stamps : nullptr;
  T.start();
  if (a.trace && tid == 0) {
    unsigned long long *tr = a.trace + (int64_t)b * 4;
    tr[0] = __builtin_amdgcn_s_memrealtime();
    tr[2] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID: wave, simd, cu, sh, se
    tr[3] = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
  }
  double *x = a.x + (int64_t)b * NX;
  double *Xw = a.Xw + (int64_t)b * (N + 1) * NX;
  double *Uw = a.Uw + (int64_t)b * N * NU;
  if (tid < NX) sx[tid] = x[tid];
  __syncthreads();
  // ---- termination checks at the top of the step (monte_carlo.py:458-488)
  if (tid == 0) {
    int out = 0;
    const double m0 = rec[13];
    bool div = false;
    for (int i = 0; i < NX; ++i) div = div || !(fabs(sx[i]) <= 1e6);
    if (a.sqp && !a.sqp_first) out = 0;                         // later SQP passes: checks done
    else if ((int)rec[1] >= a.max_steps) out = 5;               // TIMEOUT
    else if (sx[1] < 0.0) out = 2;                              // CRASH
    else if (sx[0] <= 1.0 + 0.01) out = 3;                      // FUEL_EXHAUSTED
    else if (div) out = 6;                                      // DIVERGENCE
    else if (sx[1] < 1.0 && fabs(sx[4]) < 5.0) out = landing_ok(sx, m0) ? 1 : 4;
    if (a.sqp && a.sqp_first) a.sqp_done[b] = 0;
    s_out = out;
    // target: incremental (monte_carlo.py:497-500) or fixed
    for (int i = 0; i < NX; ++i) st_tgt[i] = a.target_mode ? sx[i] : a.xt[(int64_t)b * NX + i];
    if (a.target_mode) {
      st_tgt[4] = st_tgt[5] = st_tgt[6] = 0.0;
      st_tgt[1] = fmax(0.5, sx[1] - 2.0);
    }
  }
  __syncthreads();
  if (s_out) {
    if (tid == 0) {
      rec[0] = s_out;
      rec[2] = rec[13] - sx[0];
      for (int i = 0; i < NX; ++i) rec[4 + i] = sx[i];
    }
    return;
  }
  // ---- QP data (osqp_rti.py:203-372 with the GPMPC sign), straight into LDS
  const int Nv = N * (NX + NU);
  for (int j = tid; j < n; j += nt) {
    double p, qq;
    if (j >= Nv) {               // x_N block: Q_f = 10 Q
      const int i = j - Nv;
      const double qd = (i == 0) ? 0.0 : (i < 4 ? 100.0 : 10.0);
      p = qd; qq = -qd * st_tgt[i];
    } else {
      const int k = j / (NX + NU), i = j - k * (NX + NU);
      if (i < NX) {
        const double qd = (i == 0) ? 0.0 : (i < 4 ? 10.0 : 1.0);
        p = qd; qq = -qd * st_tgt[i];
      } else {
        p = 0.01; qq = 0.0;
      }
      (void)k;
    }
    s.P[j] = p;
    s.q[j] = qq;
    // warm start / linearisation point vector
    if (j >= Nv) s.x[j] = Xw[N * NX + (j - Nv)];
    else {
      const int k = j / (NX + NU), i = j - k * (NX + NU);
      s.x[j] = (i < NX) ? Xw[k * NX + i] : Uw[k * NU + (i - NX)];
    }
  }
  // x0 rows and bound rows
  for (int r = tid; r < m; r += nt) {
    if (r < NX) {
      s.A[r] = 1.0;
      s.l[r] = sx[r];
      s.u[r] = sx[r];
    } else if (r >= NX * (N + 1)) {
      const int j = r - NX * (N + 1);
      s.A[NX + N * DYN_NNZ + j] = 1.0;
      double lo, hi;
      const int i = (j >= Nv) ? j - Nv : j % (NX + NU);
      if (i < NX) {
        const double xmin[NX] = {-INFINITY, -100, -100, -100, -50, -50, -50};
        const double xmax[NX] = {INFINITY, 500, 100, 100, 50, 50, 50};
        lo = xmin[i]; hi = xmax[i];
      } else {
        const double umin[NU] = {0.3, -5, -5}, umax[NU] = {5, 5, 5};
        lo = umin[i - NX]; hi = umax[i - NX];
      }
      s.l[r] = lo;
      s.u[r] = hi;
    }
  }
  // dynamics blocks: one thread per stage k
  for (int k = tid; k < N; k += nt) {
    const double *xk = Xw + k * NX;
    const double *uk = Uw + k * NU;
    const double mk = xk[0], tx = uk[0], ty = uk[1], tz = uk[2];
    const double tm = sqrt(tx * tx + ty * ty + tz * tz) + 1e-10;
    const double al = 1.0 / 30.0;
    // FastRTI3DoF._linearize (osqp_rti.py:656-710)
    const double a40 = -tx / (mk * mk) * dt, a50 = -ty / (mk * mk) * dt, a60 = -tz / (mk * mk) * dt;
    const double b00 = -al * tx / tm * dt, b01 = -al * ty / tm * dt, b02 = -al * tz / tm * dt;
    const double bv = dt / mk;
    double *Ak = s.A + NX + k * DYN_NNZ;
    Ak[0] = 1.0; Ak[1] = b00; Ak[2] = b01; Ak[3] = b02; Ak[4] = -1.0;
    Ak[5] = 1.0; Ak[6] = dt; Ak[7] = -1.0;
    Ak[8] = 1.0; Ak[9] = dt; Ak[10] = -1.0;
    Ak[11] = 1.0; Ak[12] = dt; Ak[13] = -1.0;
    Ak[14] = a40; Ak[15] = 1.0; Ak[16] = bv; Ak[17] = -1.0;
    Ak[18] = a50; Ak[19] = 1.0; Ak[20] = bv; Ak[21] = -1.0;
    Ak[22] = a60; Ak[23] = 1.0; Ak[24] = bv; Ak[25] = -1.0;
    // c_k = f(x,u) - A x - B u (+ dt * GP mean on the velocity rows)
    double f[NX];
    plant_euler(xk, uk, dt, f);
    // (f - A x) - B u, as osqp_rti.py:340-341 evaluates it
    double ax[NX], bu[NX];
    ax[0] = xk[0];
    ax[1] = xk[1] + dt * xk[4];
    ax[2] = xk[2] + dt * xk[5];
    ax[3] = xk[3] + dt * xk[6];
    ax[4] = a40 * xk[0] + xk[4];
    ax[5] = a50 * xk[0] + xk[5];
    ax[6] = a60 * xk[0] + xk[6];
    bu[0] = b00 * tx + b01 * ty + b02 * tz;
    bu[1] = bu[2] = bu[3] = 0.0;
    bu[4] = bv * tx; bu[5] = bv * ty; bu[6] = bv * tz;
    const double *gm = a.gmean + ((int64_t)(a.gp_by_slot ? (int)blockIdx.x : b) * N + k) * 3;
    for (int i = 0; i < NX; ++i) {
      double c = (f[i] - ax[i]) - bu[i];
      if (a.use_gp && i >= 4) c += gm[i - 4] * dt;
      const int r = NX * (k + 1) + i;
      s.l[r] = -c;   // A x + B u - x+ = -c   <=>   x+ = A x + B u + c
      s.u[r] = -c;
    }
  }
  for (int r = tid; r < m; r += nt) s.y[r] = a.ysc[(int64_t)b * m + r];
  if (tid == 0) s.rho_s = a.rho[b];
  __syncthreads();
  T.mark(0);
  // ---- ADMM (qp_device.h)
  QPResult res = qp_solve(a.pt, s, a.st, &T);
  T.mark(7);
  const bool has = !res.factor_fail && (res.status == 1 || res.status == 2 || res.status == -2);
  // ---- solution, plant step, warm-start shift
  if (has) {
    for (int j = tid; j < n; j += nt) s.x[j] = s.D[j] * s.x[j];  // unscale
  }
  __syncthreads();
  if (!has && a.target_mode == 1) {  // solve protocol: failed solve -> DIVERGENCE
    if (tid == 0) {
      rec[0] = 6;
      rec[14] = res.factor_fail ? -100 : res.status;
      for (int i = 0; i < NX; ++i) rec[4 + i] = sx[i];
      rec[2] = rec[13] - sx[0];
    }
    return;
  }
  if (a.sqp) {
    // GPMPC.solve's loop (gp_mpc.py:336-353), as k_fleet_control2: the change of the
    // trajectory, X_pred <- X_new (no shift), stop below sqp_tol
    __shared__ double s_dm[4];
    double dm = 0.0;
    for (int j = tid; j < n; j += nt) {
      const int i = (j >= Nv) ? j - Nv : j % (NX + NU), k = j / (NX + NU);
      const double old = (j >= Nv) ? Xw[N * NX + i] : (i < NX ? Xw[k * NX + i] : Uw[k * NU + i - NX]);
      dm = fmax(dm, fabs(s.x[j] - old));
    }
    for (int o = 32; o > 0; o >>= 1) dm = fmax(dm, __shfl_xor(dm, o));
    if ((tid & 63) == 0) s_dm[tid >> 6] = dm;
    __syncthreads();  // (also orders every read of Xw / Uw before the writes)
    dm = s_dm[0];
    for (int w = 1; w < nt / 64; ++w) dm = fmax(dm, s_dm[w]);
    for (int e = tid; e < (N + 1) * NX; e += nt) {
      const int k = e / NX, i = e - k * NX;
      Xw[e] = s.x[(k == N) ? Nv + i : k * (NX + NU) + i];
    }
    for (int e = tid; e < N * NU; e += nt) {
      const int k = e / NU, i = e - k * NU;
      Uw[e] = s.x[k * (NX + NU) + NX + i];
    }
    for (int r = tid; r < m; r += nt) a.ysc[(int64_t)b * m + r] = s.y[r];
    if (tid == 0) {
      const bool conv = dm < a.sqp_tol;
      a.rho[b] = s.rho_s;
      rec[11] += res.iter;
      a.lastit[b] = res.iter;
      rec[12] += (res.status == 1) ? 1.0 : 0.0;
      rec[14] = res.status;
      rec[15] = s.rho_s;
      if (conv) {
        const double u0[NU] = {s.x[NX], s.x[NX + 1], s.x[NX + 2]};
        double xn[NX], dr[3];
        plant_euler(sx, u0, dt, xn);
        if (a.residual_model) {
          drag_residual(sx, dr);
          xn[4] += dr[0] * dt; xn[5] += dr[1] * dt; xn[6] += dr[2] * dt;
        }
        for (int i = 0; i < NX; ++i) x[i] = xn[i];
        rec[1] += 1.0;
        rec[3] = rec[1] * dt;
        rec[2] = rec[13] - xn[0];
        for (int i = 0; i < NX; ++i) rec[4 + i] = xn[i];
        a.sqp_done[b] = 1;
      } else if (a.sqp_last) {  // MPCSolution.success False -> DIVERGENCE (monte_carlo.py:506-508)
        rec[0] = 6;
        rec[2] = rec[13] - sx[0];
        for (int i = 0; i < NX; ++i) rec[4 + i] = sx[i];
      }
    }
    T.mark(7);
    T.flush();
    if (a.trace && tid == 0) a.trace[(int64_t)b * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    return;
  }
  if (has) {
    // shifted solution -> next linearisation point (X[1:], X[-1]), (U[1:], U[-1])
    for (int e = tid; e < (N + 1) * NX; e += nt) {
      const int k = e / NX, i = e - k * NX;
      const int ks = (k + 1 <= N) ? k + 1 : N;
      const int src = (ks == N) ? Nv + i : ks * (NX + NU) + i;
      Xw[e] = s.x[src];
    }
    for (int e = tid; e < N * NU; e += nt) {
      const int k = e / NU, i = e - k * NU;
      const int ks = (k + 1 < N) ? k + 1 : N - 1;
      Uw[e] = s.x[ks * (NX + NU) + NX + i];
    }
    for (int r = tid; r < m; r += nt) a.ysc[(int64_t)b * m + r] = s.y[r];
  }
  if (tid == 0) {
    double u0[NU];
    if (has) {
      u0[0] = s.x[NX]; u0[1] = s.x[NX + 1]; u0[2] = s.x[NX + 2];
    } else {  // step protocol fallback: shifted previous plan (osqp_rti.py:546-552)
      u0[0] = Uw[0]; u0[1] = Uw[1]; u0[2] = Uw[2];
    }
    double xn[NX], dr[3];
    plant_euler(sx, u0, dt, xn);
    if (a.residual_model) {
      drag_residual(sx, dr);
      xn[4] += dr[0] * dt; xn[5] += dr[1] * dt; xn[6] += dr[2] * dt;
    }
    for (int i = 0; i < NX; ++i) x[i] = xn[i];
    a.rho[b] = s.rho_s;
    rec[1] += 1.0;
    rec[3] = rec[1] * dt;
    rec[2] = rec[13] - xn[0];
    for (int i = 0; i < NX; ++i) rec[4 + i] = xn[i];
    rec[11] += res.iter;
    a.lastit[b] = res.iter;
    rec[12] += (res.status == 1) ? 1.0 : 0.0;
    rec[14] = res.factor_fail ? -100 : res.status;
    rec[15] = s.rho_s;
  }
  T.mark(7);
  T.flush();
  if (a.trace && tid == 0) a.trace[(int64_t)b * 4 + 1] = __builtin_amdgcn_s_memrealtime();
}

// initial linearisation point: X linear to the target, U hover (osqp_rti.py:425-446)
// The same control step on the fleet-specialised solver (fleet_qp.h): 128
// threads and ~37 KB of LDS per landing, four landings per CU.  Assembly goes
// straight into the owners' registers; results and the plant step as above.
// STAMPS: the diagnostic phase-cycle instance (gpmpc_fleet_set_stamps); the
// production instance has no stamp code or state at all.
#endif  // FLEET_WIDE_TU
// the control kernel lives in a namespace of its build: fleet.hip (128 threads, four
// landings per CU) and fleet_wide.hip (256 threads, one wave per SIMD) each have one
namespace FQ_KNS {
template <bool STAMPS>
#ifndef FQ_WPE
#define FQ_WPE FQ_NW  // waves per SIMD the register budget is sized for
#endif
__global__ __launch_bounds__(FQ_T) __attribute__((amdgpu_waves_per_eu(FQ_WPE, FQ_WPE))) void k_fleet_control2(FleetArgs a) {
  __shared__ FleetSmem s;
  __shared__ double sx[NX], st_tgt[NX];
  __shared__ int s_out;
  const int b = a.order ? a.order[blockIdx.x] : (int)blockIdx.x, tid = threadIdx.x;
  const int N = a.N, n = a.pt.n, m = a.pt.m;
  const double dt = a.dt;
  double *rec = a.rec + (int64_t)b * GPMPC_REC_LEN;
  // The posterior finish of this slot's queries (k_post_finish's arithmetic) for a landing
  // that returns before its QP assembly: every launched slot is finished, so a slot never
  // keeps the values another landing left in it at an earlier step; the
  // posterior is the one at this landing's linearisation trajectory, as on the unfused path
  auto finish_only = [&]() {
    if (!(a.part && a.use_gp)) return;
    for (int k = tid; k < N; k += FQ_T) {
      const int64_t q = (int64_t)(a.gp_by_slot ? (int)blockIdx.x : b) * N + k;
      const double lat = fleet_latent_var(a, q);
      for (int c = 0; c < 3; ++c) {
        a.mean_out[q * 3 + c] = a.meanT[(int64_t)c * a.pld + q] * a.ystd[c] + a.ymean[c];
        a.var_out[q * 3 + c] = lat * a.ystd[c] * a.ystd[c];
      }
    }
  };
  if (rec[0] != 0.0) {  // terminated landing
    finish_only();
    return;
  }
  if (a.sqp && !a.sqp_first && a.sqp_done[b]) {  // converged in an earlier SQP pass
    finish_only();
    return;
  }
  QPStamps T;
  T.out = (STAMPS && b == 0) ? a.stamps : nullptr;
  T.start();
  if (a.trace && (tid & 63) == 0 && tid < 128) {
    // [0] start, [1] end (realtime), [2] wave 0 HW_ID | XCC_ID << 32, [3] wave 1 the same
    unsigned long long *tr = a.trace + (int64_t)b * 4;
    if (tid == 0) tr[0] = __builtin_amdgcn_s_memrealtime();
    tr[2 + (tid >> 6)] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                         ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
  }
  double *x = a.x + (int64_t)b * NX;
  double *Xw = a.Xw + (int64_t)b * (N + 1) * NX;
  double *Uw = a.Uw + (int64_t)b * N * NU;
  // Chain wave: the two waves of a workgroup sit on two SIMDs, and the four
  // workgroups of a CU fill each SIMD with two waves.  Two KKT chains on one
  // SIMD slow both (the slowest landings, which set the kernel time, are the
  // ones sharing), so each workgroup claims a SIMD of its CU for its chain:
  // wave 0's if no earlier workgroup of this launch took it, else wave 1's.
  __shared__ int s_simd[FQ_NW], s_cw;
  if (a.claims && (tid & 63) == 0) s_simd[tid >> 6] = (__builtin_amdgcn_s_getreg(4 | (31 << 11)) >> 4) & 3;
  if (tid < NX) sx[tid] = x[tid];
  __syncthreads();
  if (tid == 0) {
    int cw0 = a.alt_wave ? (int)(blockIdx.x & 1) : 0;
    if (a.claims) {
      const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
      const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 15;
      const unsigned key = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
      unsigned *cl = a.claims + key;
      unsigned old = __hip_atomic_load(cl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int tries = 0; tries < 16; ++tries) {  // bounded: contention is at most 4 workgroups
        const unsigned mask = (old >> 8) == a.epoch ? (old & 15u) : 0u;
        int w = 0;  // the first wave whose SIMD no earlier workgroup claimed (else wave 0)
        while (w < FQ_NW && (mask & (1u << s_simd[w]))) ++w;
        if (w == FQ_NW) w = 0;
        const unsigned nv = (a.epoch << 8) | mask | (1u << s_simd[w]);
        const unsigned prev = atomicCAS(cl, old, nv);
        if (prev == old) { cw0 = w; break; }
        old = prev;
      }
    }
    s_cw = cw0;
  }
  if (tid == 0) {  // termination checks (monte_carlo.py:458-488), as k_fleet_control
    int out = 0;
    const double m0 = rec[13];
    bool div = false;
    for (int i = 0; i < NX; ++i) div = div || !(fabs(sx[i]) <= 1e6);
    if (a.sqp && !a.sqp_first) out = 0;  // later SQP passes: same state, checks done
    else if ((int)rec[1] >= a.max_steps) out = 5;
    else if (sx[1] < 0.0) out = 2;
    else if (sx[0] <= 1.0 + 0.01) out = 3;
    else if (div) out = 6;
    else if (sx[1] < 1.0 && fabs(sx[4]) < 5.0) out = landing_ok(sx, m0) ? 1 : 4;
    if (a.sqp && a.sqp_first) a.sqp_done[b] = 0;
    s_out = out;
    for (int i = 0; i < NX; ++i) st_tgt[i] = a.target_mode ? sx[i] : a.xt[(int64_t)b * NX + i];
    if (a.target_mode) {
      st_tgt[4] = st_tgt[5] = st_tgt[6] = 0.0;
      st_tgt[1] = fmax(0.5, sx[1] - 2.0);
    }
  }
  __syncthreads();
  if (s_out) {
    if (tid == 0) {
      rec[0] = s_out;
      rec[2] = rec[13] - sx[0];
      for (int i = 0; i < NX; ++i) rec[4 + i] = sx[i];
    }
    finish_only();
    return;
  }
  FleetRegs R;
  fq_init_pattern(a.pt, R, n);
  const int Nv = N * (NX + NU);
  const int MD = NX * (N + 1);
  // ---- QP data (osqp_rti.py:203-372 with the GPMPC sign): variables + bound rows
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (!R.vok[h]) continue;
    const int j = R.vj[h];
    double p, qq, lo, hi, xw;
    const int i = (j >= Nv) ? j - Nv : j % (NX + NU);
    if (j >= Nv) {
      const double qd = (i == 0) ? 0.0 : (i < 4 ? 100.0 : 10.0);
      p = qd; qq = -qd * st_tgt[i];
      xw = Xw[N * NX + i];
    } else {
      const int k = j / (NX + NU);
      if (i < NX) {
        const double qd = (i == 0) ? 0.0 : (i < 4 ? 10.0 : 1.0);
        p = qd; qq = -qd * st_tgt[i];
        xw = Xw[k * NX + i];
      } else {
        p = 0.01; qq = 0.0;
        xw = Uw[k * NU + (i - NX)];
      }
    }
    if (i < NX) {
      const double xmin[NX] = {-INFINITY, -100, -100, -100, -50, -50, -50};
      const double xmax[NX] = {INFINITY, 500, 100, 100, 50, 50, 50};
      lo = xmin[i]; hi = xmax[i];
    } else {
      const double umin[NU] = {0.3, -5, -5}, umax[NU] = {5, 5, 5};
      lo = umin[i - NX]; hi = umax[i - NX];
    }
    R.P[h] = p; R.q[h] = qq; R.x[h] = xw;
    R.Ab[h] = 1.0; R.lb[h] = lo; R.ub[h] = hi;
    R.yb_(h) = a.ysc[(int64_t)b * m + MD + j];
  }
  // dynamics rows: A values (one thread per stage) and c_k, staged in zt for the row owners
  for (int r = tid; r < NX; r += FQ_T) {
    s.A[r] = 1.0;
    s.zt[r] = sx[r];
  }
  for (int k = tid; k < N; k += FQ_T) {
    const double *xk = Xw + k * NX;
    const double *uk = Uw + k * NU;
    const double mk = xk[0], tx = uk[0], ty = uk[1], tz = uk[2];
    const double tm = sqrt(tx * tx + ty * ty + tz * tz) + 1e-10;
    const double al = 1.0 / 30.0;
    const double a40 = -tx / (mk * mk) * dt, a50 = -ty / (mk * mk) * dt, a60 = -tz / (mk * mk) * dt;
    const double b00 = -al * tx / tm * dt, b01 = -al * ty / tm * dt, b02 = -al * tz / tm * dt;
    const double bv = dt / mk;
    double *Ak = s.A + NX + k * DYN_NNZ;
    Ak[0] = 1.0; Ak[1] = b00; Ak[2] = b01; Ak[3] = b02; Ak[4] = -1.0;
    Ak[5] = 1.0; Ak[6] = dt; Ak[7] = -1.0;
    Ak[8] = 1.0; Ak[9] = dt; Ak[10] = -1.0;
    Ak[11] = 1.0; Ak[12] = dt; Ak[13] = -1.0;
    Ak[14] = a40; Ak[15] = 1.0; Ak[16] = bv; Ak[17] = -1.0;
    Ak[18] = a50; Ak[19] = 1.0; Ak[20] = bv; Ak[21] = -1.0;
    Ak[22] = a60; Ak[23] = 1.0; Ak[24] = bv; Ak[25] = -1.0;
    double f[NX];
    plant_euler(xk, uk, dt, f);
    double ax[NX], bu[NX];
    ax[0] = xk[0];
    ax[1] = xk[1] + dt * xk[4];
    ax[2] = xk[2] + dt * xk[5];
    ax[3] = xk[3] + dt * xk[6];
    ax[4] = a40 * xk[0] + xk[4];
    ax[5] = a50 * xk[0] + xk[5];
    ax[6] = a60 * xk[0] + xk[6];
    bu[0] = b00 * tx + b01 * ty + b02 * tz;
    bu[1] = bu[2] = bu[3] = 0.0;
    bu[4] = bv * tx; bu[5] = bv * ty; bu[6] = bv * tz;
    const int64_t q = (int64_t)(a.gp_by_slot ? (int)blockIdx.x : b) * N + k;  // query row
    double gm[3];
    if (a.part && a.use_gp) {
      // the posterior finish of this landing's query (k_post_finish / k_fitc_finish arithmetic)
      const double lat = fleet_latent_var(a, q);
      for (int c = 0; c < 3; ++c) {
        gm[c] = a.meanT[(int64_t)c * a.pld + q] * a.ystd[c] + a.ymean[c];
        a.mean_out[q * 3 + c] = gm[c];
        a.var_out[q * 3 + c] = lat * a.ystd[c] * a.ystd[c];
      }
    } else {
      for (int c = 0; c < 3; ++c) gm[c] = a.gmean[q * 3 + c];
    }
    for (int i = 0; i < NX; ++i) {
      double c = (f[i] - ax[i]) - bu[i];
      if (a.use_gp && i >= 4) c += gm[i - 4] * dt;
      s.zt[NX * (k + 1) + i] = -c;
    }
  }
  if (tid == 0) s.rho_s = a.rho[b];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < FQ_H; ++h)
    if (R.rok[h]) {
      R.ur(h) = s.zt[R.rr[h]];  // l = u
      R.yr(h) = a.ysc[(int64_t)b * m + R.rr[h]];
    }
  __syncthreads();
  T.mark(0);
  QPResult res = fq_solve(a.pt, s, R, a.st, &T, s_cw);
  T.mark(7);
  const bool has = !res.factor_fail && (res.status == 1 || res.status == 2 || res.status == -2);
  if (has) {
#pragma unroll
    for (int h = 0; h < FQ_H; ++h)
      if (R.vok[h]) s.rhs[R.vj[h]] = R.D[h] * R.x[h];  // unscaled solution
  }
  __syncthreads();
  if (!has && a.target_mode == 1) {
    if (tid == 0) {
      rec[0] = 6;
      rec[14] = res.factor_fail ? -100 : res.status;
      for (int i = 0; i < NX; ++i) rec[4 + i] = sx[i];
      rec[2] = rec[13] - sx[0];
    }
    return;
  }
  if (a.sqp) {
    // GPMPC.solve's loop (gp_mpc.py:336-353): the change of the trajectory,
    // X_pred <- X_new (no shift), stop below sqp_tol
    double dm[1] = {0.0};
#pragma unroll
    for (int h = 0; h < FQ_H; ++h)
      if (R.vok[h]) {
        const int j = R.vj[h], i = (j >= Nv) ? j - Nv : j % (NX + NU), k = j / (NX + NU);
        const double old = (j >= Nv) ? Xw[N * NX + i] : (i < NX ? Xw[k * NX + i] : Uw[k * NU + i - NX]);
        dm[0] = fmax(dm[0], fabs(s.rhs[j] - old));
      }
    fq_max<1>(dm, s.red);  // (its barriers order the reads of Xw / Uw before the writes)
    for (int e = tid; e < (N + 1) * NX; e += FQ_T) {
      const int k = e / NX, i = e - k * NX;
      Xw[e] = s.rhs[(k == N) ? Nv + i : k * (NX + NU) + i];
    }
    for (int e = tid; e < N * NU; e += FQ_T) {
      const int k = e / NU, i = e - k * NU;
      Uw[e] = s.rhs[k * (NX + NU) + NX + i];
    }
#pragma unroll
    for (int h = 0; h < FQ_H; ++h) {
      if (R.rok[h]) a.ysc[(int64_t)b * m + R.rr[h]] = R.yr(h);
      if (R.vok[h]) a.ysc[(int64_t)b * m + MD + R.vj[h]] = R.yb_(h);
    }
    if (tid == 0) {
      const bool conv = dm[0] < a.sqp_tol;
      a.rho[b] = s.rho_s;
      rec[11] += res.iter;
      a.lastit[b] = res.iter;
      rec[12] += (res.status == 1) ? 1.0 : 0.0;
      rec[14] = res.status;
      rec[15] = s.rho_s;
      if (conv) {
        const double u0[NU] = {s.rhs[NX], s.rhs[NX + 1], s.rhs[NX + 2]};
        double xn[NX], dr[3];
        plant_euler(sx, u0, dt, xn);
        if (a.residual_model) {
          drag_residual(sx, dr);
          xn[4] += dr[0] * dt; xn[5] += dr[1] * dt; xn[6] += dr[2] * dt;
        }
        for (int i = 0; i < NX; ++i) x[i] = xn[i];
        rec[1] += 1.0;
        rec[3] = rec[1] * dt;
        rec[2] = rec[13] - xn[0];
        for (int i = 0; i < NX; ++i) rec[4 + i] = xn[i];
        a.sqp_done[b] = 1;
      } else if (a.sqp_last) {  // MPCSolution.success False -> DIVERGENCE (monte_carlo.py:506-508)
        rec[0] = 6;
        rec[2] = rec[13] - sx[0];
        for (int i = 0; i < NX; ++i) rec[4 + i] = sx[i];
      }
    }
    T.mark(7);
    T.flush();
    if (a.trace && tid == 0) a.trace[(int64_t)b * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    return;
  }
  if (has) {
    for (int e = tid; e < (N + 1) * NX; e += FQ_T) {
      const int k = e / NX, i = e - k * NX;
      const int ks = (k + 1 <= N) ? k + 1 : N;
      const int src = (ks == N) ? Nv + i : ks * (NX + NU) + i;
      Xw[e] = s.rhs[src];
    }
    for (int e = tid; e < N * NU; e += FQ_T) {
      const int k = e / NU, i = e - k * NU;
      const int ks = (k + 1 < N) ? k + 1 : N - 1;
      Uw[e] = s.rhs[ks * (NX + NU) + NX + i];
    }
#pragma unroll
    for (int h = 0; h < FQ_H; ++h) {
      if (R.rok[h]) a.ysc[(int64_t)b * m + R.rr[h]] = R.yr(h);
      if (R.vok[h]) a.ysc[(int64_t)b * m + MD + R.vj[h]] = R.yb_(h);
    }
  }
  if (tid == 0) {
    double u0[NU];
    if (has) {
      u0[0] = s.rhs[NX]; u0[1] = s.rhs[NX + 1]; u0[2] = s.rhs[NX + 2];
    } else {
      u0[0] = Uw[0]; u0[1] = Uw[1]; u0[2] = Uw[2];
    }
    double xn[NX], dr[3];
    plant_euler(sx, u0, dt, xn);
    if (a.residual_model) {
      drag_residual(sx, dr);
      xn[4] += dr[0] * dt; xn[5] += dr[1] * dt; xn[6] += dr[2] * dt;
    }
    for (int i = 0; i < NX; ++i) x[i] = xn[i];
    a.rho[b] = s.rho_s;
    rec[1] += 1.0;
    rec[3] = rec[1] * dt;
    rec[2] = rec[13] - xn[0];
    for (int i = 0; i < NX; ++i) rec[4 + i] = xn[i];
    rec[11] += res.iter;
    a.lastit[b] = res.iter;
    rec[12] += (res.status == 1) ? 1.0 : 0.0;
    rec[14] = res.factor_fail ? -100 : res.status;
    rec[15] = s.rho_s;
  }
  T.mark(7);
  T.flush();
  if (a.trace && tid == 0) a.trace[(int64_t)b * 4 + 1] = __builtin_amdgcn_s_memrealtime();
}


// gpmpc_qp_solve_batched on this solver (qp.hip picks it): problems whose pattern is the
// fleet's MPC pattern at N = 20 (fleet_qp.h's fixed row layout: dynamics rows 0..MD-1 as
// equalities, then the identity bound rows) -- the host surface's QPWorkspace.solve.  The
// QP data come from global memory instead of the fleet's assembly; rho, the scaled y and
// the outputs are the generic kernel's (k_qp_batched), one problem per workgroup.
__global__ __launch_bounds__(FQ_T) __attribute__((amdgpu_waves_per_eu(FQ_WPE, FQ_WPE))) void k_qp_fleet(
    QPPattern pt, QPSettingsDev st, const double *__restrict__ Aval, const double *__restrict__ Pd,
    const double *__restrict__ q, const double *__restrict__ l, const double *__restrict__ u,
    const double *__restrict__ xws, double *rho, double *yst, double *xo, double *yo, int *iters, int *status,
    double *obj) {
  __shared__ FleetSmem s;
  const int b = blockIdx.x, tid = threadIdx.x, n = pt.n, m = pt.m;
  const double *Ab = Aval + (int64_t)b * pt.nnz;
  FleetRegs R;
  fq_init_pattern(pt, R, n);
  for (int e = tid; e < FQ_NNZD; e += FQ_T) s.A[e] = Ab[e];
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (!R.vok[h]) continue;
    const int j = R.vj[h];
    R.P[h] = Pd[(int64_t)b * n + j];
    R.q[h] = q[(int64_t)b * n + j];
    R.x[h] = xws ? xws[(int64_t)b * n + j] : 0.0;
    R.Ab[h] = Ab[FQ_NNZD + j];  // bound row MD + j: its one entry
    R.lb[h] = l[(int64_t)b * m + FQ_MD + j];
    R.ub[h] = u[(int64_t)b * m + FQ_MD + j];
    R.yb_(h) = yst[(int64_t)b * m + FQ_MD + j];
  }
#pragma unroll
  for (int h = 0; h < FQ_H; ++h)
    if (R.rok[h]) {
      R.ur(h) = l[(int64_t)b * m + R.rr[h]];  // l = u (checked by the host)
      R.yr(h) = yst[(int64_t)b * m + R.rr[h]];
    }
  if (tid == 0) s.rho_s = rho[b];
  __syncthreads();
  QPStamps T;
  const QPResult res = fq_solve(pt, s, R, st, &T, 0);
  if (res.factor_fail) {
    if (tid == 0) { status[b] = -100; iters[b] = 0; obj[b] = nan(""); }
    return;
  }
  const bool has = (res.status == 1 || res.status == 2 || res.status == -2);
  const double c = s.c;
#pragma unroll
  for (int h = 0; h < FQ_H; ++h) {
    if (R.vok[h]) {
      const int j = R.vj[h];
      xo[(int64_t)b * n + j] = has ? R.D[h] * R.x[h] : nan("");
      yo[(int64_t)b * m + FQ_MD + j] = has ? s.E[FQ_MD + j] * R.yb_(h) / c : nan("");
      yst[(int64_t)b * m + FQ_MD + j] = R.yb_(h);
    }
    if (R.rok[h]) {
      yo[(int64_t)b * m + R.rr[h]] = has ? s.E[R.rr[h]] * R.yr(h) / c : nan("");
      yst[(int64_t)b * m + R.rr[h]] = R.yr(h);
    }
  }
  if (tid == 0) {
    rho[b] = s.rho_s;
    iters[b] = res.iter;
    status[b] = res.status;
    obj[b] = has ? res.obj : nan("");
  }
}

}  // namespace FQ_KNS

#define QP_FLEET_LAUNCH                                                                                      \
  (hipStream_t s, int batch, const QPPattern &pt, const QPSettingsDev &st, const double *Aval, const double *Pd, \
   const double *q, const double *l, const double *u, const double *xws, double *rho, double *yst, double *xo,  \
   double *yo, int *iters, int *status, double *obj) {                                                         \
    hipLaunchKernelGGL(FQ_KNS::k_qp_fleet, dim3(batch), dim3(FQ_T), 0, s, pt, st, Aval, Pd, q, l, u, xws, rho,   \
                       yst, xo, yo, iters, status, obj);                                                        \
    return hipGetLastError();                                                                                  \
  }
#ifdef FLEET_WIDE_TU
hipError_t launch_qp_fleet_wide QP_FLEET_LAUNCH
hipError_t launch_fleet_control_wide(hipStream_t s, int nb, const FleetArgs &a, bool stamps) {
  if (stamps)
    hipLaunchKernelGGL(FQ_KNS::k_fleet_control2<true>, dim3(nb), dim3(FQ_T), 0, s, a);
  else
    hipLaunchKernelGGL(FQ_KNS::k_fleet_control2<false>, dim3(nb), dim3(FQ_T), 0, s, a);
  return hipGetLastError();
}
#else
hipError_t launch_qp_fleet_narrow QP_FLEET_LAUNCH
// the fleet solver's pattern: the MPC pattern at N = 20 (fleet_qp.h's compiled sizes)
static_assert(FQ_MD == QP_FLEET_MD, "qp.h's copy of the dynamics row count");
bool qp_is_fleet_pattern(int n, int m, const int *rowptr, const int *colidx) {
  static std::vector<int> rp, ci;
  static std::once_flag once;
  std::call_once(once, [] { mpc_pattern(20, rp, ci); });
  const int nv = (20 + 1) * NX + 20 * NU;
  if (n != nv || m + 1 != (int)rp.size() || rowptr[m] != (int)ci.size()) return false;
  return !memcmp(rowptr, rp.data(), sizeof(int) * rp.size()) && !memcmp(colidx, ci.data(), sizeof(int) * ci.size());
}
__global__ void k_fleet_reset(int first, int count, int N, int target_mode,
                              const double *__restrict__ x0, double *x, double *Xw, double *Uw,
                              double *ysc, int m, double *rho, double rho0, double *rec,
                              double *xt) {
  const int i = blockIdx.x;
  if (i >= count) return;
  const int b = first + i;
  const double *xi = x0 + (int64_t)i * NX;
  double tg[NX];
  for (int c = 0; c < NX; ++c) tg[c] = 0.0;
  tg[0] = xi[0];                       // x_target = [m0, 0, ...] (monte_carlo.py:428-430)
  if (target_mode) {
    for (int c = 0; c < NX; ++c) tg[c] = xi[c];
    tg[4] = tg[5] = tg[6] = 0.0;
    tg[1] = fmax(0.5, xi[1] - 2.0);
  }
  for (int e = threadIdx.x; e < (N + 1) * NX; e += blockDim.x) {
    const int k = e / NX, c = e - k * NX;
    const double al = (double)k / N;
    Xw[(int64_t)b * (N + 1) * NX + e] = (1.0 - al) * xi[c] + al * tg[c];
  }
  for (int e = threadIdx.x; e < N * NU; e += blockDim.x)
    Uw[(int64_t)b * N * NU + e] = (e % NU == 0) ? xi[0] * 1.0 : 0.0;
  for (int r = threadIdx.x; r < m; r += blockDim.x) ysc[(int64_t)b * m + r] = 0.0;
  if (threadIdx.x < GPMPC_REC_LEN) rec[(int64_t)b * GPMPC_REC_LEN + threadIdx.x] = 0.0;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int c = 0; c < NX; ++c) {
      x[(int64_t)b * NX + c] = xi[c];
      xt[(int64_t)b * NX + c] = tg[c];
      rec[(int64_t)b * GPMPC_REC_LEN + 4 + c] = xi[c];
    }
    rec[(int64_t)b * GPMPC_REC_LEN + 13] = xi[0];
    rho[b] = rho0;
  }
}

// ---------------------------------------------------------------------------
static int fleet_create(gpmpc_ctx *ctx, gpmpc_gp *gp, gpmpc_fitc *fitc, const gpmpc_fleet_config *cfg,
                        int batch, int fleet_batch, gpmpc_fleet **out) {
  GPMPC_CHECK_ARG(ctx && (gp || fitc) && cfg && out && batch > 0 && fleet_batch >= batch);
  const GpView g = fitc ? fitc_view(fitc) : gp_view(gp);
  GPMPC_CHECK_ARG(g.d == NFEAT && g.n_out == 3);
  if (g.kind < GPMPC_SE_ARD || g.kind > GPMPC_MATERN52) {
    gpmpc_set_error("fleet: the GP must use one of the four stationary kernels (not a composite program)");
    return -2;
  }
  // the fleet runs MonteCarloSimulator's solve protocol (monte_carlo.py:495-512)
  // with the GPMPC adapter; FastRTI3DoF's step protocol (unshifted linearisation,
  // D2 sign, fallback to the shifted plan) is the host mirror mpc/osqp_rti.py
  if (cfg->target_mode != 1) {
    gpmpc_set_error("fleet: target_mode must be 1 (solve protocol); the step protocol of "
                    "FastRTI3DoF runs on the host mirror");
    return -2;
  }
  {
    // sqp_qp.max_iter = 0 means "use qp".  sqp_qp left at the defaults (a caller that
    // edits only qp) or equal to qp is that; any other field edited alongside max_iter 0
    // would be silently ignored, so such a config is refused
    auto same = [](const gpmpc_qp_settings &a, const gpmpc_qp_settings &b) {
      return a.rho == b.rho && a.sigma == b.sigma && a.alpha == b.alpha && a.eps_abs == b.eps_abs &&
             a.eps_rel == b.eps_rel && a.eps_prim_inf == b.eps_prim_inf && a.eps_dual_inf == b.eps_dual_inf &&
             a.check_termination == b.check_termination && a.adaptive_rho == b.adaptive_rho &&
             a.adaptive_rho_interval == b.adaptive_rho_interval &&
             a.adaptive_rho_tolerance == b.adaptive_rho_tolerance && a.scaling == b.scaling &&
             a.warm_start == b.warm_start;
    };
    gpmpc_qp_settings def;
    gpmpc_qp_default_settings(&def);
    if (cfg->sqp_iters > 1 && cfg->sqp_qp.max_iter == 0 && !same(cfg->sqp_qp, cfg->qp) &&
        !same(cfg->sqp_qp, def)) {
      gpmpc_set_error("fleet: sqp_qp was edited but sqp_qp.max_iter is 0 (= use qp); set "
                      "sqp_qp.max_iter to use the SQP passes' own settings");
      return -2;
    }
  }
  const int N = cfg->horizon;
  const int n = (N + 1) * NX + N * NU, m = NX * (N + 1) + n;
  GPMPC_CHECK_ARG(N >= 1 && n <= QP_NMAX && m <= QP_MMAX && NX + N * DYN_NNZ + n <= QP_NNZMAX);
  GPMPC_HIP(hipSetDevice(ctx->device));
  auto *f = new gpmpc_fleet();
  f->ctx = ctx; f->gp = gp; f->fitc = fitc; f->cfg = *cfg; f->B = batch; f->N = N; f->n = n; f->m = m;
  f->gp_n = g.n;
  f->n_active = batch;
  std::vector<int> rp, ci;
  mpc_pattern(N, rp, ci);
  if (f->pat.build(n, m, rp.data(), ci.data(), ctx->stream) || !f->pat.fits()) {
    delete f;
    gpmpc_set_error("fleet: QP pattern setup failed");
    return -1;
  }
  const size_t B = batch, P = (size_t)batch * N;
  f->plan_B = fleet_batch;
  f->post_kind = gemm_sumsq_kind(g.n + 3, (int)std::min<int64_t>((int64_t)fleet_batch * N, 1 << 30), g.n);
  f->post_few = (int64_t)fleet_batch * N <= 64 && g.d == NFEAT;
  // partial rows of any posterior path: W rows + the 3 alpha^T rows in 64-row tiles (the
  // most rows any kernel writes), at least the column-stationary posterior's two halves
  const int nrt = std::max(gemm_sumsq_rows(GEMM_SUMSQ_64, g.n + 3), POST_CS_PARTS);
  if (fitc) {
    f->post_kind2 = gemm_sumsq_kind(g.n, (int)std::min<int64_t>((int64_t)fleet_batch * N, 1 << 30), g.n);
    f->post_nrt2 = gemm_sumsq_rows(f->post_kind2, g.n);
    if (f->part2.alloc(sizeof(double) * gemm_sumsq_rows(GEMM_SUMSQ_64, g.n) * P)) {
      delete f;
      gpmpc_set_error("fleet: out of device memory");
      return -1;
    }
  }
  if (f->x.alloc(sizeof(double) * B * NX) || f->Xw.alloc(sizeof(double) * B * (N + 1) * NX) ||
      f->Uw.alloc(sizeof(double) * B * N * NU) || f->ysc.alloc(sizeof(double) * B * m) ||
      f->rho.alloc(sizeof(double) * B) || f->rec.alloc(sizeof(double) * B * GPMPC_REC_LEN) ||
      f->xt.alloc(sizeof(double) * B * NX) || f->Q.alloc(sizeof(double) * P * NFEAT) ||
      f->Qn.alloc(sizeof(double) * P) || f->Ks.alloc(sizeof(double) * P * g.n) ||
      f->part.alloc(sizeof(double) * nrt * P) || f->meanT.alloc(sizeof(double) * 3 * P) ||
      f->mean.alloc(sizeof(double) * P * 3) || f->var.alloc(sizeof(double) * P * 3) ||
      f->order.alloc(sizeof(int) * B) || f->lastit.alloc(sizeof(int) * B) ||
      f->claims.alloc(sizeof(unsigned) * 4096) || f->sqp_done.alloc(sizeof(int) * B)) {
    delete f;
    gpmpc_set_error("fleet: out of device memory");
    return -1;
  }
  // every landing starts terminated until reset
  std::vector<double> r(B * GPMPC_REC_LEN, 0.0);
  for (size_t b = 0; b < B; ++b) r[b * GPMPC_REC_LEN] = -1.0;
  hipMemcpyAsync(f->rec.p, r.data(), sizeof(double) * r.size(), hipMemcpyHostToDevice, ctx->stream);
  hipMemsetAsync(f->lastit.p, 0, sizeof(int) * B, ctx->stream);
  hipMemsetAsync(f->claims.p, 0, sizeof(unsigned) * 4096, ctx->stream);
  hipMemsetAsync(f->sqp_done.p, 0, sizeof(int) * B, ctx->stream);
  {  // identity dispatch order until the first order kernel (every slot maps in range)
    std::vector<int> id(B);
    for (size_t b = 0; b < B; ++b) id[b] = (int)b;
    hipMemcpyAsync(f->order.p, id.data(), sizeof(int) * B, hipMemcpyHostToDevice, ctx->stream);
    GPMPC_HIP(hipStreamSynchronize(ctx->stream));
  }
  const char *oe = getenv("GPMPC_FLEET_ORDER");
  f->use_order = !oe || atoi(oe) != 0;
  const char *aw = getenv("GPMPC_FLEET_ALTWAVE");
  f->alt_wave = aw ? atoi(aw) != 0 : 0;
  const char *sp = getenv("GPMPC_FLEET_SIMD");
  f->simd_pick = !sp || atoi(sp) != 0;
  const char *fp = getenv("GPMPC_FLEET_FUSE_POST");
  f->fuse_post = !fp || atoi(fp) != 0;
  const char *se = getenv("GPMPC_FLEET_SOLVER");
  // the specialised solver assumes the N = 20 stage layout of its LDS caps
  f->use_fq = (!se || atoi(se) != 0) && N == 20 && f->pat.mode == 1 && f->pat.nblk == FQ_NBLK &&
              m - n == FQ_MD && f->pat.nnz - n == FQ_NNZD;
  // small fleets (at most one landing per CU) take the 256-thread, one-wave-per-SIMD build of
  // the control kernel: twice the threads for the parallel ADMM phases and no register
  // spills (single landing 216 -> 192 us per step); decided by the fleet size, not by the
  // running count, so a fleet's landings always see the same arithmetic (GPMPC_FLEET_WIDE
  // = 0 / 1 forces it)
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
  const char *we = getenv("GPMPC_FLEET_WIDE");
  f->wide = f->use_fq && (we ? atoi(we) != 0 : fleet_batch <= cus);
  GPMPC_HIP(hipStreamSynchronize(ctx->stream));
  *out = f;
  return 0;
}

extern "C" int gpmpc_fleet_create_shard(gpmpc_ctx *ctx, gpmpc_gp *gp, const gpmpc_fleet_config *cfg,
                                        int batch, int fleet_batch, gpmpc_fleet **out) {
  GPMPC_CHECK_ARG(gp);
  return fleet_create(ctx, gp, nullptr, cfg, batch, fleet_batch, out);
}

extern "C" int gpmpc_fleet_create(gpmpc_ctx *ctx, gpmpc_gp *gp, const gpmpc_fleet_config *cfg, int batch,
                                  gpmpc_fleet **out) {
  return gpmpc_fleet_create_shard(ctx, gp, cfg, batch, batch, out);
}

extern "C" int gpmpc_fleet_create_fitc(gpmpc_ctx *ctx, gpmpc_fitc *gp, const gpmpc_fleet_config *cfg, int batch,
                                       int fleet_batch, gpmpc_fleet **out) {
  GPMPC_CHECK_ARG(gp);
  return fleet_create(ctx, nullptr, gp, cfg, batch, fleet_batch, out);
}

extern "C" int gpmpc_fleet_reset(gpmpc_fleet *f, int first, int count, const double *x0) {
  GPMPC_CHECK_ARG(f && x0 && first >= 0 && count >= 0 && first + count <= f->B);
  if (count == 0) return 0;
  hipStream_t s = f->ctx->stream;
  DevBuf d;
  GPMPC_HIP(d.alloc(sizeof(double) * count * NX));
  GPMPC_HIP(hipMemcpyAsync(d.p, x0, sizeof(double) * count * NX, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_fleet_reset, dim3(count), dim3(256), 0, s, first, count, f->N,
                     f->cfg.target_mode, d.as<double>(), f->x.as<double>(), f->Xw.as<double>(),
                     f->Uw.as<double>(), f->ysc.as<double>(), f->m, f->rho.as<double>(),
                     f->cfg.qp.rho, f->rec.as<double>(), f->xt.as<double>());
  GPMPC_HIP(hipGetLastError());
  GPMPC_HIP(hipStreamSynchronize(s));
  f->n_active = f->B;  // conservative until the host reads the records
  return 0;
}

// GP posterior of every landing's horizon, in three timed sub-phases:
//   bit 0: features + K* gram;  bit 2: one MFMA pass over K* with [W; alpha^T]:
//   variance partial sums (SUMSQ epilogue) and the means;  bit 3: finish
static hipError_t fleet_gp_posterior(gpmpc_fleet *f, int mask) {
  hipStream_t s = f->ctx->stream;
  const GpView g = fleet_view(f);
  const int nb = f->use_order ? f->n_active : f->B;  // slots 0 .. nb-1 (running first)
  const int P = nb * f->N;
  if (P == 0) return hipSuccess;
  // GPMPC_POST_FUSED=1: K* formed inside the posterior GEMM (no K* in HBM).
  // Measured slower (0.60 ms vs 0.062 ms gram + 0.415 ms GEMM at 1024 x 20):
  // each of the 8 row tiles regenerates its K* columns (4.6x the exps of the
  // gram kernel) and the exp/scalar-load stream does not hide under the FP64
  // MFMAs at 2 waves per SIMD.  Off by default.
  static const int fused_env = [] {
    const char *v = getenv("GPMPC_POST_FUSED");
    return v ? atoi(v) : 0;
  }();
  // GPMPC_POST_CS=1: the column-stationary posterior (post.hip), K* formed once per
  // workgroup inside the MFMA pass, never in HBM; two partial rows
  const bool cs = !f->fitc && g.Wf && post_cs_env();
  const bool fused = !f->fitc && !cs && fused_env && g.d >= 11 && g.d <= 13;
  const int nrt = cs ? POST_CS_PARTS : fused ? (g.n + 3 + 127) / 128 : gemm_sumsq_rows(f->post_kind, g.n + 3);
  hipError_t e = hipSuccess;
  if ((mask & 1) && !fused && !cs && f->post_few) {
    hipLaunchKernelGGL(k_fleet_queries_gram, dim3((g.n + 63) / 64), dim3(256), 0, s, nb, f->N, f->Xw.as<double>(),
                       f->Uw.as<double>(), g.ls, g.kind == GPMPC_SE_ISO, f->use_order ? f->order.as<int>() : nullptr,
                       g.kind, g.Xs, g.Xn, g.n, g.sigma2, g.iso_scale, f->Ks.as<double>());
    if ((e = hipGetLastError()) != hipSuccess) return e;
  } else if (mask & 1) {
    hipLaunchKernelGGL(k_fleet_queries, dim3((P + 255) / 256), dim3(256), 0, s, nb, f->N,
                       f->Xw.as<double>(), f->Uw.as<double>(), g.ls, g.kind == GPMPC_SE_ISO,
                       f->use_order ? f->order.as<int>() : nullptr, f->Q.as<double>(),
                       f->Qn.as<double>());
    if (!fused && !cs) {
      e = launch_gram(s, g.kind, f->Q.as<double>(), f->Qn.as<double>(), P, g.Xs, g.Xn, g.n, g.d,
                      g.sigma2, g.iso_scale, f->Ks.as<double>(), g.n, 0);
      if (e != hipSuccess) return e;
    }
  }
  if (mask & 4) {
    if (cs)
      e = launch_post_cs(s, g.n, 3, P, g.Wf, g.Xp, f->Q.as<double>(), f->Qn.as<double>(), g.d, g.kind, g.sigma2,
                         g.iso_scale, f->part.as<double>(), P, f->meanT.as<double>(), P);
    else if (fused)
      e = launch_gemm_post_fused(s, g.n, 3, P, g.W, f->Q.as<double>(), f->Qn.as<double>(), g.Xs,
                                 g.Xn, g.d, g.kind, g.sigma2, g.iso_scale, f->part.as<double>(), P,
                                 f->meanT.as<double>(), P);
    else
      e = launch_gemm_sumsq_mean(s, g.n, 3, P, g.W, f->Ks.as<double>(), f->part.as<double>(), P,
                                 f->meanT.as<double>(), P, f->post_kind);
    if (e != hipSuccess) return e;
    if (f->fitc) {  // |w|^2 = |L_B^-1 L_uu^-1 k*|^2 (sparse_gp.py:293-299)
      e = launch_gemm_sumsq(s, g.n, P, fitc_W2(f->fitc), f->Ks.as<double>(), f->part2.as<double>(), P,
                            f->post_kind2);
      if (e != hipSuccess) return e;
    }
  }
  if (mask & 4) {
    f->post_P = P;
    f->post_nrt = nrt;
  }
  // fused: k_fleet_control2 finishes each landing's own queries as it assembles
  if ((mask & 8) && !(f->use_fq && f->fuse_post)) {
    if (f->fitc)
      e = launch_fitc_finish(s, P, 3, nrt, f->post_nrt2, f->part.as<double>(), f->part2.as<double>(), P,
                             f->meanT.as<double>(), P, g.ymean, g.ystd, g.sigma2, f->mean.as<double>(),
                             f->var.as<double>());
    else
      e = launch_post_finish(s, P, 3, nrt, f->part.as<double>(), P, f->meanT.as<double>(), P,
                             g.ymean, g.ystd, g.sigma2, f->mean.as<double>(), f->var.as<double>());
  }
  return e;
}

// Dispatch order for the control kernel.  Workgroups start in blockIdx order
// and a landing's solve costs ~proportional to its ADMM iterations (25 or 50
// here: 237 vs 490 us), so launching the landings whose last solve was
// longest first is the LPT schedule over the 512 resident slots (measured
// span 916 us vs 826 us LPT-ideal).  Terminated landings (they return at once)
// go last.  Counting sort in one workgroup; the order inside a bucket is
// arbitrary, which cannot change results: landings are independent.
#define ORDER_BUCKETS 256
__global__ __launch_bounds__(1024) void k_fleet_order(int B, const double *__restrict__ rec,
                                                      const int *__restrict__ lastit,
                                                      int *__restrict__ order) {
  __shared__ int cnt[ORDER_BUCKETS];
  for (int i = threadIdx.x; i < ORDER_BUCKETS; i += blockDim.x) cnt[i] = 0;
  __syncthreads();
  auto key = [&](int b) {  // larger = earlier; 0 = terminated
    if (rec[(int64_t)b * GPMPC_REC_LEN] != 0.0) return 0;
    return min(lastit[b], ORDER_BUCKETS - 2) + 1;
  };
  // Wave-aggregated LDS atomics: nearly every landing sits in one of two or
  // three buckets (25 / 50 iterations, terminated), and per-lane atomics on one
  // LDS word serialise.  Each wave adds once per distinct key it holds; lanes
  // take base + their rank among the wave's lanes with that key.
  const int lane = threadIdx.x & 63;
  auto wave_add = [&](int k, bool active) {
    int slot = 0;
    unsigned long long todo = __ballot(active);
    while (todo) {
      const int leader = __ffsll((long long)todo) - 1;
      const int lk = __shfl(k, leader);
      const unsigned long long same = __ballot(active && k == lk);
      int base = 0;
      if (lane == leader) base = atomicAdd(&cnt[lk], __popcll(same));
      base = __shfl(base, leader);
      if (active && k == lk) slot = base + __popcll(same & ((1ull << lane) - 1));
      todo &= ~same;
    }
    return slot;
  };
  for (int b0 = 0; b0 < B; b0 += blockDim.x) {
    const int b = b0 + threadIdx.x;
    wave_add(b < B ? key(b) : 0, b < B);
  }
  __syncthreads();
  // descending exclusive scan over the buckets, 256 threads (4 waves, shuffles)
  static_assert(ORDER_BUCKETS == 256, "scan is laid out for 256 buckets");
  __shared__ int wsum[4];
  int c = 0, inc = 0;
  if (threadIdx.x < ORDER_BUCKETS) {
    c = cnt[ORDER_BUCKETS - 1 - threadIdx.x];
    inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o);
      if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[threadIdx.x >> 6] = inc;
  }
  __syncthreads();
  if (threadIdx.x < ORDER_BUCKETS) {
    int pre = 0;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) pre += wsum[w];
    cnt[ORDER_BUCKETS - 1 - threadIdx.x] = pre + inc - c;
  }
  __syncthreads();
  for (int b0 = 0; b0 < B; b0 += blockDim.x) {
    const int b = b0 + threadIdx.x;
    const int slot = wave_add(b < B ? key(b) : 0, b < B);
    if (b < B) order[slot] = b;
  }
}

static FleetArgs fleet_args(gpmpc_fleet *f) {
  FleetArgs a;
  a.pt = f->pat.dev;
  a.st = to_dev(f->cfg.sqp_iters > 1 && f->cfg.sqp_qp.max_iter > 0 ? f->cfg.sqp_qp : f->cfg.qp);
  a.N = f->N;
  a.target_mode = f->cfg.target_mode;
  a.use_gp = f->cfg.use_gp;
  a.residual_model = f->cfg.residual_model;
  a.max_steps = f->cfg.max_steps;
  a.dt = f->cfg.dt;
  a.x = f->x.as<double>(); a.Xw = f->Xw.as<double>(); a.Uw = f->Uw.as<double>();
  a.ysc = f->ysc.as<double>(); a.rho = f->rho.as<double>(); a.rec = f->rec.as<double>();
  a.xt = f->xt.as<double>();
  a.gmean = f->mean.as<double>();
  a.gp_by_slot = f->use_order && f->cfg.use_gp;
  a.order = f->use_order ? f->order.as<int>() : nullptr;
  a.alt_wave = f->alt_wave;
  a.claims = f->simd_pick ? f->claims.as<unsigned>() : nullptr;
  a.part = nullptr;
  a.part2 = nullptr;
  a.nrt2 = 0;
  if (f->use_fq && f->fuse_post && f->cfg.use_gp && f->post_P > 0) {
    const GpView g = fleet_view(f);
    if (f->fitc) {
      a.part2 = f->part2.as<double>();
      a.nrt2 = f->post_nrt2;
    }
    a.part = f->part.as<double>();
    a.meanT = f->meanT.as<double>();
    a.ymean = g.ymean;
    a.ystd = g.ystd;
    a.mean_out = f->mean.as<double>();
    a.var_out = f->var.as<double>();
    a.sigma2 = g.sigma2;
    a.nrt = f->post_nrt;
    a.pld = f->post_P;
  }
  f->epoch = (f->epoch + 1) & 0xffffff;
  if (f->epoch == 0) f->epoch = 1;
  a.epoch = f->epoch;
  a.lastit = f->lastit.as<int>();
  a.stamps = f->stamps;
  a.trace = f->trace;
  a.sqp = f->cfg.sqp_iters > 1;
  a.sqp_first = f->sqp_it == 0;
  a.sqp_last = f->sqp_it >= f->cfg.sqp_iters - 1;
  a.sqp_tol = f->cfg.sqp_tol;
  a.sqp_done = f->sqp_done.as<int>();
  return a;
}

extern "C" int gpmpc_fleet_step_phases(gpmpc_fleet *f, int phase_mask) {
  GPMPC_CHECK_ARG(f);
  if (fleet_view(f).n != f->gp_n) {  // gpmpc_gp_append grew the GP under the fleet
    gpmpc_set_error("fleet: the GP has %d training rows, the fleet was built for %d; recreate it",
                    fleet_view(f).n, f->gp_n);
    return -2;
  }
  GPMPC_HIP(hipSetDevice(f->ctx->device));
  if (f->cfg.sqp_iters > 1 && f->sqp_it == 0 && (phase_mask & 3))
    hipLaunchKernelGGL(k_fleet_x0_to_plan, dim3((f->B * NX + 255) / 256), dim3(256), 0, f->ctx->stream, f->B,
                       f->cfg.horizon, f->x.as<double>(), f->rec.as<double>(), f->Xw.as<double>());
  // the dispatch order of this step, before the GP phase when there is one:
  // the posterior rows then follow the same slots as the control workgroups
  // (one landing: the identity order set at creation is the only one)
  const bool order_now = f->use_order && f->sqp_it == 0 && f->B > 1 &&
                         ((f->cfg.use_gp && (phase_mask & 1)) || (!f->cfg.use_gp && (phase_mask & 2)));
  if (order_now)
    hipLaunchKernelGGL(k_fleet_order, dim3(1), dim3(1024), 0, f->ctx->stream, f->B,
                       f->rec.as<double>(), f->lastit.as<int>(), f->order.as<int>());
  if ((phase_mask & 13) && f->cfg.use_gp) GPMPC_HIP(fleet_gp_posterior(f, phase_mask));
  if (phase_mask & 2) {
    const int nb = f->use_order ? f->n_active : f->B;
    if (nb > 0) {
      if (f->use_fq && f->wide) {
        GPMPC_HIP(launch_fleet_control_wide(f->ctx->stream, nb, fleet_args(f), f->stamps != nullptr));
      } else if (f->use_fq) {
        if (f->stamps)
          hipLaunchKernelGGL(FQ_KNS::k_fleet_control2<true>, dim3(nb), dim3(FQ_T), 0, f->ctx->stream,
                             fleet_args(f));
        else
          hipLaunchKernelGGL(FQ_KNS::k_fleet_control2<false>, dim3(nb), dim3(FQ_T), 0, f->ctx->stream,
                             fleet_args(f));
      } else {
        hipLaunchKernelGGL(k_fleet_control, dim3(nb), dim3(256), 0, f->ctx->stream, fleet_args(f));
      }
    }
    GPMPC_HIP(hipGetLastError());
  }
  return 0;
}

extern "C" int gpmpc_fleet_step(gpmpc_fleet *f, int nsteps) {
  GPMPC_CHECK_ARG(f && nsteps >= 0);
  const int passes = f->cfg.sqp_iters > 1 ? f->cfg.sqp_iters : 1;
  for (int it = 0; it < nsteps; ++it) {
    // SQP mode: every pass re-linearises around the last QP solution (GP
    // posterior at the new horizon points, QP); landings that converged skip
    // the later passes' control launches
    for (int p = 0; p < passes; ++p) {
      f->sqp_it = p;
      const int rc = gpmpc_fleet_step_phases(f, 15);
      if (rc) { f->sqp_it = 0; return rc; }
    }
    f->sqp_it = 0;
  }
  return 0;
}

extern "C" int gpmpc_fleet_read(gpmpc_fleet *f, double *records, double *x) {
  GPMPC_CHECK_ARG(f);
  hipStream_t s = f->ctx->stream;
  if (records)
    GPMPC_HIP(hipMemcpyAsync(records, f->rec.p, sizeof(double) * f->B * GPMPC_REC_LEN,
                             hipMemcpyDeviceToHost, s));
  if (x) GPMPC_HIP(hipMemcpyAsync(x, f->x.p, sizeof(double) * f->B * NX, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  if (records) {
    int run = 0;
    for (int b = 0; b < f->B; ++b) run += records[(size_t)b * GPMPC_REC_LEN] == 0.0;
    f->n_active = run;
  }
  return 0;
}

extern "C" int gpmpc_fleet_get_state(gpmpc_fleet *f, double *Xw, double *Uw, double *y_scaled,
                                     double *rho) {
  GPMPC_CHECK_ARG(f);
  hipStream_t s = f->ctx->stream;
  const size_t B = (size_t)f->B, N = (size_t)f->N;
  if (Xw) GPMPC_HIP(hipMemcpyAsync(Xw, f->Xw.p, sizeof(double) * B * (N + 1) * NX, hipMemcpyDeviceToHost, s));
  if (Uw) GPMPC_HIP(hipMemcpyAsync(Uw, f->Uw.p, sizeof(double) * B * N * NU, hipMemcpyDeviceToHost, s));
  if (y_scaled)
    GPMPC_HIP(hipMemcpyAsync(y_scaled, f->ysc.p, sizeof(double) * B * f->m, hipMemcpyDeviceToHost, s));
  if (rho) GPMPC_HIP(hipMemcpyAsync(rho, f->rho.p, sizeof(double) * B, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

// The GP posterior of the last control step at every landing's N horizon points, per
// landing (B x N x 3 each, row-major): the mean and variance the step's QP assembly
// consumed (the variance is computed beside it, exact_gp.py:256-266, and not read by
// the QP).  The device rows follow the dispatch slots of that step; they are put back
// in landing order here.  Every slot of the step's launched prefix is finished (the
// control kernel finishes the slots of landings that return before their QP too), so a
// landing in it reads the posterior at its own trajectory; landings past it read NaN.
extern "C" int gpmpc_fleet_get_posterior(gpmpc_fleet *f, double *mean, double *var) {
  GPMPC_CHECK_ARG(f && (mean || var));
  if (!f->cfg.use_gp) {
    gpmpc_set_error("fleet: use_gp = 0, the fleet runs no GP posterior");
    return -2;
  }
  hipStream_t s = f->ctx->stream;
  GPMPC_HIP(hipSetDevice(f->ctx->device));
  const size_t B = (size_t)f->B, N = (size_t)f->N, P = B * N;
  std::vector<double> dm(P * 3), dv(P * 3), rec(B * GPMPC_REC_LEN);
  std::vector<int> ord(B);
  GPMPC_HIP(hipMemcpyAsync(dm.data(), f->mean.p, sizeof(double) * P * 3, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipMemcpyAsync(dv.data(), f->var.p, sizeof(double) * P * 3, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipMemcpyAsync(ord.data(), f->order.p, sizeof(int) * B, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  const bool by_slot = f->use_order;  // gp_by_slot of fleet_args (use_gp holds here)
  const size_t nslots = by_slot ? (size_t)f->post_P / N : B;
  std::vector<char> ran(B, 0);
  for (size_t sl = 0; sl < nslots && sl < B; ++sl) {
    const int b = by_slot ? ord[sl] : (int)sl;
    if (b < 0 || (size_t)b >= B) continue;
    ran[b] = 1;
    for (size_t e = 0; e < N * 3; ++e) {
      if (mean) mean[(size_t)b * N * 3 + e] = dm[sl * N * 3 + e];
      if (var) var[(size_t)b * N * 3 + e] = dv[sl * N * 3 + e];
    }
  }
  for (size_t b = 0; b < B; ++b)
    if (!ran[b])
      for (size_t e = 0; e < N * 3; ++e) {
        if (mean) mean[b * N * 3 + e] = NAN;
        if (var) var[b * N * 3 + e] = NAN;
      }
  return 0;
}

extern "C" double *gpmpc_fleet_records_dev(gpmpc_fleet *f) { return f ? f->rec.as<double>() : nullptr; }

extern "C" int gpmpc_fleet_destroy(gpmpc_fleet *f) {
  if (f && f->ctx) (void)hipStreamSynchronize(f->ctx->stream);
  delete f;
  return 0;
}


// ---------------------------------------------------------------------------
// UncertaintyPropagator._propagate_linear (uncertainty_prop.py:117-177) for the 3-DoF model
// on the device, batch trajectories at once (gpmpc_uprop3_linear).  The mean recursion is
// sequential -- x_k+1 needs the GP mean at x_k -- so one workgroup per trajectory walks the
// N steps: the query's features (features3, the fleet's), the exact GP mean over the n
// training rows (256 threads, a fixed-order block reduction), the explicit-Euler step of
// rocket_3dof.py (x + dt f, f = [-alpha |u|, v, u / m + g], products and sums unfused as
// numpy forms them) plus dt d_v on the velocity rows, and A_k = I + dt J(x_k, u_k).  The
// variances of all B N queries then come from the GP's own batched posterior, and one
// launch propagates every covariance (k_cov_propagate).
#define UP3_R 4  // training rows per thread held in registers (n <= 1024); larger n reads them per step
#define UP_NCAP 256  // horizon steps whose controls the propagation kernels stage in LDS
__global__ __launch_bounds__(256) void k_uprop3_means(GpView g, int N, double dt, double alpha, double g0,
                                                      double g1, double g2, const double *__restrict__ x0,
                                                      const double *__restrict__ U, double *__restrict__ Q,
                                                      double *__restrict__ A, double *__restrict__ means) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ double sx[NX], sz[NFEAT], szn, red[4][3];
  // this thread's training rows j = tid + 256 r (scaled features, |x_j|^2, alpha), loaded once:
  // the N sequential steps then read no global memory on their critical path
  const bool reg = g.n <= 256 * UP3_R;
  double xr[UP3_R][NFEAT], xnr[UP3_R], ar[UP3_R][3];
#pragma unroll
  for (int r = 0; r < UP3_R; ++r) {
    const int j = tid + 256 * r;
    const bool ok = reg && j < g.n;
#pragma unroll
    for (int f = 0; f < NFEAT; ++f) xr[r][f] = ok ? g.Xs[(int64_t)j * NFEAT + f] : 0.0;
    xnr[r] = ok ? g.Xn[j] : 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) ar[r][c] = ok ? g.alphaT[(int64_t)c * g.n + j] : 0.0;
  }
  // the trajectory's controls staged in LDS once (up to UP_NCAP steps): no global
  // round trip on the step chain
  __shared__ double sU[UP_NCAP * NU];
  const bool uc = N <= UP_NCAP;
  for (int e = tid; uc && e < N * NU; e += 256) sU[e] = U[(int64_t)b * N * NU + e];
  const double *Ub = uc ? sU : U + (int64_t)b * N * NU;
  if (tid < NX) {
    sx[tid] = x0[(int64_t)b * NX + tid];
    means[(int64_t)b * (N + 1) * NX + tid] = sx[tid];
  }
  __syncthreads();
  for (int k = 0; k < N; ++k) {
    const double *u = Ub + k * NU;
    if (tid == 0) {
      double z[NFEAT];
      features3(sx, u, z);
      double sn = 0.0;
      for (int f = 0; f < NFEAT; ++f) {
        Q[((int64_t)b * N + k) * NFEAT + f] = z[f];
        const double v = g.kind == GPMPC_SE_ISO ? z[f] : z[f] / g.ls[f];
        sz[f] = v;
        sn += v * v;
      }
      szn = sn;
    } else if (tid >= 64 && tid < 64 + NX * NX) {
      // A_k = I + dt J: J[1:4, 4:7] = I, J[4:7, 0] = -u / m^2 (rocket_3dof.py jacobian_x), one entry a thread
      const int e = tid - 64, r = e / NX, c = e - r * NX;
      double v = (r == c) ? 1.0 : 0.0;
      if (r >= 1 && r <= 3 && c == r + 3) v = __dmul_rn(1.0, dt);
      if (r >= 4 && c == 0) v = __dmul_rn(-u[r - 4] / __dmul_rn(sx[0], sx[0]), dt);
      A[((int64_t)b * N + k) * NX * NX + e] = v;
    }
    __syncthreads();
    double acc[3] = {0.0, 0.0, 0.0};
    const double zn = szn;
    if (reg) {
      double zv[NFEAT];
#pragma unroll
      for (int f = 0; f < NFEAT; ++f) zv[f] = sz[f];
#pragma unroll
      for (int r = 0; r < UP3_R; ++r) {
        if (tid + 256 * r >= g.n) break;
        double dot = 0.0;
#pragma unroll
        for (int f = 0; f < NFEAT; ++f) dot = fma(zv[f], xr[r][f], dot);
        const double kv = kernel_epilogue(g.kind, (zn + xnr[r]) - 2.0 * dot, g.sigma2, g.iso_scale);
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] = fma(kv, ar[r][c], acc[c]);
      }
    } else {
      for (int j = tid; j < g.n; j += 256) {
        double dot = 0.0;
#pragma unroll
        for (int f = 0; f < NFEAT; ++f) dot = fma(sz[f], g.Xs[(int64_t)j * NFEAT + f], dot);
        const double kv = kernel_epilogue(g.kind, (zn + g.Xn[j]) - 2.0 * dot, g.sigma2, g.iso_scale);
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] = fma(kv, g.alphaT[(int64_t)c * g.n + j], acc[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc[c] += __shfl_xor(acc[c], o);
    if (lane == 0)
      for (int c = 0; c < 3; ++c) red[wave][c] = acc[c];
    __syncthreads();
    if (tid == 0) {
      double dv[3];
      for (int c = 0; c < 3; ++c) {
        const double m = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
        dv[c] = __dadd_rn(__dmul_rn(m, g.ystd[c]), g.ymean[c]);
      }
      // x + dt f(x, u), then + d_v dt on the velocity rows
      const double um = sqrt(__dadd_rn(__dadd_rn(__dmul_rn(u[0], u[0]), __dmul_rn(u[1], u[1])), __dmul_rn(u[2], u[2])));
      double f[NX];
      f[0] = __dmul_rn(-alpha, um);
      f[1] = sx[4]; f[2] = sx[5]; f[3] = sx[6];
      f[4] = __dadd_rn(u[0] / sx[0], g0); f[5] = __dadd_rn(u[1] / sx[0], g1); f[6] = __dadd_rn(u[2] / sx[0], g2);
      double xn[NX];
      for (int i = 0; i < NX; ++i) xn[i] = __dadd_rn(sx[i], __dmul_rn(dt, f[i]));
      for (int c = 0; c < 3; ++c) xn[4 + c] = __dadd_rn(xn[4 + c], __dmul_rn(dv[c], dt));
      for (int i = 0; i < NX; ++i) {
        sx[i] = xn[i];
        means[((int64_t)b * (N + 1) + k + 1) * NX + i] = xn[i];
      }
    }
    __syncthreads();
  }
}

// q_k = var dt^2 on the velocity rows (uncertainty_prop.py:160-161)
__global__ void k_uprop3_q(int P, double dt2, const double *__restrict__ var, double *__restrict__ q) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= P) return;
  for (int i = 0; i < NX; ++i) q[(int64_t)j * NX + i] = (i >= 4) ? __dmul_rn(var[(int64_t)j * 3 + i - 4], dt2) : 0.0;
}

extern "C" int gpmpc_uprop3_linear(gpmpc_ctx *ctx, gpmpc_gp *gp, int batch, int N, double dt, double alpha,
                                   const double *g3, const double *x0, const double *U, const double *S0,
                                   double s0_diag, double *means, double *covs) {
  GPMPC_CHECK_ARG(ctx && gp && g3 && x0 && U && means && covs && batch >= 0 && N >= 0);
  const GpView g = gp_view(gp);
  if (g.d != NFEAT || g.n_out != 3 || g.kind == GPMPC_KPROG) {
    gpmpc_set_error("uprop3_linear: needs the 3-DoF exact GP (11 features, 3 outputs, a leaf kernel)");
    return -2;
  }
  if (batch == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const size_t B = batch, P = B * N;
  DevBuf dQ, dA, dq, dvar, dmu;
  GPMPC_HIP(dQ.alloc(s, sizeof(double) * (P * NFEAT + 1)));
  GPMPC_HIP(dA.alloc(s, sizeof(double) * (P * NX * NX + 1)));
  GPMPC_HIP(dq.alloc(s, sizeof(double) * (P * NX + 1)));
  // inputs in one pinned upload, means and covariances in one read-back
  const size_t bytes = Stage::pad(8 * B * NX) + Stage::pad(8 * P * NU) + (S0 ? Stage::pad(8 * B * NX * NX) : 0) +
                       Stage::pad(8 * B * (N + 1) * NX) + Stage::pad(8 * B * (N + 1) * NX * NX);
  Stage sg(s, bytes);
  if (!sg.ok()) {
    gpmpc_set_error("uprop3_linear: staging buffers: out of memory");
    return -1;
  }
  const double *dx0 = sg.in(x0, B * NX), *dU = sg.in(U, P * NU);
  const double *dS0 = S0 ? sg.in(S0, B * NX * NX) : nullptr;
  double *dmeans = sg.out(means, B * (N + 1) * NX), *dcov = sg.out(covs, B * (N + 1) * NX * NX);
  GPMPC_HIP(sg.upload());
  hipLaunchKernelGGL(k_uprop3_means, dim3(batch), dim3(256), 0, s, g, N, dt, alpha, g3[0], g3[1], g3[2], dx0, dU,
                     dQ.as<double>(), dA.as<double>(), dmeans);
  GPMPC_HIP(hipGetLastError());
  if (P) {
    GPMPC_HIP(dmu.alloc(s, sizeof(double) * P * 3));
    GPMPC_HIP(dvar.alloc(s, sizeof(double) * P * 3));
    const int rc = gp_posterior_dev(ctx, gp, dQ.as<double>(), (int)P, dmu.as<double>(), dvar.as<double>());
    if (rc) return rc;
    hipLaunchKernelGGL(k_uprop3_q, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, (int)P, dt * dt,
                       dvar.as<double>(), dq.as<double>());
    GPMPC_HIP(hipGetLastError());
  }
  const int rc = gpmpc_cov_propagate_dev(ctx, batch, N, NX, dA.as<double>(), dq.as<double>(), dS0, s0_diag, dcov);
  if (rc) return rc;
  GPMPC_HIP(sg.download());
  return 0;
}

#endif  // FLEET_WIDE_TU