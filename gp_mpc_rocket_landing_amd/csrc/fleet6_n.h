// fleet6_n.h -- the horizon-dependent half of fleet6.hip: the predict, control and
// plant kernels and their launchers for ONE horizon R6_N (defined by the includer,
// inside a namespace of its own).  Included once per supported horizon.
#ifndef R6_N
#error "define R6_N before including fleet6_n.h"
#endif
#define R6_NBLK (R6_N + 1)
#define R6_NV (R6_N * R6_SZ + R6_NX)          // 524 variables at N = 30 (354 at 20)
#define R6_MD (R6_NX * (R6_N + 1))            // 434 equality rows (294)
#define R6_MT R6_N                            // 30 thrust rows
#define R6_MG (4 * (R6_N - 1))                // 116 glideslope rows (76)
#define R6_MGEN (R6_MT + R6_MG)               // 146 general rows (96)
#define R6_M (R6_MD + R6_NV + R6_MGEN)        // 1104 rows (744)
static_assert(R6_N >= 2, "the twisted factor needs a top and a bottom end");
static_assert(R6_NV <= 2 * R6_T && R6_NV + R6_MD <= 2 * R6_T && R6_MGEN <= R6_T, "two items per thread");

// diagnostic phase cycles of the predict kernel's rollout 0 (GPMPC_R6_STAMPS=1)
__device__ unsigned long long g_r6p_stamps[8];

// Per horizon point k (the points are sequential: X[k+1] needs the GP mean at X[k]):
//   waves 0 .. R6_PT/64 - 2: the 2 x M kernel rows of both GPs (K*u . coefficients);
//   the last wave, lane 0, meanwhile: RK4(X[k], U[k]) (the GP mean is added after);
//   barrier; lanes 0 of waves 0 .. 5: the means, X[k+1] = RK4 + [.., d_v dt, .., d_w dt],
//   then the six roles of point k+1's features (r6_features_role);
//   barrier.
// Split (a.parts > 1, r6_predict_parts): a rollout's kernel rows run on a.parts co-resident
// workgroups, by whole waves (part p: waves [2p, min(2p + 2, 7)) of the 7 kernel-row
// waves), each wave's six sums published as twelve tagged 8-byte granules {tag = point
// + 1, one 32-bit word} with agent-scope (sc1) stores; one idle wave of every part polls
// all 84 granules of the point until every tag matches (bounded: a.tmo on give-up) and
// rebuilds the per-wave sums.  Every part then runs the same serial tail (means, RK4,
// next features) on the same values, so all parts agree bit for bit with each other and
// with the unsplit kernel; part 0 alone writes the outputs.  Two point parities per
// rollout: a part writes point k + 2 only after every part has published point k + 1,
// hence finished reading point k.
__device__ __forceinline__ bool r6_spin_fail(unsigned &spins, unsigned *tmo, int lane) {
  if (++spins < (1u << 20)) {
    __builtin_amdgcn_s_sleep(2);
    return false;
  }
  if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

template <bool ST>
__global__ __launch_bounds__(R6_PT) void k_r6_predict(R6Args a) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  constexpr int NW = R6_PT / 64, NRT = R6_PT - 64;  // waves; kernel-row threads
  static_assert(NW == 8 && (NW - 1) * 12 == R6_GRAN, "seven kernel-row waves of twelve granules");
  // the parts of a rollout on one XCD (blocks L and L + 8 share one): block L is part
  // (L / 8) % parts of rollout (L / 8 / parts) * 8 + L % 8
  int b = blockIdx.x, part = 0;
  if (a.parts > 1) {
    const int m = (int)blockIdx.x >> 3;
    b = (m / a.parts) * 8 + ((int)blockIdx.x & 7);
    part = m % a.parts;
    if (b >= a.nb) return;
  }
  const bool out_here = part == 0;               // the part that writes the outputs
  const int wlo = 2 * part, whi = min(2 * part + 2, NW - 1);
  const int poller = wlo > 0 ? 0 : NW - 2;       // a kernel-row wave idle in this part
  const unsigned long long t_start = ST ? __builtin_amdgcn_s_memtime() : 0;
  unsigned long long tl = 0;
  auto mark = [&](int k) {
    if (ST && b == 0 && out_here && tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (k >= 0) g_r6p_stamps[k] += t - tl;
      tl = t;
    }
  };
  double *rec = a.rec + (int64_t)b * GPMPC_REC_LEN;
  if (a.mode == 0 ? rec[0] != 0.0 : a.done[b] != 0) return;
  __shared__ double X[R6_N + 1][R6_NX];
  __shared__ double zq[2][16];
  __shared__ double red[NW][6];
  __shared__ double xrk[R6_NX];
  __shared__ unsigned gwords[R6_GRAN];
  __shared__ int s_out;
  const double dt = a.dt;
  const bool relin = a.mode == 2;  // a later GPMPC.solve pass: X_pred = the last plan
  if (relin) {
    for (int e = tid; e < (R6_N + 1) * R6_NX; e += R6_PT)
      (&X[0][0])[e] = a.Xo[(int64_t)b * (R6_N + 1) * R6_NX + e];
  } else if (tid < R6_NX) {
    X[0][tid] = a.x[(int64_t)b * R6_NX + tid];
  }
  if (tid == 0) s_out = 0;
  __syncthreads();
  if (a.mode == 0 && tid == 0) {  // monte_carlo.py:458-488 on [m, r, v]; then any non-finite 6-DoF state
    const double *x = X[0];
    const double m0 = rec[13];
    bool div7 = false, div = false;
    for (int i = 0; i < 7; ++i) div7 = div7 || !(fabs(x[i]) <= 1e6);
    for (int i = 0; i < R6_NX; ++i) div = div || !(fabs(x[i]) <= 1e6);
    int out = 0;
    if ((int)rec[1] >= a.max_steps) out = 5;
    else if (x[1] < 0.0) out = 2;
    else if (x[0] <= 1.0 + 0.01) out = 3;
    else if (div7) out = 6;
    else if (x[1] < 1.0 && fabs(x[4]) < 5.0) out = r6_landing_ok(x, m0) ? 1 : 4;
    else if (div) out = 6;
    if (out && out_here) {
      rec[0] = out;
      rec[2] = m0 - x[0];
      for (int i = 0; i < 7; ++i) rec[4 + i] = x[i];
    }
    s_out = out;
  }
  __syncthreads();
  if (s_out) return;
  const double *Ub = a.U + (int64_t)b * R6_N * R6_NU;
  const bool feat_lane = lane == 0 && wave < R6_FEAT_ROLES;
  // features of point 0
  if (a.use_gp && feat_lane) r6_features_role(wave, X[0], Ub, a.gv.ls, a.gw.ls, zq[0], zq[1]);
  // the first mcv / mcw inducing rows of either GP, feature-major in LDS
  extern __shared__ double r6_sx[];
  double *sxv = r6_sx, *sxw = r6_sx + a.mcv * 13;
  if (a.use_gp) {
    for (int e = tid; e < a.mcv * 13; e += R6_PT) {
      const int i = e / 13, f = e - i * 13;
      sxv[f * a.mcv + i] = a.gv.Xs[e];
    }
    for (int e = tid; e < a.mcw * 12; e += R6_PT) {
      const int i = e / 12, f = e - i * 12;
      sxw[f * a.mcw + i] = a.gw.Xs[e];
    }
  }
  __syncthreads();
  if (ST && b == 0 && out_here && tid == 0) g_r6p_stamps[3] += __builtin_amdgcn_s_memtime() - t_start;
  mark(-1);
  for (int k = 0; k < R6_N; ++k) {
    // K*u . coefficients of both GPs: the expansion form of the gram kernel (same
    // bits per kernel value); 3 outputs each
    double acc[6] = {0, 0, 0, 0, 0, 0};
    if (tid < NRT) {
      if (a.parts == 1 || (wave >= wlo && wave < whi)) {
        const unsigned long long tr0 = ST ? __builtin_amdgcn_s_memtime() : 0;
        if (a.use_gp) {
          r6_kernel_rows<13>(a.gv, a.Mv, a.cv, zq[0], tid, NRT, acc, sxv, a.mcv);
          r6_kernel_rows<12>(a.gw, a.Mw, a.cw, zq[1], tid, NRT, acc + 3, sxw, a.mcw);
        }
#pragma unroll
        for (int c = 0; c < 6; ++c)
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) acc[c] += __shfl_xor(acc[c], o);
        if (ST && b == 0 && out_here && tid == 0) g_r6p_stamps[5] += __builtin_amdgcn_s_memtime() - tr0;
        if (a.parts == 1) {
          if (lane == 0)
#pragma unroll
            for (int c = 0; c < 6; ++c) red[wave][c] = acc[c];
        } else if (lane < 12) {  // every lane holds the sums: lane 2c + h publishes word h of sum c
          double v = acc[0];
#pragma unroll
          for (int c = 1; c < 6; ++c) v = (lane >> 1) == c ? acc[c] : v;
          const unsigned wd = (lane & 1) ? (unsigned)__double2hiint(v) : (unsigned)__double2loint(v);
          unsigned long long *g = a.gran + ((size_t)b * 2 + (k & 1)) * R6_GRAN + wave * 12 + lane;
          __hip_atomic_store(g, ((unsigned long long)(k + 1) << 32) | wd, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      } else if (wave == poller) {  // every wave's granules of point k, this part's included
        const unsigned long long *g = a.gran + ((size_t)b * 2 + (k & 1)) * R6_GRAN;
        const unsigned tag = (unsigned)(k + 1);
        const bool two = lane + 64 < R6_GRAN;
        unsigned long long x0, x1;
        const unsigned long long tp0 = ST ? __builtin_amdgcn_s_memtime() : 0;
        for (unsigned spins = 0;;) {
          x0 = __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          x1 = two ? __hip_atomic_load(g + lane + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : ((unsigned long long)tag << 32);
          if (__all((unsigned)(x0 >> 32) == tag && (unsigned)(x1 >> 32) == tag)) break;
          if (r6_spin_fail(spins, a.tmo, lane)) break;
        }
        if (ST && b == 0 && out_here && lane == 0) g_r6p_stamps[6] += __builtin_amdgcn_s_memtime() - tp0;
        gwords[lane] = (unsigned)x0;
        if (two) gwords[lane + 64] = (unsigned)x1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < (NW - 1) * 6) {
          const int w = lane / 6, c = lane - 6 * (lane / 6);
          red[w][c] = __hiloint2double((int)gwords[w * 12 + 2 * c + 1], (int)gwords[w * 12 + 2 * c]);
        }
      }
    } else if (!relin && lane == 0) {  // _predict_with_gp's nominal step (gp_mpc.py:156)
      double xn[R6_NX];
      const unsigned long long t0 = ST ? __builtin_amdgcn_s_memtime() : 0;
      r6_step(a.rk, X[k], Ub + k * R6_NU, dt, xn);
      if (ST && b == 0 && out_here) g_r6p_stamps[2] += __builtin_amdgcn_s_memtime() - t0;
      for (int i = 0; i < R6_NX; ++i) xrk[i] = xn[i];
    }
    __syncthreads();
    mark(1);
    if (feat_lane) {
      double gmk[6];
      for (int c = 0; c < 6; ++c) {
        double sm = 0.0;
        for (int w = 0; w < NW - 1; ++w) sm += red[w][c];
        const GpView &v = c < 3 ? a.gv : a.gw;
        gmk[c] = a.use_gp ? sm * v.ystd[c % 3] + v.ymean[c % 3] : 0.0;
      }
      double xn[R6_NX];
      if (relin) {
        for (int i = 0; i < R6_NX; ++i) xn[i] = X[k + 1][i];
      } else {  // gp_mpc.py:166-168
        for (int i = 0; i < R6_NX; ++i) xn[i] = xrk[i];
        for (int i = 0; i < 3; ++i) { xn[4 + i] += gmk[i] * dt; xn[11 + i] += gmk[3 + i] * dt; }
      }
      if (wave == 0) {
        if (out_here)
          for (int c = 0; c < 6; ++c) a.gm[((int64_t)b * R6_N + k) * 6 + c] = gmk[c];
        if (!relin)
          for (int i = 0; i < R6_NX; ++i) X[k + 1][i] = xn[i];
      }
      if (a.use_gp && k + 1 < R6_N)  // the next point's features, from this lane's own copy of X[k+1]
        r6_features_role(wave, xn, Ub + (k + 1) * R6_NU, a.gv.ls, a.gw.ls, zq[0], zq[1]);
    }
    __syncthreads();
    mark(0);
  }
  if (!out_here) return;
  for (int e = tid; e < (R6_N + 1) * R6_NX; e += R6_PT)
    a.Xp[(int64_t)b * (R6_N + 1) * R6_NX + e] = (&X[0][0])[e];
  // linearisation at the simulated points (gp_mpc.py:303-304): -[A_d | B_d] per stage
  double *lin = a.lin + (int64_t)b * R6_N * R6_NX * R6_SZ;
  for (int e = tid; e < R6_N * R6_NX * R6_SZ; e += R6_PT) lin[e] = 0.0;
  __syncthreads();
  if (tid < R6_N) r6_neg_lin(a.rk, X[tid], Ub + tid * R6_NU, dt, lin + tid * R6_NX * R6_SZ);
  if (ST && b == 0) {
    __syncthreads();
    if (tid == 0) g_r6p_stamps[4] += __builtin_amdgcn_s_memtime() - tl;
  }
}

// ---------------------------------------------------------------------------
// 2. QP + ADMM + plant
struct R6Smem {
  double Sinv[R6_NBLK * R6_TRI];      // packed lower S_k^-1 (D_k during the assembly)
  double G[R6_N * R6_NX * R6_SZ];     // staged dynamics rows (scaled), then G_k = C_k S_k^-1
  double rhs[R6_NBLK * R6_SZ];        // x~ right-hand side, forward chain y
  double xs[R6_NBLK * R6_SZ];         // diagonal products u, backward chain x = x~
  double w[R6_MD + R6_MGEN];          // rho z - y of equality + general rows (scratch at checks)
  double E[R6_M];                     // row scaling
  double dsc[R6_NV];                  // per-pass column scaling / factor scratch
  double dpl[R6_MD];                  // each equality row's identity entry (scaled)
  double gen[R6_MGEN * 3];            // general rows' values (scaled)
  // per end of the twisted sweep (0 top, 1 bottom):
  double T[2][2][R6_TRI];             // the swept block, packed lower (ping-pong: one barrier per step)
  double Ct[2][R6_NX * R6_SZ];        // the coupling C_k (top) / E_k (bottom), 14 x 17
  double Sch[2][R6_NX * R6_NX];       // G_k C_k^T / H_k E_k^T, the next block's update
  double red[16][12];
  double zero[R6_SZ];                 // the forward chain's operand row for its pass-through lanes
  double zmid[16];                    // the bottom chain's z'_15 = -H_15 z_16
  double dump[64];                    // the chains' store target for lanes that keep no result
  double c, rho_s;
  int flag, bad[2];
};

// threadIdx.x behind an opaque copy (R6_LAUNDER): the phases of the ADMM loop derive
// their addresses from it afresh on every iteration instead of from hoisted registers
__device__ __forceinline__ int r6_tid() {
  int t = threadIdx.x;
#if R6_LAUNDER
  asm volatile("" : "+v"(t));
#endif
  return t;
}

__device__ __forceinline__ int r6_tri(int a, int b) { return a >= b ? a * (a + 1) / 2 + b : b * (b + 1) / 2 + a; }

template <int K>
__device__ __forceinline__ void r6_max(double (&v)[K], double (*red)[12]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] = fmax(v[k], __shfl_xor(v[k], o));
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[wv][k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double m = red[0][k];
    for (int w = 1; w < R6_T / 64; ++w) m = fmax(m, red[w][k]);
    v[k] = m;
  }
  __syncthreads();
}

template <int K>
__device__ __forceinline__ void r6_sum(double (&v)[K], double (*red)[12]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[wv][k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = red[0][k];
    for (int w = 1; w < R6_T / 64; ++w) s += red[w][k];
    v[k] = s;
  }
  __syncthreads();
}

__device__ __forceinline__ double r6_rho(double l, double u, double rs) {
  if (l < -QP_OSQP_INFTY * QP_MIN_SCALING && u > QP_OSQP_INFTY * QP_MIN_SCALING) return QP_RHO_MIN;
  if (u - l < QP_RHO_TOL) return QP_RHO_EQ * rs;
  return rs;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// general row g: its entries (count, variables, value slots)
__device__ __forceinline__ int r6_gen_cols(int g, int *col) {
  if (g < R6_MT) {
    const int o = g * R6_SZ + R6_NX;
    col[0] = o; col[1] = o + 1; col[2] = o + 2;
    return 3;
  }
  const int gg = g - R6_MT, k = 1 + gg / 4, c = gg % 4;
  col[0] = k * R6_SZ + 1;
  col[1] = k * R6_SZ + (c < 2 ? 2 : 3);
  return 2;
}

// the e-th general-row entry (e < 4) of variable (k, i) in row order: its
// general row g and value slot sl; false past the variable's entries
__device__ __forceinline__ bool r6_gen_slot(int k, int i, int e, int &g, int &sl) {
  if (k < R6_N && i >= R6_NX) {  // thrust row k
    g = k; sl = i - R6_NX;
    return e == 0;
  }
  if (k >= 1 && k < R6_N && i >= 1 && i <= 3) {  // glideslope rows of stage k
    const int g0 = R6_MT + 4 * (k - 1);
    g = g0 + (i == 3 ? 2 : 0) + e;
    sl = (i == 1) ? 0 : 1;
    return e < (i == 1 ? 4 : 2);
  }
  g = 0; sl = 0;
  return false;
}

struct R6Var {  // variable j and its bound row MD + j; general row j (< 146)
  bool ok;
  int j, k, i;
  double x, P, q, D, Ab, lb, ub, yb, zb;
  // colA[0..13]: -A_d[:, i] / -B_d[:, i-14] of the dynamics rows of block k
  // (scaled).  An equality-row thread (no variable) keeps its row here instead.
  double colA[R6_SZ + 1];
  bool gok;
  int gn;
  double gA[3], gl, gu, gy, gz;
};
// an item's changes of one ADMM iteration (dx, the bound row's / equality row's dy,
// the general row's dy): read by that iteration's termination checks only, so they
// live in the iteration's scope instead of the items' persistent registers
struct R6Dy {
  double dx, dyb, gdy;
};
// equality row r (x0 row r < 14, else dynamics row (k, i)).  Rows and variables
// live on different threads, so the row's registers alias the variable slots.
struct R6Row {
  bool ok;
  int r, k, i;
  double (&A)[R6_SZ + 1];
  double &ur, &yr, &zr;
  __device__ explicit R6Row(R6Var &V) : A(V.colA), ur(V.lb), yr(V.yb), zr(V.zb) {}
};

__device__ __forceinline__ int r6_eqid_row(int k, int i) { return k == 0 ? i : R6_NX + R6_NX * (k - 1) + i; }

// (A' w)_j in row order: equality identity row, dynamics rows of block k, bound row, general rows
__device__ __forceinline__ double r6_col_dot(const R6Smem &s, const R6Var &V, const double *wv, double wb,
                                             const double *wg) {
  double acc = 0.0;
  if (V.i < R6_NX) {
    const int r = r6_eqid_row(V.k, V.i);
    acc += s.dpl[r] * wv[r];
  }
  if (V.k < R6_N) {
    const double *wr = wv + R6_NX + R6_NX * V.k;
#pragma unroll
    for (int e = 0; e < R6_NX; ++e) acc += V.colA[e] * wr[e];
  }
  acc += V.Ab * wb;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int g, sl;
    if (r6_gen_slot(V.k, V.i, e, g, sl)) acc += s.gen[g * 3 + sl] * wg[g];
  }
  return acc;
}

__device__ __forceinline__ double r6_row_dot(const R6Row &R, const double *v) {
  if (R.r < R6_NX) return 0.0 + R.A[0] * v[R.r];
  const double *vb = v + R.k * R6_SZ;
  double acc = 0.0;
#pragma unroll
  for (int e = 0; e < R6_SZ; ++e) acc += R.A[e] * vb[e];
  acc += R.A[R6_SZ] * v[(R.k + 1) * R6_SZ + R.i];
  return acc;
}
__device__ __forceinline__ double r6_gen_dot(const R6Var &V, const double *v) {
  int col[3];
  const int n = r6_gen_cols(V.j, col);
  double acc = 0.0;
#pragma unroll
  for (int e = 0; e < 3; ++e)
    if (e < n) acc += V.gA[e] * v[col[e]];
  return acc;
}

// The reduced KKT matrix M = P + sigma I + A' R A is block tridiagonal.  It is
// factored from both ends at once (the 3-DoF fleet's twist, fleet_twist.h), in
// 31 factor blocks of natural variables (r6_nat):
//   top     k = 0..14:  the stage block [x_k, u_k], coupled to x_k+1 through
//                       C_k (14 x 17: rho_eq dpl(k, i) g_k[i][:], stage k's dynamics rows);
//   middle  k = 15:     x_15 alone (14 x 14);
//   bottom  k = 16..30: [x_k, u_k-1], coupled to x_k-1 through E_k-1 (14 x 17:
//                       x_k columns from stage k-1's dynamics rows, u_k-1
//                       columns from stage k-1's x-u block).
// Neither end's coupling reaches a block's entries 14-16 (u_k on top, u_k-1 at the
// bottom), so the two ends are the same recursion, 15 block steps each:
//   top     S_0 = D_0,   S_k+1 = D_k+1 - G_k C_k^T,      G_k = C_k S_k^-1
//   bottom  T_30 = D_30, T_k-1 = D_k-1 - H_k-1 E_k-1^T,  H_k-1 = E_k-1 T_k^-1
//   middle  Z = D_15 - G_14 C_14^T - H_15 E_15^T
// -G_k goes to slot k (k < 15) and -H_k to slot k (k = 15..29) of s.G, over the
// staged dynamics rows of its own stage once their last reader is done.
// the middle block x_MID; the top end runs MID block steps, the bottom end BOTS = N - MID
// (one fewer for an odd N: it then idles through the top's last step)
#define R6_MID ((R6_N + 1) / 2)
#define R6_BOTS (R6_N - R6_MID)

__device__ __forceinline__ int r6_nat(int k, int e) {
  return k * R6_SZ + e - ((k > R6_MID && e >= R6_NX) ? R6_SZ : 0);
}

// M entry of variables (k, a) and (k, bb) of one stage, the terms in the banded oracle's row order
__device__ __forceinline__ double r6_m_stage(const R6Smem &s, int k, int a, int bb, double re, double rs) {
  double v = 0.0;
  if (a == bb) {
    v = s.dsc[k * R6_SZ + a];
    if (a < R6_NX) {
      const int r = r6_eqid_row(k, a);
      v += re * s.dpl[r] * s.dpl[r];
    }
  }
  if (k < R6_N) {
    const double *g = s.G + k * R6_NX * R6_SZ;
    for (int i = 0; i < R6_NX; ++i) v += re * g[i * R6_SZ + a] * g[i * R6_SZ + bb];
  }
  if (a == bb) v += s.xs[k * R6_SZ + a];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    int g1, s1;
    if (!r6_gen_slot(k, a, p, g1, s1)) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int g2, s2;
      if (r6_gen_slot(k, bb, q, g2, s2) && g1 == g2) v += rs * s.gen[g1 * 3 + s1] * s.gen[g2 * 3 + s2];
    }
  }
  return v;
}
// M entry of x_k+1[i] and (k, e): dynamics row (k, i) alone
__device__ __forceinline__ double r6_m_next(const R6Smem &s, int k, int i, int e, double re) {
  return (re * s.dpl[R6_NX + R6_NX * k + i]) * s.G[(k * R6_NX + i) * R6_SZ + e];
}

// (row, column) of packed-lower entry t
__device__ __forceinline__ void r6_untri(int t, int &i, int &j) {
  i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while (i * (i + 1) / 2 > t) --i;
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  j = t - i * (i + 1) / 2;
}

// The block inverse by the symmetric sweep operator on the packed lower triangle
// (153 entries instead of Gauss-Jordan's 289: the block is SPD, so every
// intermediate is symmetric), two pivots P = {p, p + 1} per barrier:
//   W'[P][P] = -A^-1,  W'[i][P] = W[i][P] A^-1,  W'[i][j] = W[i][j] - W[i][P] A^-1 W[P][j]
// with A = W[P][P]; after all pivots W = -S^-1.  Thread lt owns entry lt of T[0]
// (one entry per thread); the result lands in T[return value].
__device__ __forceinline__ int r6_sweep(double (*T)[R6_TRI], int lt, int nb, int kfail, int &bad) {
  const bool own = lt < nb * (nb + 1) / 2;
  int i = 0, j = 0;  // recomputed per call: kept live across the sweep loop they spilled more
  if (own) r6_untri(lt, i, j);
  int cb = 0;
  for (int p = 0; p < nb; p += 2) {
    const double *W = T[cb];
    double v = 0.0;
    if (p + 1 < nb) {
      const double a = W[r6_tri(p, p)], b = W[r6_tri(p + 1, p)], d = W[r6_tri(p + 1, p + 1)];
      const double det = fma(a, d, -(b * b));
      if (!(a > 0.0 && det > 0.0) && !bad) bad = kfail;  // both pivots positive (uniform)
      // 1/det by v_rcp_f64 + two Newton steps (blk_recip, within an ulp of the division)
      const double rd = blk_recip(det);
      const double ia = d * rd, ib = -b * rd, id = a * rd;  // A^-1 = [ia ib; ib id]
      if (own) {
        const double wij = W[lt];
        const double wip = W[r6_tri(i, p)], wiq = W[r6_tri(i, p + 1)];
        const double wjp = W[r6_tri(j, p)], wjq = W[r6_tri(j, p + 1)];
        const int di = i - p, dj = j - p;  // i >= j
        const bool ip = di == 0 || di == 1, jp = dj == 0 || dj == 1;
        if (ip && jp) v = -(di + dj == 0 ? ia : (di + dj == 1 ? ib : id));
        else if (jp) v = dj == 0 ? wip * ia + wiq * ib : wip * ib + wiq * id;  // W[i][P] A^-1
        else if (ip) v = di == 0 ? ia * wjp + ib * wjq : ib * wjp + id * wjq;  // A^-1 W[P][j]
        else v = wij - ((wip * ia + wiq * ib) * wjp + (wip * ib + wiq * id) * wjq);
      }
    } else {
      const double d = W[r6_tri(p, p)];
      if (!(d > 0.0) && !bad) bad = kfail;
      const double inv = blk_recip(d);
      if (own) {
        const double wij = W[lt], wip = W[r6_tri(i, p)], wjp = W[r6_tri(j, p)];
        if (i == p && j == p) v = -inv;
        else if (j == p) v = wip * inv;
        else if (i == p) v = wjp * inv;
        else v = wij - (wip * inv) * wjp;
      }
    }
    if (own) T[cb ^ 1][lt] = v;
    cb ^= 1;
    __syncthreads();
  }
  return cb;
}

// assemble M and factor it: returns 0 or a failing block + 1
template <class MK>
__device__ __forceinline__ int r6_factor(R6Smem &s, R6Var (&V)[2], R6Row (&R)[2], double sigma, MK &mark) {
  const int tid = r6_tid();
  const double rs = s.rho_s, re = QP_RHO_EQ * rs;
  // stage: dynamics rows' block values, per-variable P + sigma and bound terms
  R6_FOR_H {
    if (R[h].ok && R[h].r >= R6_NX)
#pragma unroll
      for (int e = 0; e < R6_SZ; ++e) s.G[(R[h].k * R6_NX + R[h].i) * R6_SZ + e] = R[h].A[e];
    if (V[h].ok) {
      s.dsc[V[h].j] = V[h].P + sigma;
      s.xs[V[h].j] = r6_rho(V[h].lb, V[h].ub, rs) * V[h].Ab * V[h].Ab;
    }
  }
  __syncthreads();
  // the 31 diagonal blocks, packed lower
  for (int e = tid; e < R6_NBLK * R6_TRI; e += R6_T) {
    const int k = e / R6_TRI, t = e - k * R6_TRI;
    int a = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (a * (a + 1) / 2 > t) --a;
    while ((a + 1) * (a + 2) / 2 <= t) ++a;
    const int bb = t - a * (a + 1) / 2;
    const int nb = (k == R6_MID) ? R6_NX : R6_SZ;
    double v = 0.0;
    if (a < nb) {
      if (k <= R6_MID || a < R6_NX) v = r6_m_stage(s, k, a, bb, re, rs);  // bb <= a
      else if (bb >= R6_NX) v = r6_m_stage(s, k - 1, a, bb, re, rs);      // u_k-1 with u_k-1
      else v = r6_m_next(s, k - 1, bb, a, re);                             // x_k[bb] with u_k-1
    } else if (a == bb) {
      v = 1.0;  // unused tail of the middle block
    }
    s.Sinv[e] = v;
  }
  __syncthreads();
  mark(2);  // (stamps: the assembly)
  // the sweep: threads 0-255 the top end, 256-511 the bottom end.  The pivot
  // steps read one copy of the block and write the other, so a step needs one
  // workgroup barrier instead of two.
  const int half = tid >> 8, lt = tid & 255;
  int bad = 0;
  for (int t = 0; t < R6_MID; ++t) {
    // an odd N: the bottom end has one block step fewer, and sweeps an identity block
    // through the top's last step (the sweep's barriers are the workgroup's), storing nothing
    const bool idle = half && t >= R6_BOTS;
    const int k = half ? (idle ? R6_N : R6_N - t) : t;  // factor block
    const int kc = half ? k - 1 : k;      // its coupling's slot
    double (*T)[R6_TRI] = s.T[half];
    if (lt < R6_TRI) {
      int ti, tj;
      r6_untri(lt, ti, tj);
      double v = s.Sinv[k * R6_TRI + lt];
      if (t > 0 && ti < R6_NX) v -= s.Sch[half][ti * R6_NX + tj];  // tj <= ti
      T[0][lt] = idle ? (ti == tj ? 1.0 : 0.0) : v;
    }
    if (!idle && lt < R6_NX * R6_SZ) {  // top C_k[i][c]: x_k+1[i] with (k, c); bottom E_k-1[i][c]: x_k-1[i] with entry c of block k
      const int i = lt / R6_SZ, c = lt - i * R6_SZ;
      double v;
      if (!half) v = r6_m_next(s, k, i, c, re);
      else if (c < R6_NX) v = r6_m_next(s, k - 1, c, i, re);
      else v = r6_m_stage(s, k - 1, i, c, re, rs);
      s.Ct[half][lt] = v;
    }
    __syncthreads();
    const int cb = r6_sweep(T, lt, R6_SZ, k + 1, bad);  // W = -S_k^-1; bad: uniform over the half
    if (!idle && lt < R6_TRI) s.Sinv[k * R6_TRI + lt] = -T[cb][lt];
    mark(10);
    // -G_k = -C_k S_k^-1 = C_k W / -H_k-1 over the staged rows of its slot
    double *Gs = s.G + kc * R6_NX * R6_SZ;
    if (!idle && lt < R6_NX * R6_SZ) {
      const int i = lt / R6_SZ, c = lt - i * R6_SZ;
      double acc = 0.0;
      for (int e = 0; e < R6_SZ; ++e) acc += s.Ct[half][i * R6_SZ + e] * T[cb][r6_tri(e, c)];
      Gs[lt] = acc;  // stored negated: the chains accumulate
    }
    __syncthreads();
    if (!idle && lt < R6_NX * R6_NX) {  // the next block's update G_k C_k^T / H_k-1 E_k-1^T (14 x 14)
      const int i = lt / R6_NX, i2 = lt - i * R6_NX;
      double acc = 0.0;
      for (int e = 0; e < R6_SZ; ++e) acc += Gs[i * R6_SZ + e] * s.Ct[half][i2 * R6_SZ + e];
      s.Sch[half][lt] = -acc;
    }
    __syncthreads();
    mark(11);
  }
  // the middle block Z = D_15 - G_14 C_14^T - H_15 E_15^T, 14 wide (packed: the first 105)
  double (*T)[R6_TRI] = s.T[0];
  constexpr int MT = R6_NX * (R6_NX + 1) / 2;
  if (tid < MT) {
    int mi, mj;
    r6_untri(tid, mi, mj);
    T[0][tid] = (s.Sinv[R6_MID * R6_TRI + tid] - s.Sch[0][mi * R6_NX + mj]) - s.Sch[1][mi * R6_NX + mj];
  }
  __syncthreads();
  const int cb = r6_sweep(T, tid, R6_NX, R6_MID + 1, bad);
  if (tid < R6_TRI) s.Sinv[R6_MID * R6_TRI + tid] = tid < MT ? -T[cb][tid] : 0.0;
  if (lt == 0) s.bad[half] = bad;
  __syncthreads();
  mark(10);
  return s.bad[0] ? s.bad[0] : s.bad[1];
}

// u = S_k^-1 y_k, row a of factor block k (the middle block on y_15 + z'_15)
__device__ __forceinline__ void r6_diag_row(R6Smem &s, int k, int a) {
  const int e = k * R6_SZ + a;
  const int nb = (k == R6_MID) ? R6_NX : R6_SZ;
  if (a < nb) {
    const double *S = s.Sinv + k * R6_TRI;
    const double *y = s.rhs + k * R6_SZ;
    const int lo = k > R6_MID ? R6_SZ : 0;   // a bottom block's u_k-1 one block down
    const bool mid = k == R6_MID;
    // unrolled over the 17 entries (the middle block's 3 masked) in three chunks
    // of loads in flight (a runtime-count loop waited on each pair; all 17 at
    // once spilled the items' registers)
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int c0 = 0; c0 < R6_SZ; c0 += R6_DIAG_CHUNK) {
      double sv[R6_DIAG_CHUNK], yv[R6_DIAG_CHUNK];
#pragma unroll
      for (int q = 0; q < R6_DIAG_CHUNK; ++q) {
        const int bb = c0 + q < R6_SZ ? c0 + q : R6_SZ - 1;
        sv[q] = S[r6_tri(a, bb)];
        yv[q] = y[bb >= R6_NX ? bb - lo : bb];
        if (bb < R6_NX && mid) yv[q] += s.zmid[bb];
      }
#pragma unroll
      for (int q = 0; q < R6_DIAG_CHUNK; ++q) {
        const int bb = c0 + q;
        if (bb >= R6_SZ) continue;
        if (bb & 1) acc1 = bb < nb ? fma(sv[q], yv[q], acc1) : acc1;
        else acc0 = bb < nb ? fma(sv[q], yv[q], acc0) : acc0;
      }
      asm volatile("" ::: "memory");
    }
    s.xs[a >= R6_NX ? e - lo : e] = acc0 + acc1;
  }
}

// the sum of a lane's value and its partner's in the other row of its row pair
// (rows 0/1, 2/3): v_permlane16_swap on both halves, one add; both rows get the
// same bits (the add commutes)
__device__ __forceinline__ double pair_sum(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}
// rows 1 and 3 rotated by 8 lanes (DPP row_ror:8 on both halves); rows 0, 2 unchanged
__device__ __forceinline__ double ror8_odd(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int l = __builtin_amdgcn_update_dpp(lo, lo, 0x128, 0xa, 0xf, false);
  const int h = __builtin_amdgcn_update_dpp(hi, hi, 0x128, 0xa, 0xf, false);
  return __hiloint2double(h, l);
}

// x~ = M^-1 rhs, twisted: the forward chains (wave 0: y down the top blocks to
// y_15; wave 1: z up the bottom blocks, then z'_15 = -H_15 z_16), the 31 diagonal
// products (the middle on y_15 + z'_15), the backward chains (wave 0: x_14 .. x_0
// from x_15; wave 1: blocks 16 .. 30 from x_15).  The chains carry their vector
// in registers and broadcast it with DPP row_newbcast inside the FMA (qp_block.h
// fmac_bc), as the 3-DoF fleet does; blocks are 17 wide and a DPP row 16:
//   forward  row 0, lane i < 14: entry i of the next block; lanes 14, 15 carry
//            the block's entries 14, 15 (which no coupling reaches) through zero
//            operands, and entry 16's term goes into the init off the chain.
//   backward lanes 0-15 compute entries 0-15, lanes 16-29 replicate entries
//            0-13 (so row 1 broadcasts the same x) and lane 30 computes entry 16.
// Both ends run the same instruction stream; a bottom block's entries 14-16
// (u_k-1) sit 17 below its x_k in the natural order (offsets rr - 17).
template <class MK>
__device__ __forceinline__ void r6_solve(R6Smem &s, MK &mark) {
  const int tid = r6_tid(), wv = tid >> 6, lane = tid & 63;
  if (wv < 2) {
    // Two DPP rows per end: row h = 0 takes terms 0-7 and row 1 terms 8-15 of the
    // 16 on the chain, row 1 holding the vector rotated by 8 lanes so that its
    // broadcasts 0-7 reach entries 8-15; the pair sum (v_permlane16_swap) gives both
    // rows the new entry and row 1 rotates it back.  Half the dependent FMAs and half
    // the operand reads per block step.  Rows 2 and 3 repeat rows 0 and 1.
    // Every term's operand pair for the NEXT step loads right after the pair's FMAs.
    const bool bot = wv == 1;
    const int m = lane & 15, h = (lane >> 4) & 1;
    const int ms = h ? (m + 8) & 15 : m;  // the entry this lane's vector register holds
    const bool pass = m >= R6_NX;         // output m: a pass-through entry (14, 15)
    auto offo = [&](int e) { return (bot && e >= R6_NX) ? e - R6_SZ : e; };
    const int o16 = bot ? -1 : R6_SZ - 1;
    const int db = bot ? -R6_SZ : R6_SZ;
    const int gs = pass ? 0 : (bot ? -R6_NX * R6_SZ : R6_NX * R6_SZ);
    const double *F = s.G;
    int go = pass ? (int)(s.zero - s.G) : (bot ? R6_N - 1 : 0) * R6_NX * R6_SZ + m * R6_SZ;
    const int gh = 8 * h;
    int ib = bot ? R6_N * R6_SZ : 0;
    double g[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = F[go + gh + e];
    double g16 = F[go + R6_SZ - 1];
    double y = s.rhs[ib + offo(ms)];
    double b16 = s.rhs[ib + o16], bn = s.rhs[ib + db + offo(m)];
    // block steps of this end (wave-uniform; a compile-time count for an even N)
    const int nst = (R6_BOTS == R6_MID) ? R6_MID : (bot ? R6_BOTS : R6_MID);
_Pragma(R6_STR(unroll R6_CHAIN_UNROLL))
    for (int t = 0; t < nst; ++t) {
      const bool last = t == nst - 1;
      const int gn = go + gs;
      const double init = h ? 0.0 : fma(g16, b16, (bot && last) ? 0.0 : bn);
      b16 = s.rhs[ib + db + o16];
      bn = s.rhs[ib + 2 * db + offo(m)];
      g16 = F[gn + R6_SZ - 1];
      double a0 = init, a1 = 0.0;
      fmac_bc<0, true>(a0, y, g[0]); fmac_bc<1, false>(a1, y, g[1]);
      g[0] = F[gn + gh + 0]; g[1] = F[gn + gh + 1];
      fmac_bc<2, false>(a0, y, g[2]); fmac_bc<3, false>(a1, y, g[3]);
      g[2] = F[gn + gh + 2]; g[3] = F[gn + gh + 3];
      fmac_bc<4, false>(a0, y, g[4]); fmac_bc<5, false>(a1, y, g[5]);
      g[4] = F[gn + gh + 4]; g[5] = F[gn + gh + 5];
      fmac_bc<6, false>(a0, y, g[6]); fmac_bc<7, false>(a1, y, g[7]);
      g[6] = F[gn + gh + 6]; g[7] = F[gn + gh + 7];
      const double sum = pair_sum(a0 + a1);  // entry m of the next block, on both rows
      y = ror8_odd(sum);
      // unconditional store (pass-through and idle lanes to the dump): no
      // exec-mask branch in the loop, so the LDS wait at the next step is exact
      double *dst = (!pass && lane < 16) ? ((bot && last) ? &s.zmid[m] : &s.rhs[ib + db + m]) : &s.dump[lane];
      *dst = sum;
      go = gn;
      ib += db;
      // the two ends walk in opposite directions, so a step's address is no
      // immediate offset from one base; left visible, the compiler hoists every
      // step's address out of the ADMM loop as a live register
      asm volatile("" : "+v"(ib), "+v"(go));
    }
  }
  __syncthreads();
  mark(4);
  for (int e = tid; e < R6_NBLK * R6_SZ; e += R6_T) r6_diag_row(s, e / R6_SZ, e % R6_SZ);
  __syncthreads();
  mark(5);
  if (wv < 2) {
    const bool bot = wv == 1;
    // entry a of lane (0-15: a = lane, 16-29: a = lane - 16, 30: 16); lanes >= 31
    // compute entry 16 too and drop it
    const int a = lane < 16 ? lane : (lane < 30 ? lane - 16 : R6_SZ - 1);
    const bool st = lane < 16 || lane == 30;
    const int off = (bot && a >= R6_NX) ? a - R6_SZ : a;
    // top: blocks 14 .. 0 (slots 14 .. 0); bottom: blocks 16 .. 30 (slots 15 .. 29)
    const int gs = bot ? R6_NX * R6_SZ : -R6_NX * R6_SZ;
    const int db = bot ? R6_SZ : -R6_SZ;
    const double *F = s.G;
    int go = (R6_MID - (bot ? 0 : 1)) * R6_NX * R6_SZ + a;
    int ib = (bot ? R6_MID + 1 : R6_MID - 1) * R6_SZ;
    double g[R6_NX];
#pragma unroll
    for (int i = 0; i < R6_NX; ++i) g[i] = F[go + i * R6_SZ];
    double x = a < R6_NX ? s.xs[R6_MID * R6_SZ + a] : 0.0;
    double u = s.xs[ib + off];
    // block steps of this end (wave-uniform; a compile-time count for an even N)
    const int nst = (R6_BOTS == R6_MID) ? R6_MID : (bot ? R6_BOTS : R6_MID);
_Pragma(R6_STR(unroll R6_CHAIN_UNROLL))
    for (int t = 0; t < nst; ++t) {
      const int gn = min(max(go + gs, a), (R6_N - 1) * R6_NX * R6_SZ + a);
      double a0 = u, a1 = 0.0;
      u = s.xs[min(max(ib + db, 0), R6_N * R6_SZ) + off];
      fmac_bc<0, true>(a0, x, g[0]); fmac_bc<1, false>(a1, x, g[1]);
      g[0] = F[gn + 0 * R6_SZ]; g[1] = F[gn + 1 * R6_SZ];
      fmac_bc<2, false>(a0, x, g[2]); fmac_bc<3, false>(a1, x, g[3]);
      g[2] = F[gn + 2 * R6_SZ]; g[3] = F[gn + 3 * R6_SZ];
      fmac_bc<4, false>(a0, x, g[4]); fmac_bc<5, false>(a1, x, g[5]);
      g[4] = F[gn + 4 * R6_SZ]; g[5] = F[gn + 5 * R6_SZ];
      fmac_bc<6, false>(a0, x, g[6]); fmac_bc<7, false>(a1, x, g[7]);
      g[6] = F[gn + 6 * R6_SZ]; g[7] = F[gn + 7 * R6_SZ];
      fmac_bc<8, false>(a0, x, g[8]); fmac_bc<9, false>(a1, x, g[9]);
      g[8] = F[gn + 8 * R6_SZ]; g[9] = F[gn + 9 * R6_SZ];
      fmac_bc<10, false>(a0, x, g[10]); fmac_bc<11, false>(a1, x, g[11]);
      g[10] = F[gn + 10 * R6_SZ]; g[11] = F[gn + 11 * R6_SZ];
      fmac_bc<12, false>(a0, x, g[12]); fmac_bc<13, false>(a1, x, g[13]);
      g[12] = F[gn + 12 * R6_SZ]; g[13] = F[gn + 13 * R6_SZ];
      x = a0 + a1;
      *(st ? &s.xs[ib + off] : &s.dump[lane]) = x;
      go = gn;
      ib += db;
      asm volatile("" : "+v"(ib), "+v"(go));
    }
  }
  __syncthreads();
  mark(6);
}

// residual norms (auxil.c update_info) + the rho-estimate quantities (as fq_update_info)
__device__ __forceinline__ void r6_update_info(R6Smem &s, R6Var (&V)[2], R6Row (&R)[2], double (&o)[8],
                                               double (&re_)[4]) {
  R6_FOR_H {
    if (V[h].ok) s.rhs[V[h].j] = V[h].x;
    if (R[h].ok) s.w[R[h].r] = R[h].yr;
    if (V[h].gok) s.w[R6_MD + V[h].j] = V[h].gy;
  }
  __syncthreads();
  double v[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  auto row = [&](double ax, double z, double e) {
    v[0] = fmax(v[0], fabs((ax - z) / e));
    v[1] = fmax(v[1], fabs(z / e));
    v[2] = fmax(v[2], fabs(ax / e));
    v[8] = fmax(v[8], fabs(ax - z));
    v[9] = fmax(v[9], fmax(fabs(z), fabs(ax)));
  };
  R6_FOR_H {
    R6Var &W = V[h];
    if (R[h].ok) row(r6_row_dot(R[h], s.rhs), R[h].zr, s.E[R[h].r]);
    if (W.ok) {
      row(0.0 + W.Ab * W.x, W.zb, s.E[R6_MD + W.j]);
      const double aty = r6_col_dot(s, W, s.w, W.yb, s.w + R6_MD);
      const double px = W.P * W.x, d = W.D, q = W.q;
      v[3] = fmax(v[3], fabs((q + px + aty) / d));
      v[4] = fmax(v[4], fabs(q / d));
      v[5] = fmax(v[5], fabs(aty / d));
      v[6] = fmax(v[6], fabs(px / d));
      v[10] = fmax(v[10], fabs(q + px + aty));
      v[11] = fmax(v[11], fmax(fmax(fabs(q), fabs(aty)), fabs(px)));
    }
    if (W.gok) row(r6_gen_dot(W, s.rhs), W.gz, s.E[R6_MD + R6_NV + W.j]);
  }
  r6_max<12>(v, s.red);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = v[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) re_[k] = v[8 + k];
}

__device__ __forceinline__ double r6_proj(double d, double l, double u) {
  const bool bu = u > QP_OSQP_INFTY * QP_MIN_SCALING, bl = l < -QP_OSQP_INFTY * QP_MIN_SCALING;
  if (bu && bl) return 0.0;
  if (bu) return fmin(d, 0.0);
  if (bl) return fmax(d, 0.0);
  return d;
}

__device__ __forceinline__ bool r6_primal_infeasible(R6Smem &s, R6Var (&V)[2], R6Row (&R)[2], R6Dy (&Dl)[2],
                                                     double eps) {
  double v[1] = {0.0};
  R6_FOR_H {
    R6Var &W = V[h];
    R6Row &Q = R[h];
    R6Dy &d = Dl[h];
    if (Q.ok) { d.dyb = r6_proj(d.dyb, Q.ur, Q.ur); v[0] = fmax(v[0], fabs(s.E[Q.r] * d.dyb)); }
    if (W.ok) { d.dyb = r6_proj(d.dyb, W.lb, W.ub); v[0] = fmax(v[0], fabs(s.E[R6_MD + W.j] * d.dyb)); }
    if (W.gok) { d.gdy = r6_proj(d.gdy, W.gl, W.gu); v[0] = fmax(v[0], fabs(s.E[R6_MD + R6_NV + W.j] * d.gdy)); }
  }
  r6_max<1>(v, s.red);
  const double nrm = v[0];
  if (!(nrm > QP_DIV_TOL)) return false;
  double sm[1] = {0.0};
  R6_FOR_H {
    R6Var &W = V[h];
    R6Row &Q = R[h];
    const R6Dy &d = Dl[h];
    if (Q.ok) sm[0] += Q.ur * fmax(d.dyb, 0.0) + Q.ur * fmin(d.dyb, 0.0);
    if (W.ok) sm[0] += W.ub * fmax(d.dyb, 0.0) + W.lb * fmin(d.dyb, 0.0);
    if (W.gok) sm[0] += W.gu * fmax(d.gdy, 0.0) + W.gl * fmin(d.gdy, 0.0);
  }
  r6_sum<1>(sm, s.red);
  if (!(sm[0] < -eps * nrm)) return false;
  R6_FOR_H {
    if (R[h].ok) s.w[R[h].r] = Dl[h].dyb;
    if (V[h].gok) s.w[R6_MD + V[h].j] = Dl[h].gdy;
  }
  __syncthreads();
  double mx[1] = {0.0};
  R6_FOR_H {
    if (V[h].ok) mx[0] = fmax(mx[0], fabs(r6_col_dot(s, V[h], s.w, Dl[h].dyb, s.w + R6_MD) / V[h].D));
  }
  r6_max<1>(mx, s.red);
  return mx[0] < eps * nrm;
}

__device__ __forceinline__ bool r6_dual_infeasible(R6Smem &s, R6Var (&V)[2], R6Row (&R)[2], const R6Dy (&Dl)[2],
                                                   double eps) {
  double v[1] = {0.0};
  R6_FOR_H {
    if (V[h].ok) v[0] = fmax(v[0], fabs(V[h].D * Dl[h].dx));
  }
  r6_max<1>(v, s.red);
  const double nrm = v[0];
  if (!(nrm > QP_DIV_TOL)) return false;
  double a[1] = {0.0}, pm[1] = {0.0};
  R6_FOR_H {
    if (V[h].ok) { a[0] += V[h].q * Dl[h].dx; pm[0] = fmax(pm[0], fabs(V[h].P * Dl[h].dx / V[h].D)); }
  }
  r6_sum<1>(a, s.red);
  r6_max<1>(pm, s.red);
  if (!(a[0] < s.c * eps * nrm)) return false;
  if (!(pm[0] < s.c * eps * nrm)) return false;
  R6_FOR_H {
    if (V[h].ok) s.rhs[V[h].j] = Dl[h].dx;
  }
  __syncthreads();
  double bad[1] = {0.0};
  auto test = [&](double vv, double l, double u) {
    if ((u < QP_OSQP_INFTY * QP_MIN_SCALING && vv > eps * nrm) ||
        (l > -QP_OSQP_INFTY * QP_MIN_SCALING && vv < -eps * nrm))
      bad[0] = 1.0;
  };
  R6_FOR_H {
    R6Var &W = V[h];
    if (R[h].ok) test(r6_row_dot(R[h], s.rhs) / s.E[R[h].r], R[h].ur, R[h].ur);
    if (W.ok) test((0.0 + W.Ab * Dl[h].dx) / s.E[R6_MD + W.j], W.lb, W.ub);
    if (W.gok) test(r6_gen_dot(W, s.rhs) / s.E[R6_MD + R6_NV + W.j], W.gl, W.gu);
  }
  r6_max<1>(bad, s.red);
  return bad[0] == 0.0;
}

__device__ __forceinline__ bool r6_check(R6Smem &s, R6Var (&V)[2], R6Row (&R)[2], R6Dy (&Dl)[2], const QPSettingsDev &st,
                                         const double (&o)[8], bool approx, int &status) {
  const double pri = o[0], dua = o[3] / s.c;
  double ea = st.eps_abs, er = st.eps_rel, epi = st.eps_prim_inf, edi = st.eps_dual_inf;
  if (pri > QP_OSQP_INFTY || dua > QP_OSQP_INFTY) { status = -7; return true; }
  if (approx) { ea *= 10; er *= 10; epi *= 10; edi *= 10; }
  bool prim_ok = false, prim_inf = false, dual_ok = false, dual_inf = false;
  if (pri < ea + er * fmax(o[1], o[2])) prim_ok = true;
  else prim_inf = r6_primal_infeasible(s, V, R, Dl, epi);
  if (dua < ea + er * fmax(fmax(o[4], o[5]), o[6]) / s.c) dual_ok = true;
  else dual_inf = r6_dual_infeasible(s, V, R, Dl, edi);
  if (prim_ok && dual_ok) { status = approx ? 2 : 1; return true; }
  if (prim_inf) { status = approx ? 3 : -3; return true; }
  if (dual_inf) { status = approx ? 4 : -4; return true; }
  return false;
}

__device__ __forceinline__ void r6_rebuild_w(R6Smem &s, R6Var (&V)[2], R6Row (&R)[2]) {
  const double rs = s.rho_s;
  R6_FOR_H {
    if (R[h].ok) s.w[R[h].r] = QP_RHO_EQ * rs * R[h].zr - R[h].yr;
    if (V[h].gok) s.w[R6_MD + V[h].j] = r6_rho(V[h].gl, V[h].gu, rs) * V[h].gz - V[h].gy;
  }
  __syncthreads();
}

// The items' indices, opaque to the compiler once per ADMM iteration: every address
// and row-structure decision derived from them is recomputed inside the loop instead
// of hoisted out of it as a live register (hoisted, they were most of the spills)
__device__ __forceinline__ void r6_launder(R6Var (&V)[2], R6Row (&R)[2]) {
#if R6_LAUNDER
  R6_FOR_H {
    asm volatile("" : "+v"(V[h].j), "+v"(V[h].k), "+v"(V[h].i));
    asm volatile("" : "+v"(R[h].r), "+v"(R[h].k), "+v"(R[h].i));
  }
#endif
}

// diagnostic phase cycles of workgroup 0 (GPMPC_R6_STAMPS=1 launches the <true> instance)
__device__ unsigned long long g_r6_stamps[12];

template <bool ST>
__global__ __launch_bounds__(R6_T) void k_r6_control(R6Args a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  unsigned long long tl = 0;
  auto mark = [&](int k) {
    if (ST && b == 0 && tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (k >= 0) g_r6_stamps[k] += t - tl;
      tl = t;
    }
  };
  mark(-1);
  double *rec = a.rec + (int64_t)b * GPMPC_REC_LEN;
  if (a.mode == 0 ? rec[0] != 0.0 : a.done[b] != 0) return;
  extern __shared__ double smem_raw[];
  R6Smem &s = *reinterpret_cast<R6Smem *>(smem_raw);
  const double dt = a.dt;
  const QPSettingsDev &st = a.st;
  const double *Xb = a.Xp + (int64_t)b * (R6_N + 1) * R6_NX;
  const double *Ub = a.U + (int64_t)b * R6_N * R6_NU;
  const double *gmb = a.gm + (int64_t)b * R6_N * 6;
  double *ysc = a.ysc + (int64_t)b * R6_M;
  const double *x0 = a.x + (int64_t)b * R6_NX;
  const double *prm = a.prm;
  // the target: GPMPC.solve's X_ref per stage (x_target tiled unless the caller
  // gave one, gp_mpc.py:442-453; read per variable below), or in a rollout step
  // the incremental target of monte_carlo.py:497-500 (x copied, v = 0, altitude
  // - 2 m, floor 0.5 m; optionally upright and at rest)
  auto xref_mc = [&](int i) -> double {
    if (i >= 4 && i < 7) return 0.0;
    if (i == 1) return fmax(0.5, x0[1] - 2.0);
    if (a.upright && i >= 7) return i == 7 ? 1.0 : 0.0;
    return x0[i];
  };
  // ---- the linearisation (-[A_d | B_d] per stage, k_r6_predict) into the staging area
  {
    const double *lin = a.lin + (int64_t)b * R6_N * R6_NX * R6_SZ;
    for (int e = tid; e < R6_N * R6_NX * R6_SZ; e += R6_T) s.G[e] = lin[e];
    if (tid < R6_SZ) s.zero[tid] = 0.0;
  }
  __syncthreads();
  // item tid + 512 h: variable j < 524 (h = 0: all of them below 512), else
  // equality row r = item - 524; general row g = tid < 146 rides on slot 0
  R6Var V[2];
  R6Row R[2] = {R6Row(V[0]), R6Row(V[1])};
  R6_FOR_H {
    const int idx = tid + h * R6_T;
    R6Var &W = V[h];
    R6Row &Q = R[h];
    W.j = idx; W.ok = idx < R6_NV;
    W.k = idx / R6_SZ; W.i = idx - W.k * R6_SZ;
    W.gok = h == 0 && tid < R6_MGEN;
    // at N = 30 slot 0 holds only variables (524 > 512), so its row code compiles away;
    // at N = 20 equality rows start in slot 0 (idx 354..511)
    Q.r = idx - R6_NV; Q.ok = (R6_NV >= R6_T ? h == 1 : true) && idx >= R6_NV && Q.r < R6_MD;
    Q.k = Q.r >= R6_NX ? (Q.r - R6_NX) / R6_NX : 0;
    Q.i = Q.r >= R6_NX ? (Q.r - R6_NX) - Q.k * R6_NX : Q.r;
    if (W.ok) {
      const int k = W.k, i = W.i;
      double xw, wq;
      if (i < R6_NX) {
        xw = Xb[k * R6_NX + i];
        wq = prm[(k == R6_N ? R6_PP : R6_PQ) + i];
        const double xrv = a.mode ? a.xt[((int64_t)b * (R6_N + 1) + k) * R6_NX + i] : xref_mc(i);
        W.P = wq; W.q = wq * (xw - xrv);
        const double tr = sqrt(prm[R6_PTRX]);
        W.lb = -tr; W.ub = tr;
      } else {
        const double ub = Ub[k * R6_NU + i - R6_NX];
        const double rr = prm[R6_PR + i - R6_NX], tr = sqrt(prm[R6_PTRU]), tmax = prm[R6_PTMAX];
        const double urv = a.mode ? a.ut[((int64_t)b * R6_N + k) * R6_NU + i - R6_NX] : 0.0;  // U_ref
        W.P = rr; W.q = rr * (ub - urv);
        W.lb = fmax(-tr, -tmax - ub);
        W.ub = fmin(tr, tmax - ub);
      }
      W.Ab = 1.0;
      W.x = 0.0;  // warm start dz = 0
      W.yb = ysc[R6_MD + W.j];
      if (k < R6_N)
#pragma unroll
        for (int e = 0; e < R6_NX; ++e) W.colA[e] = s.G[(k * R6_NX + e) * R6_SZ + i];
      else
#pragma unroll
        for (int e = 0; e < R6_NX; ++e) W.colA[e] = 0.0;
    }
    if (W.gok) {
      const int g = W.j;
      if (g < R6_MT) {
        const double *u = Ub + g * R6_NU;
        const double tm = sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
        W.gA[0] = u[0] / tm; W.gA[1] = u[1] / tm; W.gA[2] = u[2] / tm;
        W.gl = prm[R6_PTMIN] - tm; W.gu = INFINITY; W.gn = 3;
      } else {
        const int gg = g - R6_MT, k = 1 + gg / 4, c = gg % 4;
        const double tg = prm[R6_PTAN];  // np.tan(gamma_gs)
        const double rx = Xb[k * R6_NX + 1], rc = Xb[k * R6_NX + (c < 2 ? 2 : 3)];
        const double sg = (c & 1) ? 1.0 : -1.0;
        W.gA[0] = tg; W.gA[1] = sg; W.gA[2] = 0.0;
        W.gl = -(tg * rx + sg * rc); W.gu = INFINITY; W.gn = 2;
      }
      W.gy = ysc[R6_MD + R6_NV + g];
    }
    if (Q.ok) {
      if (Q.r < R6_NX) {
        Q.A[0] = 1.0;
#pragma unroll
        for (int e = 1; e <= R6_SZ; ++e) Q.A[e] = 0.0;
        Q.ur = x0[Q.r] - Xb[Q.r];  // dX_0 = x0 - X_nom[0] (gp_mpc.py:402)
      } else {
#pragma unroll
        for (int e = 0; e < R6_SZ; ++e) Q.A[e] = s.G[(Q.k * R6_NX + Q.i) * R6_SZ + e];
        Q.A[R6_SZ] = 1.0;
        const int i = Q.i;
        Q.ur = (i >= 4 && i < 7) ? gmb[Q.k * 6 + i - 4] * dt : ((i >= 11) ? gmb[Q.k * 6 + 3 + i - 11] * dt : 0.0);
      }
      Q.yr = ysc[Q.r];
    }
    // ---- OSQP solve (qp_device.h order): clip bounds, Ruiz scaling, rho, factor
    if (W.ok) { W.lb = fmax(W.lb, -QP_OSQP_INFTY); W.ub = fmin(W.ub, QP_OSQP_INFTY); }
    if (W.gok) { W.gl = fmax(W.gl, -QP_OSQP_INFTY); W.gu = fmin(W.gu, QP_OSQP_INFTY); }
    if (Q.ok) Q.ur = fmin(fmax(Q.ur, -QP_OSQP_INFTY), QP_OSQP_INFTY);
  }
  mark(0);
  for (int r = tid; r < R6_M; r += R6_T) s.E[r] = 1.0;
  R6_FOR_H {
    if (R[h].ok) s.dpl[R[h].r] = R[h].r < R6_NX ? R[h].A[0] : R[h].A[R6_SZ];
    if (V[h].gok)
#pragma unroll
      for (int e = 0; e < 3; ++e) s.gen[V[h].j * 3 + e] = V[h].gA[e];
    if (V[h].ok) V[h].D = 1.0;
  }
  if (tid == 0) { s.c = 1.0; s.rho_s = fmin(fmax(a.rho[b], QP_RHO_MIN), QP_RHO_MAX); }
  __syncthreads();
  for (int it = 0; it < st.scaling; ++it) {
    // column factors -> dsc, row factors -> w (equality: [0, MD), general: MD + g)
    double eb[2] = {1.0, 1.0};
    R6_FOR_H {
      R6Var &W = V[h];
      R6Row &Q = R[h];
      if (W.ok) {
        double v = fabs(W.P);
        if (W.i < R6_NX) v = fmax(v, fabs(s.dpl[r6_eqid_row(W.k, W.i)]));
        if (W.k < R6_N)
#pragma unroll
          for (int e = 0; e < R6_NX; ++e) v = fmax(v, fabs(W.colA[e]));
        v = fmax(v, fabs(W.Ab));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int g, sl;
          if (r6_gen_slot(W.k, W.i, e, g, sl)) v = fmax(v, fabs(s.gen[g * 3 + sl]));
        }
        s.dsc[W.j] = 1.0 / sqrt(qp_limit(v));
        eb[h] = 1.0 / sqrt(qp_limit(fmax(0.0, fabs(W.Ab))));
      }
      if (Q.ok) {
        double v = 0.0;
        const int ne = Q.r < R6_NX ? 1 : R6_SZ + 1;
#pragma unroll
        for (int e = 0; e < R6_SZ + 1; ++e)
          if (e < ne) v = fmax(v, fabs(Q.A[e]));
        s.w[Q.r] = 1.0 / sqrt(qp_limit(v));
      }
      if (W.gok) {
        double v = 0.0;
#pragma unroll
        for (int e = 0; e < 3; ++e)
          if (e < W.gn) v = fmax(v, fabs(W.gA[e]));
        s.w[R6_MD + W.j] = 1.0 / sqrt(qp_limit(v));
      }
    }
    __syncthreads();
    double v[1] = {0.0}, mx[1] = {0.0};
    R6_FOR_H {
      R6Var &W = V[h];
      R6Row &Q = R[h];
      if (Q.ok) {
        const double e = s.w[Q.r];
        if (Q.r < R6_NX) {
          Q.A[0] = e * Q.A[0] * s.dsc[Q.r];
          s.dpl[Q.r] = Q.A[0];
        } else {
          const int o = Q.k * R6_SZ;
#pragma unroll
          for (int c = 0; c < R6_SZ; ++c) Q.A[c] = e * Q.A[c] * s.dsc[o + c];
          Q.A[R6_SZ] = e * Q.A[R6_SZ] * s.dsc[(Q.k + 1) * R6_SZ + Q.i];
          s.dpl[Q.r] = Q.A[R6_SZ];
        }
        s.E[Q.r] *= e;
      }
      if (W.gok) {
        const double e = s.w[R6_MD + W.j];
        int col[3];
        r6_gen_cols(W.j, col);
#pragma unroll
        for (int c = 0; c < 3; ++c)
          if (c < W.gn) {
            W.gA[c] = e * W.gA[c] * s.dsc[col[c]];
            s.gen[W.j * 3 + c] = W.gA[c];
          }
        s.E[R6_MD + R6_NV + W.j] *= e;
      }
      if (W.ok) {
        const double d = s.dsc[W.j];
        if (W.k < R6_N)
#pragma unroll
          for (int e = 0; e < R6_NX; ++e) W.colA[e] = s.w[R6_NX + R6_NX * W.k + e] * W.colA[e] * d;
        W.Ab = eb[h] * W.Ab * d;
        s.E[R6_MD + W.j] *= eb[h];
        W.P = d * W.P * d;
        W.q = d * W.q;
        W.D *= d;
        v[0] += fabs(W.P);
        mx[0] = fmax(mx[0], fabs(W.q));
      }
    }
    r6_sum<1>(v, s.red);
    r6_max<1>(mx, s.red);
    double ct = v[0] / R6_NV;
    const double nq = qp_limit(mx[0]);
    ct = qp_limit(fmax(ct, nq));
    ct = 1.0 / ct;
    R6_FOR_H {
      if (V[h].ok) { V[h].P *= ct; V[h].q *= ct; }
    }
    if (tid == 0) s.c *= ct;
    __syncthreads();
  }
  R6_FOR_H {
    R6Var &W = V[h];
    if (W.ok) { const double e = s.E[R6_MD + W.j]; W.lb = e * W.lb; W.ub = e * W.ub; }
    if (W.gok) { const double e = s.E[R6_MD + R6_NV + W.j]; W.gl = e * W.gl; W.gu = e * W.gu; }
    if (R[h].ok) R[h].ur = s.E[R[h].r] * R[h].ur;
  }
  mark(1);
  int f = r6_factor(s, V, R, st.sigma, mark);
  mark(2);
  QPResult res{-10, 0, 0.0, 0};
  if (f) res.factor_fail = f;
  if (!f) {
    // warm start x = 0 / D = 0, z = A x = 0; y persisted (osqp_rti.py:521-524)
    R6_FOR_H {
      V[h].x = 0.0; V[h].zb = 0.0; R[h].zr = 0.0; V[h].gz = 0.0;
      if (V[h].ok) V[h].zb = 0.0 + V[h].Ab * V[h].x;
    }
    r6_rebuild_w(s, V, R);
    const double sig = st.sigma, al = st.alpha;
    double o[8], re_[4];
    for (int it = 1; it <= st.max_iter; ++it) {
      r6_launder(V, R);
      {
        const double rs = s.rho_s;
        R6_FOR_H {
          // the bound row's rho z - y (formed here rather than kept per item)
          const double ztb = r6_rho(V[h].lb, V[h].ub, rs) * V[h].zb - V[h].yb;
          if (V[h].ok) s.rhs[V[h].j] = sig * V[h].x - V[h].q + r6_col_dot(s, V[h], s.w, ztb, s.w + R6_MD);
        }
      }
      __syncthreads();
      mark(3);
      r6_solve(s, mark);
#if R6_LAUNDER > 1
      r6_launder(V, R);
#endif
      const double rs = s.rho_s;
      R6Dy Dl[2];
      R6_FOR_H {
        R6Var &W = V[h];
        R6Row &Q = R[h];
        if (W.ok) {
          const double xt = s.xs[W.j], xo = W.x;
          const double xn = al * xt + (1.0 - al) * xo;
          Dl[h].dx = xn - xo;
          W.x = xn;
          const double ztl = 0.0 + W.Ab * xt;
          const double rho = r6_rho(W.lb, W.ub, rs), zo = W.zb, yo = W.yb;
          const double zr = al * ztl + (1.0 - al) * zo;
          double zn = zr + yo / rho;
          zn = fmin(fmax(zn, W.lb), W.ub);
          const double d = rho * (zr - zn);
          Dl[h].dyb = d; W.yb = yo + d; W.zb = zn;
        }
        if (W.gok) {
          const double ztl = r6_gen_dot(W, s.xs);
          const double rho = r6_rho(W.gl, W.gu, rs), zo = W.gz, yo = W.gy;
          const double zr = al * ztl + (1.0 - al) * zo;
          double zn = zr + yo / rho;
          zn = fmin(fmax(zn, W.gl), W.gu);
          const double d = rho * (zr - zn);
          Dl[h].gdy = d; W.gy = yo + d; W.gz = zn;
        }
        if (Q.ok) {
          const double ztl = r6_row_dot(Q, s.xs);
          const double rho = QP_RHO_EQ * rs, zo = Q.zr, yo = Q.yr;
          const double zr = al * ztl + (1.0 - al) * zo;
          double zn = zr + yo / rho;
          zn = fmin(fmax(zn, Q.ur), Q.ur);
          const double d = rho * (zr - zn);
          Dl[h].dyb = d; Q.yr = yo + d; Q.zr = zn;
        }
      }
      __syncthreads();  // every read of s.w / s.xs of this iteration is done
      R6_FOR_H {
        if (R[h].ok) s.w[R[h].r] = QP_RHO_EQ * rs * R[h].zr - R[h].yr;
        if (V[h].gok) s.w[R6_MD + V[h].j] = r6_rho(V[h].gl, V[h].gu, rs) * V[h].gz - V[h].gy;
      }
      __syncthreads();
      mark(7);
      const bool can_check = st.check_termination && (it % st.check_termination == 0);
      const bool adapt = st.adaptive_rho && st.adaptive_rho_interval && (it % st.adaptive_rho_interval == 0);
      const bool last = it == st.max_iter;
      if (can_check || adapt || last) {
        res.iter = it;
        r6_update_info(s, V, R, o, re_);
      }
      if (can_check && r6_check(s, V, R, Dl, st, o, false, res.status)) break;
      if (adapt) {
        const double pr = re_[0] / (re_[1] + 1e-10);
        const double du = re_[2] / (re_[3] + 1e-10);
        double est = s.rho_s * sqrt(pr / (du + 1e-10));
        est = fmin(fmax(est, QP_RHO_MIN), QP_RHO_MAX);
        if (est > s.rho_s * st.adaptive_rho_tolerance || est < s.rho_s / st.adaptive_rho_tolerance) {
          __syncthreads();
          if (tid == 0) s.rho_s = est;
          __syncthreads();
          if (it < st.max_iter) {
            f = r6_factor(s, V, R, st.sigma, mark);
            if (f) { res.factor_fail = f; break; }
          }
        }
      }
      if (can_check || adapt) r6_rebuild_w(s, V, R);
      mark(8);
      if (last) {
        // max_iter reached (inside the iteration, where its dx / dy live): the final
        // check unless one just ran, then the approximate one (qp_device.h).  max_iter
        // >= 1 always: r6_create refuses less, as OSQP's settings check does
        for (int ap = can_check ? 1 : 0; ap < 2; ++ap) {
          if (r6_check(s, V, R, Dl, st, o, ap == 1, res.status)) break;
          if (ap == 1) res.status = -2;
        }
      }
    }
  }
  const bool has = !res.factor_fail && (res.status == 1 || res.status == 2 || res.status == -2);
  // ---- solution: the unscaled deviations onto the plan, kept unshifted (gp_mpc.py:358-359)
  R6_FOR_H {
    if (has && V[h].ok) s.xs[V[h].j] = V[h].D * V[h].x;
  }
  __syncthreads();
  double *Xo = a.Xo + (int64_t)b * (R6_N + 1) * R6_NX;
  double *Uw = a.U + (int64_t)b * R6_N * R6_NU;
  double chg[2] = {0.0, 0.0};  // max |X_new - X_pred|, max |U_new - U_pred| (gp_mpc.py:337-338)
  if (has) {
    for (int e = tid; e < (R6_N + 1) * R6_NX; e += R6_T) {
      const int k = e / R6_NX, i = e - k * R6_NX;
      const double xo = Xb[e] + s.xs[k * R6_SZ + i];
      Xo[e] = xo;
      const double d = fabs(xo - Xb[e]);
      if (!(d <= chg[0])) chg[0] = d != d ? INFINITY : d;  // a NaN never converges
    }
    double un = 0.0;
    if (tid < R6_N * R6_NU) {
      const int k = tid / R6_NU, i = tid - k * R6_NU;
      un = Ub[tid] + s.xs[k * R6_SZ + R6_NX + i];
      const double d = fabs(un - Ub[tid]);
      chg[1] = d != d ? INFINITY : d;
    }
    __syncthreads();  // every thread read U before it is overwritten
    if (tid < R6_N * R6_NU) Uw[tid] = un;
    R6_FOR_H {
      if (R[h].ok) ysc[R[h].r] = R[h].yr;
      if (V[h].ok) ysc[R6_MD + V[h].j] = V[h].yb;
      if (V[h].gok) ysc[R6_MD + R6_NV + V[h].j] = V[h].gy;
    }
    __syncthreads();
  } else if (a.mode) {
    // _solve_qp's fallback (gp_mpc.py:478-482): the nominal trajectory
    for (int e = tid; e < (R6_N + 1) * R6_NX; e += R6_T) Xo[e] = Xb[e];
  }
  if (a.mode) r6_max<2>(chg, s.red);  // a.mode is uniform over the launch
  if (tid == 0 && a.mode) {  // GPMPC.solve pass bookkeeping
    a.passes[b] += 1;
    a.qit[b] += res.iter;
    a.qst[b] = res.factor_fail ? -100 : res.status;
    a.done[b] = (chg[0] < a.sqp_tol && chg[1] < a.sqp_tol) ? 1 : 0;  // a failed QP: X_new = X_pred
    rec[11] += res.iter;
    rec[12] += (res.status == 1 && !res.factor_fail) ? 1.0 : 0.0;
    rec[14] = res.factor_fail ? -100 : res.status;
    if (has) { a.rho[b] = s.rho_s; rec[15] = s.rho_s; }
  } else if (tid == 0) {
    if (!has) {  // MPCSolution without a solution -> DIVERGENCE
      const double *x = a.x + (int64_t)b * R6_NX;
      rec[0] = 6;
      rec[14] = res.factor_fail ? -100 : res.status;
      rec[2] = rec[13] - x[0];
      for (int i = 0; i < 7; ++i) rec[4 + i] = x[i];
    } else {
      a.rho[b] = s.rho_s;
      rec[11] += res.iter;
      rec[12] += (res.status == 1) ? 1.0 : 0.0;
      rec[14] = res.status;
      rec[15] = s.rho_s;
      a.pending[b] = 1;
    }
  }
  mark(9);
}

// 3. the truth plant step with the plan's first control: RK4 + the drag
// dispersion at the pre-step state (dispersion.py:349-360) + the -0.05 w rate
// damping the config-5 GP is trained on (data.synthetic_6dof_training_data)
__global__ __launch_bounds__(64) void k_r6_plant(R6Args a, int B) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= B || !a.pending[b]) return;
  a.pending[b] = 0;
  double *rec = a.rec + (int64_t)b * GPMPC_REC_LEN;
  double *x = a.x + (int64_t)b * R6_NX;
  const double dt = a.dt;
  double xc[R6_NX], xn[R6_NX];
  for (int i = 0; i < R6_NX; ++i) xc[i] = x[i];
  const double *u0 = a.U + (int64_t)b * R6_N * R6_NU;
  r6_step(a.rk, xc, u0, dt, xn);
  const double vx = xc[4], vy = xc[5], vz = xc[6];
  const double sp = sqrt((vx * vx + vy * vy) + vz * vz);
  if (sp > 1.0) {
    const double ac = (0.5 * 0.02 * sp * sp) / xc[0];
    xn[4] += -ac * (vx / sp) * dt; xn[5] += -ac * (vy / sp) * dt; xn[6] += -ac * (vz / sp) * dt;
  }
  for (int i = 11; i < 14; ++i) xn[i] += -0.05 * xc[i] * dt;
  for (int i = 0; i < R6_NX; ++i) x[i] = xn[i];
  rec[1] += 1.0;
  rec[2] = rec[13] - xn[0];
  rec[3] = rec[1] * dt;
  for (int i = 0; i < 7; ++i) rec[4 + i] = xn[i];
}

__global__ void k_r6_reset(int first, int count, const double *__restrict__ x0, double *x, double *U,
                           double *ysc, double *rho, double rho0, double *rec, double g0) {
  const int i = blockIdx.x;
  if (i >= count) return;
  const int b = first + i;
  const double *xi = x0 + (int64_t)i * R6_NX;
  for (int e = threadIdx.x; e < R6_N * R6_NU; e += blockDim.x)  // hover guess as written (gp_mpc.py:271-275)
    U[(int64_t)b * R6_N * R6_NU + e] = (e % R6_NU == 2) ? xi[0] * g0 : 0.0;
  for (int r = threadIdx.x; r < R6_M; r += blockDim.x) ysc[(int64_t)b * R6_M + r] = 0.0;
  if (threadIdx.x < GPMPC_REC_LEN) rec[(int64_t)b * GPMPC_REC_LEN + threadIdx.x] = 0.0;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int c = 0; c < R6_NX; ++c) x[(int64_t)b * R6_NX + c] = xi[c];
    for (int c = 0; c < 7; ++c) rec[(int64_t)b * GPMPC_REC_LEN + 4 + c] = xi[c];
    rec[(int64_t)b * GPMPC_REC_LEN + 13] = xi[0];
    rho[b] = rho0;
  }
}

// GPMPC.solve: x0 / x_target already in x / xt; cold = hover guess + fresh ADMM state
__global__ void k_r6_solve_begin(R6Args a, int cold, double rho0) {
  const int b = blockIdx.x;
  const double m0 = a.x[(int64_t)b * R6_NX];
  if (cold == 1) {
    // gp_mpc.py:271-275 as intended: [0, 0, m0 g0] at every stage (as written it reads
    // X_pred[k, 0] before the simulation has filled it, i.e. zero thrust for k >= 1,
    // whose thrust-magnitude rows have no linearisation)
    for (int e = threadIdx.x; e < R6_N * R6_NU; e += blockDim.x)
      a.U[(int64_t)b * R6_N * R6_NU + e] = (e % R6_NU == 2) ? m0 * a.rk.g0 : 0.0;
  }
  if (cold)
    for (int r = threadIdx.x; r < R6_M; r += blockDim.x) a.ysc[(int64_t)b * R6_M + r] = 0.0;
  if (threadIdx.x == 0) {
    if (cold) a.rho[b] = rho0;
    a.done[b] = 0; a.passes[b] = 0; a.qit[b] = 0; a.qst[b] = -10;
    double *rec = a.rec + (int64_t)b * GPMPC_REC_LEN;
    rec[11] = 0.0; rec[12] = 0.0;
  }
}

// ---------------------------------------------------------------------------
// launchers of this horizon's kernels (the C-ABI in fleet6.hip reaches them through impl)
static hipError_t r6_init() {
  static const hipError_t e = [] {
    (void)hipFuncSetAttribute((const void *)k_r6_control<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(R6Smem));
    return hipFuncSetAttribute((const void *)k_r6_control<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(R6Smem));
  }();
  return e;
}
static void r6_launch_predict(hipStream_t s, int B, const R6Args &a0, bool st) {
  static const int cap = [] {
    const char *v = getenv("GPMPC_R6_PCACHE");
    return v ? atoi(v) : R6_PCACHE_ROWS;
  }();
  static const bool attr = [] {
    const int mx = (int)(sizeof(double) * (13 + 12) * R6_PCACHE_ROWS);  // the largest dynamic size used
    return hipFuncSetAttribute((const void *)k_r6_predict<false>, hipFuncAttributeMaxDynamicSharedMemorySize, mx) ==
               hipSuccess &&
           hipFuncSetAttribute((const void *)k_r6_predict<true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx) ==
               hipSuccess;
  }();
  R6Args a = a0;
  const int c = (attr && a.use_gp) ? max(0, min(cap, R6_PCACHE_ROWS)) : 0;
  a.mcv = min(a.Mv, c);
  a.mcw = min(a.Mw, c);
  a.nb = B;
  if (!a.use_gp) a.parts = 1;  // (no kernel rows to split)
  const size_t lds = sizeof(double) * (size_t)(a.mcv * 13 + a.mcw * 12);
  if (a.parts > 1) {
    // every granule zeroed before the launch (the timeout word behind them is sticky: zeroed
    // at creation, read by gpmpc_rollout6_read / _solve)
    (void)hipMemsetAsync(a.gran, 0, sizeof(unsigned long long) * (size_t)B * 2 * R6_GRAN, s);
    if (st) hipLaunchKernelGGL(k_r6_predict<true>, dim3((B + 7) / 8 * 8 * a.parts), dim3(R6_PT), lds, s, a);
    else hipLaunchKernelGGL(k_r6_predict<false>, dim3((B + 7) / 8 * 8 * a.parts), dim3(R6_PT), lds, s, a);
  } else if (st) {
    hipLaunchKernelGGL(k_r6_predict<true>, dim3(B), dim3(R6_PT), lds, s, a);
  } else {
    hipLaunchKernelGGL(k_r6_predict<false>, dim3(B), dim3(R6_PT), lds, s, a);
  }
}
static void r6_launch_control(hipStream_t s, int B, const R6Args &a, bool st) {
  if (st) hipLaunchKernelGGL(k_r6_control<true>, dim3(B), dim3(R6_T), sizeof(R6Smem), s, a);
  else hipLaunchKernelGGL(k_r6_control<false>, dim3(B), dim3(R6_T), sizeof(R6Smem), s, a);
}
static void r6_launch_plant(hipStream_t s, int B, const R6Args &a) {
  hipLaunchKernelGGL(k_r6_plant, dim3((B + 63) / 64), dim3(64), 0, s, a, B);
}
static void r6_launch_reset(hipStream_t s, int first, int count, const double *x0, const R6Args &a, double rho0) {
  hipLaunchKernelGGL(k_r6_reset, dim3(count), dim3(256), 0, s, first, count, x0, a.x, a.U, a.ysc, a.rho, rho0,
                     a.rec, a.rk.g0);
}
static void r6_launch_solve_begin(hipStream_t s, int B, const R6Args &a, int cold, double rho0) {
  hipLaunchKernelGGL(k_r6_solve_begin, dim3(B), dim3(256), 0, s, a, cold, rho0);
}
static void r6_print_stamps() {  // diagnostic: phase cycles of rollout 0, summed over the steps
  static const char *nm[12] = {"setup", "scaling", "factor0", "rhs", "kkt_forward", "kkt_diagonal",
                               "kkt_backward", "update", "checks_adapt", "tail", "factor_gj", "factor_prod"};
  unsigned long long h[12] = {0};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_r6_stamps), sizeof(h)) == hipSuccess) {
    unsigned long long tot = 0;
    for (int k = 0; k < 12; ++k) tot += h[k];
    for (int k = 0; k < 12; ++k)
      fprintf(stderr, "r6 stamps N=%d %-14s %12llu cycles %5.1f%%\n", R6_N, nm[k], h[k],
              tot ? 100.0 * h[k] / tot : 0.0);
  }
  unsigned long long hp[8] = {0};
  if (hipMemcpyFromSymbol(hp, HIP_SYMBOL(g_r6p_stamps), sizeof(hp)) == hipSuccess)
    fprintf(stderr, "r6 predict stamps N=%d: start %llu, kernel rows + rk4 %llu means + next features %llu "
            "(rk4 alone %llu), end (states, Jacobians) %llu; part-0 wave-0 rows %llu, poll %llu\n", R6_N, hp[3], hp[1],
            hp[0], hp[2], hp[4], hp[5], hp[6]);
}
// (a host function, not a namespace-scope object: the device pass would emit the object
// with references to these host launchers)
const R6Impl *impl() {
  static const R6Impl i = {R6_N, R6_M, sizeof(R6Smem), r6_init, r6_launch_predict, r6_launch_control,
                           r6_launch_plant, r6_launch_reset, r6_launch_solve_begin, r6_print_stamps};
  return &i;
}

#undef R6_NBLK
#undef R6_NV
#undef R6_MD
#undef R6_MT
#undef R6_MG
#undef R6_MGEN
#undef R6_M
#undef R6_MID
#undef R6_BOTS
