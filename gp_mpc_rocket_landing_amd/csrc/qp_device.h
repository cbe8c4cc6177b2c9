// qp_device.h -- one OSQP-0.6-style ADMM solve per workgroup, everything in LDS.
//
// Algorithm (oracle/admm_oracle.py + oracle/admm_ref.c restate it; OSQP itself
// is absent): Ruiz scaling (scaling.c), rho vector by constraint
// type, then per iteration
//     x~ = (P + sigma I + A' R A)^-1 (sigma x - q + A'(R z - y)),  z~ = A x~
//     x  = a x~ + (1-a) x ;  z = Pi(a z~ + (1-a) z + y/R) ;  y += R(a z~ + (1-a) z - z)
// with the termination check / adaptive rho every 25 iterations.  The reduced
// KKT matrix of an MPC QP is banded (half-bandwidth w = 2 nx + nu - 1 = 16 for
// the 3-DoF problem); it is factored by a right-looking banded Cholesky and
// solved by column-oriented substitution in ONE wave, the right-hand side held
// in a 64-lane modular register window: row i lives in lane i mod 64, so each
// step is readlane(pivot) -> one FMA on the w lanes below -> no shuffles.
//
// LDS layout (doubles) for the caps NMAX/MMAX/NNZMAX/W: ~72 KB at the 3-DoF
// caps -> two landings per CU.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#define QP_OSQP_INFTY 1e30
#define QP_MIN_SCALING 1e-4
#define QP_MAX_SCALING 1e4
#define QP_RHO_MIN 1e-6
#define QP_RHO_MAX 1e6
#define QP_RHO_TOL 1e-4
#define QP_RHO_EQ 1e3
#define QP_DIV_TOL 1e-30
#define QP_RMAX 8   // max entries per row of A (register-hoisted pattern)
#define QP_CMAX 12  // max entries per column of A

struct QPSettingsDev {
  double rho, sigma, alpha, eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
  int max_iter, check_termination, adaptive_rho, adaptive_rho_interval;
  double adaptive_rho_tolerance;
  int scaling, warm_start;
};

// shared sparsity pattern (device memory), prepared on the host once per batch
struct QPPattern {
  int n, m, nnz, w;
  const int *rowptr;   // m+1
  const int *colidx;   // nnz
  const int *colptr;   // n+1   (CSC)
  const int *csc2csr;  // nnz   CSC entry -> CSR value index
  const int *cscrow;   // nnz   CSC entry -> row
  const int *bandptr;  // n*(w+1)+1  band entry (j,t) -> term range
  const int *terms;    // 3*nterms: (row, a, b) value pairs with rho_row*A[a]*A[b]
};

template <int NMAX, int MMAX, int NNZMAX, int W>
struct QPSmem {
  static constexpr int BAND_FRONT = (W + 1) * (W + 2);
  __device__ double *band() { return band_store + BAND_FRONT; }
  double A[NNZMAX];
  double P[NMAX], q[NMAX], D[NMAX], x[NMAX], rhs[NMAX], dx[NMAX], aux[NMAX], tmpn[NMAX];
  double E[MMAX], l[MMAX], u[MMAX], rho[MMAX], y[MMAX], z[MMAX], zt[MMAX], dy[MMAX], tmpm[MMAX];
  // column band, stride W+2: slot 0 holds 1/D_j after factoring, slots 1..W
  // the multipliers, slot W+1 is always zero; W+1 zero columns in front so
  // clamped backward-sweep addresses land on a zero slot
  double band_store[(W + 1) * (W + 2) + NMAX * (W + 2) + 4 * (W + 2)];
  double red[4][8];
  double c, rho_s;
  int flag;
};

// ---------------------------------------------------------------------------
__device__ __forceinline__ double readlane_d(double v, int l) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_readlane(lo, l);
  hi = __builtin_amdgcn_readlane(hi, l);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double qp_limit(double v) {
  v = v < QP_MIN_SCALING ? 1.0 : v;
  return v > QP_MAX_SCALING ? QP_MAX_SCALING : v;
}

// block-wide max of K values (non-negative); every thread gets the result
template <int K>
__device__ void block_max(double (&v)[K], double (*red)[8]) {
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
  for (int k = 0; k < K; ++k) v[k] = fmax(fmax(red[0][k], red[1][k]), fmax(red[2][k], red[3][k]));
  __syncthreads();
}

template <int K>
__device__ void block_sum(double (&v)[K], double (*red)[8]) {
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
  for (int k = 0; k < K; ++k) v[k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
  __syncthreads();
}

// out[r] = (A x)[r]
template <class S>
__device__ void qp_spmv(const QPPattern &pt, S &s, const double *x, double *out) {
  for (int r = threadIdx.x; r < pt.m; r += blockDim.x) {
    double acc = 0.0;
    for (int k = pt.rowptr[r]; k < pt.rowptr[r + 1]; ++k) acc += s.A[k] * x[pt.colidx[k]];
    out[r] = acc;
  }
}

// out[j] = (A' y)[j]
template <class S>
__device__ void qp_spmv_t(const QPPattern &pt, S &s, const double *y, double *out) {
  for (int j = threadIdx.x; j < pt.n; j += blockDim.x) {
    double acc = 0.0;
    for (int k = pt.colptr[j]; k < pt.colptr[j + 1]; ++k) acc += s.A[pt.csc2csr[k]] * y[pt.cscrow[k]];
    out[j] = acc;
  }
}

// scaling.c scale_data (Ruiz equilibration + cost normalisation), then l,u <- E l, E u
template <class S>
__device__ void qp_scale(const QPPattern &pt, S &s, int iters) {
  const int n = pt.n, m = pt.m, tid = threadIdx.x, nt = blockDim.x;
  for (int j = tid; j < n; j += nt) s.D[j] = 1.0;
  for (int r = tid; r < m; r += nt) s.E[r] = 1.0;
  if (tid == 0) s.c = 1.0;
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    // column norms of [P; A] -> aux, row norms of A -> dy (scratch)
    for (int j = tid; j < n; j += nt) {
      double v = fabs(s.P[j]);
      for (int k = pt.colptr[j]; k < pt.colptr[j + 1]; ++k) v = fmax(v, fabs(s.A[pt.csc2csr[k]]));
      s.aux[j] = 1.0 / sqrt(qp_limit(v));
    }
    for (int r = tid; r < m; r += nt) {
      double v = 0.0;
      for (int k = pt.rowptr[r]; k < pt.rowptr[r + 1]; ++k) v = fmax(v, fabs(s.A[k]));
      s.dy[r] = 1.0 / sqrt(qp_limit(v));
    }
    __syncthreads();
    for (int r = tid; r < m; r += nt) {
      const double e = s.dy[r];
      for (int k = pt.rowptr[r]; k < pt.rowptr[r + 1]; ++k) s.A[k] = e * s.A[k] * s.aux[pt.colidx[k]];
      s.E[r] *= e;
    }
    double v[1] = {0.0};
    for (int j = tid; j < n; j += nt) {
      const double d = s.aux[j];
      s.P[j] = d * s.P[j] * d;
      s.q[j] = d * s.q[j];
      s.D[j] *= d;
      v[0] += fabs(s.P[j]);
    }
    double mx[1] = {0.0};
    for (int j = tid; j < n; j += nt) mx[0] = fmax(mx[0], fabs(s.q[j]));
    block_sum<1>(v, s.red);
    block_max<1>(mx, s.red);
    double ct = v[0] / n;
    const double nq = qp_limit(mx[0]);
    ct = qp_limit(fmax(ct, nq));
    ct = 1.0 / ct;
    for (int j = tid; j < n; j += nt) {
      s.P[j] *= ct;
      s.q[j] *= ct;
    }
    if (tid == 0) s.c *= ct;
    __syncthreads();
  }
  for (int r = tid; r < m; r += nt) {
    s.l[r] = s.E[r] * s.l[r];
    s.u[r] = s.E[r] * s.u[r];
  }
  __syncthreads();
}

template <class S>
__device__ void qp_set_rho(const QPPattern &pt, S &s) {
  const double rs = s.rho_s;
  for (int r = threadIdx.x; r < pt.m; r += blockDim.x) {
    const double lr = s.l[r], ur = s.u[r];
    double v;
    if (lr < -QP_OSQP_INFTY * QP_MIN_SCALING && ur > QP_OSQP_INFTY * QP_MIN_SCALING) v = QP_RHO_MIN;
    else if (ur - lr < QP_RHO_TOL) v = QP_RHO_EQ * rs;
    else v = rs;
    s.rho[r] = v;
  }
  __syncthreads();
}

// assemble M = P + sigma I + A' R A into the column band and factor it as
// M = L^ D L^T (L^ unit lower).  band[j*(w+2)+t] = M[j+t][j] -> L^[j+t][j]
// (1 <= t <= w), band[j*(w+2)] = 1/D[j], band[j*(w+2)+w+1] = 0.  The sweeps
// then need no division and no lane masks on their critical path.  Returns 0 or a 1-based failing column.
template <class S>
__device__ int qp_factor(const QPPattern &pt, S &s, double sigma) {
  const int n = pt.n, w = pt.w, nb = w + 2, tid = threadIdx.x, nt = blockDim.x;
  double *band = s.band();
  for (int e = tid; e < S::BAND_FRONT; e += nt) s.band_store[e] = 0.0;
  for (int e = tid; e < (n + 4) * nb; e += nt) {
    const int j = e / nb, t = e - j * nb;
    double v = 0.0;
    if (j < n && t <= w) {
      const int eb = j * (w + 1) + t;  // pattern's (w+1)-stride band index
      v = (t == 0) ? s.P[j] + sigma : 0.0;
      for (int k = pt.bandptr[eb]; k < pt.bandptr[eb + 1]; ++k) {
        const int r = pt.terms[3 * k], a = pt.terms[3 * k + 1], b = pt.terms[3 * k + 2];
        v += s.rho[r] * s.A[a] * s.A[b];
      }
    }
    band[e] = v;
  }
  if (tid == 0) s.flag = 0;
  // (t, u) pair of this thread for the trailing update, 1 <= u <= t <= w
  const int nup = w * (w + 1) / 2;
  const bool upd = tid < nup;
  int t = 0, u = 0;
  if (upd) {
    t = (int)((sqrt(8.0 * tid + 1.0) + 1.0) * 0.5);
    while (t * (t - 1) / 2 > tid) --t;
    while ((t + 1) * t / 2 <= tid) ++t;
    u = tid - t * (t - 1) / 2 + 1;
  }
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    double *col = band + j * nb;
    const double dj = col[0];
    const double ct = upd ? col[t] : 0.0, cu = upd ? col[u] : 0.0;
    const double cw = (tid >= 1 && tid <= w) ? col[tid] : 0.0;
    __syncthreads();
    if (!(dj > 0.0)) {
      if (tid == 0) s.flag = j + 1;
      __syncthreads();
      return s.flag;
    }
    const double inv = 1.0 / dj;
    if (tid == 0) col[0] = inv;  // the pivot lane's own update is discarded
    if (tid >= 1 && tid <= w && j + tid < n) col[tid] = cw * inv;
    // M[j+t][j+u] -= l_t d_j l_u = (c_t / d_j) c_u   (stored at band[(j+u)*nb + (t-u)])
    if (upd && j + t < n) band[(j + u) * nb + (t - u)] -= (ct * inv) * cu;
    __syncthreads();
  }
  return 0;
}

// b <- M^-1 b with M = L^ D L^T in the column band (wave 0 only; others idle).
// Row i of the right-hand side lives in lane i mod 64 ("modular window").  At
// step j the lane at offset t = (row - j) mod 64 multiplies band slot min(t,
// w+1) of column j: slot 0 and slot w+1 hold zeros, so lanes outside the band
// need no mask.  The pivot value is read with readlane and captured with
// writelane; lanes that pivoted are refilled from the prefetched next window
// in bulk every 16 steps (a refilled row is first updated >= 48 steps after
// its lane pivots).  Band multipliers are prefetched 4 steps ahead.  A step is
// 2 readlane + 1 FMA + 2 writelane + the prefetch.
__device__ __forceinline__ void writelane_d(double &dst, double v, int l) {
  // v is wave-uniform (a readlane result), l an SGPR lane index
  int lo = __double2loint(dst), hi = __double2hiint(dst);
  // gfx9 constant bus: one SGPR operand per VOP3, so the lane index goes in m0
  asm("v_writelane_b32 %0, %2, m0\n\tv_writelane_b32 %1, %3, m0"
      : "+v"(lo), "+v"(hi)
      : "s"(__double2loint(v)), "s"(__double2hiint(v)), "{m0}"(l));
  dst = __hiloint2double(hi, lo);
}

template <class S>
__device__ void qp_band_solve(const QPPattern &pt, S &s, double *b) {
  if (threadIdx.x >= 64) return;
  const int n = pt.n, w = pt.w, nb = w + 2, wz = w + 1;
  const int lane = threadIdx.x;
  const double *band = s.band();
  // ---- forward: L^ z = b ; stores w = z / D in b.  L^[j+t][j] = band[j*nb + t]
  {
    double win = (lane < n) ? b[lane] : 0.0;
    for (int j0 = 0; j0 < n; j0 += 64) {
      const int rn = j0 + 64 + lane;
      const double nxt = (rn < n) ? b[rn] : 0.0;
      const int jend = min(n, j0 + 64);
      double mine = 0.0;
#define QP_LDF(jj) band[(jj) * nb + min((lane - (jj)) & 63, wz)]
#define QP_FSTEP(jj, lv)                          \
  {                                               \
    const int pl = (jj) & 63;                     \
    const double zj = readlane_d(win, pl);        \
    win = fma(-(lv), zj, win);                    \
    writelane_d(mine, zj, pl);                    \
  }
      for (int g = j0; g < jend; g += 16) {
        const int gend = min(jend, g + 16);
        if (gend - g == 16) {
          double l0 = QP_LDF(g), l1 = QP_LDF(g + 1), l2 = QP_LDF(g + 2), l3 = QP_LDF(g + 3);
#pragma unroll
          for (int q = 0; q < 16; q += 4) {
            const int j = g + q;
            const double n0 = QP_LDF(j + 4), n1 = QP_LDF(j + 5), n2 = QP_LDF(j + 6), n3 = QP_LDF(j + 7);
            QP_FSTEP(j, l0);
            QP_FSTEP(j + 1, l1);
            QP_FSTEP(j + 2, l2);
            QP_FSTEP(j + 3, l3);
            l0 = n0; l1 = n1; l2 = n2; l3 = n3;
          }
        } else {
          for (int j = g; j < gend; ++j) {
            const double l0 = QP_LDF(j);
            QP_FSTEP(j, l0);
          }
        }
        // lanes that pivoted in [g, gend) take their row of the next window
        win = ((unsigned)(lane - (g - j0)) < (unsigned)(gend - g)) ? nxt : win;
      }
#undef QP_FSTEP
#undef QP_LDF
      if (j0 + lane < jend) b[j0 + lane] = mine * band[(j0 + lane) * nb];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // ---- backward: L^T x = w.  lane's row r = i - t;  L^[i][r] = band[r*nb + t]
  //      with t clamped to w+1: band[i*nb - (nb-1)*min(t, w+1)]
  {
    // lanes past the (partial) top window start on their row of the block below,
    // as if they had already pivoted in the top window
    const int top = ((n - 1) >> 6) << 6;
    double win = (top + lane < n) ? b[top + lane] : ((top - 64 + lane >= 0) ? b[top - 64 + lane] : 0.0);
    for (int i0 = top; i0 >= 0; i0 -= 64) {
      const int rp = i0 - 64 + lane;
      const double nxt = (rp >= 0) ? b[rp] : 0.0;
      const int ihi = min(n, i0 + 64) - 1;
      double mine = 0.0;
#define QP_LDB(ii) band[(ii) * nb - (nb - 1) * min(((ii) - lane) & 63, wz)]
#define QP_BSTEP(ii, lv)                          \
  {                                               \
    const int pl = (ii) & 63;                     \
    const double xi = readlane_d(win, pl);        \
    win = fma(-(lv), xi, win);                    \
    writelane_d(mine, xi, pl);                    \
  }
      for (int g = ihi; g >= i0; g -= 16) {
        const int gend = max(i0 - 1, g - 16);  // exclusive
        if (g - gend == 16) {
          double l0 = QP_LDB(g), l1 = QP_LDB(g - 1), l2 = QP_LDB(g - 2), l3 = QP_LDB(g - 3);
#pragma unroll
          for (int q = 0; q < 16; q += 4) {
            const int i = g - q;
            const double n0 = QP_LDB(i - 4), n1 = QP_LDB(i - 5), n2 = QP_LDB(i - 6), n3 = QP_LDB(i - 7);
            QP_BSTEP(i, l0);
            QP_BSTEP(i - 1, l1);
            QP_BSTEP(i - 2, l2);
            QP_BSTEP(i - 3, l3);
            l0 = n0; l1 = n1; l2 = n2; l3 = n3;
          }
        } else {
          for (int i = g; i > gend; --i) {
            const double l0 = QP_LDB(i);
            QP_BSTEP(i, l0);
          }
        }
        // lanes that pivoted in (gend, g] take their row of the window below
        win = ((unsigned)(lane - (gend + 1 - i0)) < (unsigned)(g - gend)) ? nxt : win;
      }
#undef QP_BSTEP
#undef QP_LDB
      if (i0 + lane <= ihi) b[i0 + lane] = mine;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// residuals (auxil.c update_info): tmpm <- A x, aux <- P x, tmpn <- A' y.
// o: 0 pri (unscaled)  1 |z/E|  2 |Ax/E|  3 dua*c  4 |q/D|  5 |A'y/D|  6 |Px/D|
template <class S>
__device__ void qp_update_info(const QPPattern &pt, S &s, double (&o)[8]) {
  const int n = pt.n, m = pt.m, tid = threadIdx.x, nt = blockDim.x;
  qp_spmv(pt, s, s.x, s.tmpm);
  qp_spmv_t(pt, s, s.y, s.tmpn);
  for (int j = tid; j < n; j += nt) s.aux[j] = s.P[j] * s.x[j];
  __syncthreads();
  double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = tid; r < m; r += nt) {
    const double e = s.E[r];
    v[0] = fmax(v[0], fabs((s.tmpm[r] - s.z[r]) / e));
    v[1] = fmax(v[1], fabs(s.z[r] / e));
    v[2] = fmax(v[2], fabs(s.tmpm[r] / e));
  }
  for (int j = tid; j < n; j += nt) {
    const double d = s.D[j];
    v[3] = fmax(v[3], fabs((s.q[j] + s.aux[j] + s.tmpn[j]) / d));
    v[4] = fmax(v[4], fabs(s.q[j] / d));
    v[5] = fmax(v[5], fabs(s.tmpn[j] / d));
    v[6] = fmax(v[6], fabs(s.aux[j] / d));
  }
  block_max<8>(v, s.red);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = v[k];
}

template <class S>
__device__ bool qp_primal_infeasible(const QPPattern &pt, S &s, double eps) {
  // auxil.c is_primal_infeasible: delta_y projected IN PLACE onto the polar of the
  // recession cone of [l,u] (as OSQP does), then the two certificate tests.
  const int n = pt.n, m = pt.m, tid = threadIdx.x, nt = blockDim.x;
  double v[1] = {0.0};
  for (int r = tid; r < m; r += nt) {
    double d = s.dy[r];
    const bool bu = s.u[r] > QP_OSQP_INFTY * QP_MIN_SCALING;
    const bool bl = s.l[r] < -QP_OSQP_INFTY * QP_MIN_SCALING;
    if (bu && bl) d = 0.0;
    else if (bu) d = fmin(d, 0.0);
    else if (bl) d = fmax(d, 0.0);
    s.dy[r] = d;
    v[0] = fmax(v[0], fabs(s.E[r] * d));
  }
  block_max<1>(v, s.red);
  const double nrm = v[0];
  if (!(nrm > QP_DIV_TOL)) return false;
  double sm[1] = {0.0};
  for (int r = tid; r < m; r += nt)
    sm[0] += s.u[r] * fmax(s.dy[r], 0.0) + s.l[r] * fmin(s.dy[r], 0.0);
  block_sum<1>(sm, s.red);
  if (!(sm[0] < -eps * nrm)) return false;
  qp_spmv_t(pt, s, s.dy, s.rhs);  // rhs is free at check time
  __syncthreads();
  double mx[1] = {0.0};
  for (int j = tid; j < n; j += nt) mx[0] = fmax(mx[0], fabs(s.rhs[j] / s.D[j]));
  block_max<1>(mx, s.red);
  return mx[0] < eps * nrm;
}

template <class S>
__device__ bool qp_dual_infeasible(const QPPattern &pt, S &s, double eps) {
  const int n = pt.n, m = pt.m, tid = threadIdx.x, nt = blockDim.x;
  double v[1] = {0.0};
  for (int j = tid; j < n; j += nt) v[0] = fmax(v[0], fabs(s.D[j] * s.dx[j]));
  block_max<1>(v, s.red);
  const double nrm = v[0];
  if (!(nrm > QP_DIV_TOL)) return false;
  double a[1] = {0.0};
  for (int j = tid; j < n; j += nt) a[0] += s.q[j] * s.dx[j];
  double pm[1] = {0.0};
  for (int j = tid; j < n; j += nt) pm[0] = fmax(pm[0], fabs(s.P[j] * s.dx[j] / s.D[j]));
  block_sum<1>(a, s.red);
  block_max<1>(pm, s.red);
  if (!(a[0] < s.c * eps * nrm)) return false;
  if (!(pm[0] < s.c * eps * nrm)) return false;
  qp_spmv(pt, s, s.dx, s.zt);  // zt is rebuilt after every check
  __syncthreads();
  double bad[1] = {0.0};
  for (int r = tid; r < m; r += nt) {
    const double vv = s.zt[r] / s.E[r];
    if ((s.u[r] < QP_OSQP_INFTY * QP_MIN_SCALING && vv > eps * nrm) ||
        (s.l[r] > -QP_OSQP_INFTY * QP_MIN_SCALING && vv < -eps * nrm))
      bad[0] = 1.0;
  }
  block_max<1>(bad, s.red);
  return bad[0] == 0.0;
}

// auxil.c check_termination; status values as OSQP 0.6
template <class S>
__device__ bool qp_check(const QPPattern &pt, S &s, const QPSettingsDev &st, const double (&o)[8],
                         bool approx, int &status) {
  const double pri = o[0], dua = o[3] / s.c;
  double ea = st.eps_abs, er = st.eps_rel, epi = st.eps_prim_inf, edi = st.eps_dual_inf;
  if (pri > QP_OSQP_INFTY || dua > QP_OSQP_INFTY) {
    status = -7;
    return true;
  }
  if (approx) { ea *= 10; er *= 10; epi *= 10; edi *= 10; }
  bool prim_ok = false, prim_inf = false, dual_ok = false, dual_inf = false;
  if (pri < ea + er * fmax(o[1], o[2])) prim_ok = true;
  else prim_inf = qp_primal_infeasible(pt, s, epi);
  if (dua < ea + er * fmax(fmax(o[4], o[5]), o[6]) / s.c) dual_ok = true;
  else dual_inf = qp_dual_infeasible(pt, s, edi);
  if (prim_ok && dual_ok) { status = approx ? 2 : 1; return true; }
  if (prim_inf) { status = approx ? 3 : -3; return true; }
  if (dual_inf) { status = approx ? 4 : -4; return true; }
  return false;
}

// compute_rho_estimate in the scaled space, from qp_update_info's scratch
// (tmpm = A x, aux = P x, tmpn = A' y)
template <class S>
__device__ double qp_rho_estimate(const QPPattern &pt, S &s) {
  const int n = pt.n, m = pt.m, tid = threadIdx.x, nt = blockDim.x;
  double v[6] = {0, 0, 0, 0, 0, 0};
  for (int r = tid; r < m; r += nt) {
    v[0] = fmax(v[0], fabs(s.tmpm[r] - s.z[r]));
    v[1] = fmax(v[1], fmax(fabs(s.z[r]), fabs(s.tmpm[r])));
  }
  for (int j = tid; j < n; j += nt) {
    v[2] = fmax(v[2], fabs(s.q[j] + s.aux[j] + s.tmpn[j]));
    v[3] = fmax(v[3], fmax(fmax(fabs(s.q[j]), fabs(s.tmpn[j])), fabs(s.aux[j])));
  }
  block_max<6>(v, s.red);
  const double pr = v[0] / (v[1] + 1e-10);
  const double du = v[2] / (v[3] + 1e-10);
  double est = s.rho_s * sqrt(pr / (du + 1e-10));
  return fmin(fmax(est, QP_RHO_MIN), QP_RHO_MAX);
}

// diagnostic phase stamps (s_memtime), thread 0 only, enabled by a non-null pointer
struct QPStamps {
  unsigned long long *out = nullptr;
  unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long last = 0;
  __device__ void start() {
    if (out && threadIdx.x == 0) last = __builtin_amdgcn_s_memtime();
  }
  __device__ void mark(int k) {
    if (out && threadIdx.x == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc[k] += t - last;
      last = t;
    }
  }
  __device__ void flush() {
    if (out && threadIdx.x == 0)
      for (int k = 0; k < 8; ++k) out[k] += acc[k];
  }
};

struct QPResult {
  int status, iter;
  double obj;
  int factor_fail;
};

// The solve.  On entry s.A/P/q/l/u hold the UNSCALED problem, s.rho_s the
// persistent rho, s.y the persistent scaled dual, s.x the unscaled warm start.
// On exit s.x/s.y hold the scaled iterates (caller unscales), s.D/E/c the scaling.
template <class S>
__device__ QPResult qp_solve(const QPPattern &pt, S &s, const QPSettingsDev &st,
                             QPStamps *ts = nullptr) {
  const int n = pt.n, m = pt.m, tid = threadIdx.x, nt = blockDim.x;
  QPResult res{-10, 0, 0.0, 0};
  QPStamps dummy;
  QPStamps &T = ts ? *ts : dummy;
  for (int r = tid; r < m; r += nt) {
    s.l[r] = fmax(s.l[r], -QP_OSQP_INFTY);
    s.u[r] = fmin(s.u[r], QP_OSQP_INFTY);
  }
  __syncthreads();
  if (st.scaling) qp_scale(pt, s, st.scaling);
  else {
    for (int j = tid; j < n; j += nt) s.D[j] = 1.0;
    for (int r = tid; r < m; r += nt) s.E[r] = 1.0;
    if (tid == 0) s.c = 1.0;
    __syncthreads();
  }
  if (tid == 0) s.rho_s = fmin(fmax(s.rho_s, QP_RHO_MIN), QP_RHO_MAX);
  __syncthreads();
  T.mark(1);
  qp_set_rho(pt, s);
  int f = qp_factor(pt, s, st.sigma);
  T.mark(2);
  if (f) { res.factor_fail = f; return res; }
  if (st.warm_start) {
    for (int j = tid; j < n; j += nt) s.x[j] = s.x[j] / s.D[j];
    __syncthreads();
    qp_spmv(pt, s, s.x, s.z);
  } else {
    for (int j = tid; j < n; j += nt) s.x[j] = 0.0;
    for (int r = tid; r < m; r += nt) { s.z[r] = 0.0; s.y[r] = 0.0; }
  }
  __syncthreads();
  const double sig = st.sigma, al = st.alpha;
  // sparsity pattern of this thread's column (A' products) and rows (A
  // products) hoisted into registers for the whole solve
  int cn = 0, cidx[QP_CMAX], crow[QP_CMAX];
  if (tid < n) {
    const int k0 = pt.colptr[tid];
    cn = pt.colptr[tid + 1] - k0;
#pragma unroll
    for (int e = 0; e < QP_CMAX; ++e) {
      cidx[e] = (e < cn) ? pt.csc2csr[k0 + e] : 0;
      crow[e] = (e < cn) ? pt.cscrow[k0 + e] : 0;
    }
  }
  int rb[2], rn[2], rc[2][QP_RMAX];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = tid + h * 256;
    rb[h] = (r < m) ? pt.rowptr[r] : 0;
    rn[h] = (r < m) ? pt.rowptr[r + 1] - rb[h] : 0;
#pragma unroll
    for (int e = 0; e < QP_RMAX; ++e) rc[h][e] = (e < rn[h]) ? pt.colidx[rb[h] + e] : 0;
  }
  for (int r = tid; r < m; r += nt) s.zt[r] = s.rho[r] * s.z[r] - s.y[r];
  __syncthreads();
  bool can_check = false;
  int it;
  double o[8];
  for (it = 1; it <= st.max_iter; ++it) {
    // rhs = sigma x - q + A'(rho z - y)
    if (tid < n) {
      double acc = 0.0;
#pragma unroll
      for (int e = 0; e < QP_CMAX; ++e)
        if (e < cn) acc += s.A[cidx[e]] * s.zt[crow[e]];
      s.rhs[tid] = sig * s.x[tid] - s.q[tid] + acc;
    }
    __syncthreads();
    T.mark(3);
    qp_band_solve(pt, s, s.rhs);  // x~
    __syncthreads();
    T.mark(4);
    if (tid < n) {
      const double xo = s.x[tid];
      const double xn = al * s.rhs[tid] + (1.0 - al) * xo;
      s.dx[tid] = xn - xo;
      s.x[tid] = xn;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = tid + h * 256;
      if (r < m) {
        double zt = 0.0;  // z~ = A x~
#pragma unroll
        for (int e = 0; e < QP_RMAX; ++e)
          if (e < rn[h]) zt += s.A[rb[h] + e] * s.rhs[rc[h][e]];
        const double rho = s.rho[r], zo = s.z[r], yo = s.y[r];
        const double zr = al * zt + (1.0 - al) * zo;
        double zn = zr + yo / rho;
        zn = fmin(fmax(zn, s.l[r]), s.u[r]);
        const double d = rho * (zr - zn);
        const double yn = yo + d;
        s.dy[r] = d;
        s.y[r] = yn;
        s.z[r] = zn;
        s.zt[r] = rho * zn - yn;  // next iteration's A' operand
      }
    }
    __syncthreads();
    T.mark(5);
    can_check = st.check_termination && (it % st.check_termination == 0);
    const bool adapt = st.adaptive_rho && st.adaptive_rho_interval && (it % st.adaptive_rho_interval == 0);
    if (can_check) {
      res.iter = it;
      qp_update_info(pt, s, o);
      if (qp_check(pt, s, st, o, false, res.status)) break;
    }
    if (adapt) {
      if (!can_check) {
        res.iter = it;
        qp_update_info(pt, s, o);
      }
      const double est = qp_rho_estimate(pt, s);
      if (est > s.rho_s * st.adaptive_rho_tolerance || est < s.rho_s / st.adaptive_rho_tolerance) {
        __syncthreads();
        if (tid == 0) s.rho_s = est;
        __syncthreads();
        qp_set_rho(pt, s);
        f = qp_factor(pt, s, st.sigma);
        if (f) { res.factor_fail = f; return res; }
      }
    }
    if (can_check || adapt) {  // rebuild rho z - y (scratch reused / rho changed)
      for (int r = tid; r < m; r += nt) s.zt[r] = s.rho[r] * s.z[r] - s.y[r];
      __syncthreads();
    }
    T.mark(6);
  }
  if (!can_check) {
    res.iter = it - 1;
    qp_update_info(pt, s, o);
    qp_check(pt, s, st, o, false, res.status);
  }
  if (res.status == -10) {
    if (!qp_check(pt, s, st, o, true, res.status)) res.status = -2;
  }
  // objective (1/c)(1/2 x'Px + q'x)
  double ob[1] = {0.0};
  for (int j = tid; j < n; j += nt) ob[0] += 0.5 * s.x[j] * (s.P[j] * s.x[j]) + s.q[j] * s.x[j];
  block_sum<1>(ob, s.red);
  res.obj = ob[0] / s.c;
  return res;
}
