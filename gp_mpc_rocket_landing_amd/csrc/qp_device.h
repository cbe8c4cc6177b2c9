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
#include <utility>

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
  // factor storage: fac_len LDS slots assembled as  [P_d + sigma] + sum rho_r A[a] A[b]
  int mode;            // 0: banded LDL^T (slot j*(W+1)+t);  1: block tridiagonal (qp_block.h)
  int fac_len;
  int nblk, bsz, bcm;  // mode 1: nblk blocks of bsz variables, coupling prefix bcm
  const int *facptr;   // fac_len+1  slot -> term range
  const int *facdiag;  // fac_len    variable d whose P_d + sigma lands in the slot, -1 none, -2 one
  const int *terms;    // 3*nterms: (row, a, b) value pairs with rho_row*A[a]*A[b]
  // mode 1, dynamics-row (rho_eq) slots only: one int4 per slot that is not a
  // variable's diagonal and is either an identity pad or has terms:
  // x = slot | pad-one << 15 | nterms << 16, y/z/w = its terms as a | b << 16.
  // Every other non-diagonal slot is zero.  n_offd < 0: not available (a slot
  // with more than 3 terms, or mode 0).
  const int4 *offd;
  int n_offd;
};

template <int NMAX, int MMAX, int NNZMAX, int W>
struct QPSmem {
  static constexpr int NB = W + 1;  // band column stride
  __device__ double *band() { return band_store; }
  double A[NNZMAX];
  double P[NMAX], q[NMAX], D[NMAX], x[NMAX], rhs[NMAX], dx[NMAX], aux[NMAX], tmpn[NMAX];
  double E[MMAX], l[MMAX], u[MMAX], rho[MMAX], y[MMAX], z[MMAX], zt[MMAX], dy[MMAX], tmpm[MMAX];
  // column band, stride W+1: slot 0 of column j holds 1/D_j after factoring,
  // slots 1..W the multipliers L^[j+t][j] (zero beyond the pattern's w);
  // 64 doubles of tail padding for the sweeps' masked-lane loads
  double band_store[NMAX * (W + 1) + 4 * (W + 1) + 64];
  double red[4][8];
  double zslot, sink;  // block solve: a 0.0 source and a write sink for idle lanes
  double gzero[64];    // block solve: zero "-G rows" of non-coupled lanes (>= (SZ-1)*CM + 1)
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
// M = L^ D L^T (L^ unit lower).  band[j*NB+t] = M[j+t][j] -> L^[j+t][j]
// (1 <= t <= w), band[j*NB] = 1/D[j].  The sweeps then need no division on
// their critical path.  Returns 0 or a 1-based failing column.
template <class S>
__device__ int blk_factor_dispatch(const QPPattern &pt, S &s);

template <class S>
__device__ int qp_factor(const QPPattern &pt, S &s, double sigma) {
  constexpr int nb = S::NB;
  const int n = pt.n, w = pt.w, tid = threadIdx.x, nt = blockDim.x;
  double *band = s.band();
  for (int e = tid; e < pt.fac_len + 4 * nb; e += nt) {
    double v = 0.0;
    if (e < pt.fac_len) {
      const int d = pt.facdiag[e];
      v = (d >= 0) ? s.P[d] + sigma : (d == -2 ? 1.0 : 0.0);
      for (int k = pt.facptr[e]; k < pt.facptr[e + 1]; ++k) {
        const int r = pt.terms[3 * k], a = pt.terms[3 * k + 1], b = pt.terms[3 * k + 2];
        v += s.rho[r] * s.A[a] * s.A[b];
      }
    }
    band[e] = v;
  }
  if (pt.mode == 1) {
    if (tid == 0) s.zslot = 0.0;
    for (int e = tid; e < (int)(sizeof(s.gzero) / sizeof(double)); e += nt) s.gzero[e] = 0.0;
    __syncthreads();
    int f = 0;
    if (tid < 64) f = blk_factor_dispatch(pt, s);
    if (tid == 0) s.flag = f;
    __syncthreads();
    return s.flag;
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
    if (tid == 0) col[0] = inv;
    if (tid >= 1 && tid <= w && j + tid < n) col[tid] = cw * inv;
    // M[j+t][j+u] -= l_t d_j l_u = (c_t / d_j) c_u   (stored at band[(j+u)*nb + (t-u)])
    if (upd && j + t < n) band[(j + u) * nb + (t - u)] -= (ct * inv) * cu;
    __syncthreads();
  }
  return 0;
}

// b <- M^-1 b with M = L^ D L^T in the column band (wave 0 only; others idle).
// Row i of the right-hand side lives in lane i mod 64 ("modular window").  At
// forward step j the pivot z_j is read from lane j mod 64 and the lanes of rows
// j+1..j+w take  win -= L^[row][j] z_j  under an exec mask (a 64-bit rotating
// SGPR pair), so no lane needs a zero multiplier and every lane's multiplier
// address is linear in the step: band + row*W + j*W (forward), band + row*W + i
// (backward).  All 16 loads of a 16-step group issue up front with immediate
// offsets.  The pivot lane keeps z_j; lanes that pivoted are captured and
// refilled from the next window in bulk at the end of the group (a refilled
// row is first updated >= 48 steps after its lane pivots).  A step is 2
// readlane + 1 masked FMA + 3 scalar ops.
__device__ __forceinline__ void fma_exec(double &acc, double l, double z, unsigned long long m) {
  unsigned long long sv;
  asm volatile(
      "s_mov_b64 %1, exec\n\t"
      "s_mov_b64 exec, %4\n\t"
      "v_fma_f64 %0, -%2, %3, %0\n\t"
      "s_mov_b64 exec, %1"
      : "+v"(acc), "=&s"(sv)
      : "v"(l), "s"(z), "s"(m));
}
__device__ __forceinline__ unsigned long long rotl64(unsigned long long x, int k) {
  k &= 63;
  return k ? (x << k) | (x >> (64 - k)) : x;
}

template <class S>
__device__ void qp_band_solve(const QPPattern &pt, S &s, double *b) {
  if (threadIdx.x >= 64) return;
  constexpr int W = S::NB - 1;
  const int n = pt.n, w = pt.w;
  const int lane = threadIdx.x;
  const double *band = s.band();
  const unsigned long long m0 = (1ull << w) - 1;  // w <= 16
  // ---- forward: L^ z = b ; stores w = z / D in b.  L^[row][j] = band[row*W + j*W + ... ]
  //      (band[j*NB + (row - j)] = band[j*W + row])
  {
    double win = (lane < n) ? b[lane] : 0.0;
    int row = lane;
    for (int j0 = 0; j0 < n; j0 += 64) {
      const int rn = j0 + 64 + lane;
      const double nxt = (rn < n) ? b[rn] : 0.0;
      const int jend = min(n, j0 + 64);
      double mine = 0.0;
      unsigned long long msk = rotl64(m0, j0 + 1);  // lanes (j+1 .. j+w) mod 64
      for (int g = j0; g < jend; g += 16) {
        const int cnt = min(16, jend - g);
        const double *p = band + g * W + row;
        if (cnt == 16) {
          double lv[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) lv[q] = p[q * W];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const double zj = readlane_d(win, (g + q) & 63);
            fma_exec(win, lv[q], zj, msk);
            msk = (msk << 1) | (msk >> 63);
          }
        } else {
          for (int q = 0; q < cnt; ++q) {
            const double lq = p[q * W];
            const double zj = readlane_d(win, (g + q) & 63);
            fma_exec(win, lq, zj, msk);
            msk = (msk << 1) | (msk >> 63);
          }
        }
        // lanes that pivoted in [g, g+cnt): capture z, take the next window's row
        const bool piv = (unsigned)(lane - (g - j0)) < (unsigned)cnt;
        mine = piv ? win : mine;
        win = piv ? nxt : win;
        row = piv ? row + 64 : row;
      }
      if (j0 + lane < jend) b[j0 + lane] = mine * band[(j0 + lane) * S::NB];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // ---- backward: L^T x = w.  L^[i][row] = band[row*NB + (i - row)] = band[row*W + i]
  {
    // lanes past the (partial) top window start on their row of the block below,
    // as if they had already pivoted in the top window
    const int top = ((n - 1) >> 6) << 6;
    int row = (top + lane < n) ? top + lane : top - 64 + lane;
    double win = (row >= 0) ? b[row] : 0.0;
    for (int i0 = top; i0 >= 0; i0 -= 64) {
      const int rp = i0 - 64 + lane;
      const double nxt = (rp >= 0) ? b[rp] : 0.0;
      const int ihi = min(n, i0 + 64) - 1;
      double mine = 0.0;
      unsigned long long msk = rotl64(m0, ihi - w);  // lanes (i-w .. i-1) mod 64
      for (int g = ihi; g >= i0; g -= 16) {
        const int cnt = min(16, g - i0 + 1);
        const double *p = band + max(row, 0) * W + g;  // step i = g - q at p[-q]
        if (cnt == 16) {
          double lv[16];
          const double *pb = p - 15;
#pragma unroll
          for (int q = 0; q < 16; ++q) lv[q] = pb[15 - q];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const double xi = readlane_d(win, (g - q) & 63);
            fma_exec(win, lv[q], xi, msk);
            msk = (msk >> 1) | (msk << 63);
          }
        } else {
          for (int q = 0; q < cnt; ++q) {
            const double lq = p[-q];
            const double xi = readlane_d(win, (g - q) & 63);
            fma_exec(win, lq, xi, msk);
            msk = (msk >> 1) | (msk << 63);
          }
        }
        // lanes that pivoted in (g-cnt, g]: capture x, take the row of the window below
        const bool piv = (unsigned)(lane - (g - cnt + 1 - i0)) < (unsigned)cnt;
        mine = piv ? win : mine;
        win = piv ? nxt : win;
        row = piv ? row - 64 : row;
      }
      if (i0 + lane <= ihi) b[i0 + lane] = mine;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// diagnostic phase stamps (s_memtime), thread 0 only, enabled by a non-null pointer
struct QPStamps {
  unsigned long long *out = nullptr;
  unsigned long long acc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long last = 0, first = 0, rt0 = 0;
  __device__ __forceinline__ void start() {
    if (out && threadIdx.x == 0) {
      last = first = __builtin_amdgcn_s_memtime();
      rt0 = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ __forceinline__ void mark(int k) {
    if (out && threadIdx.x == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc[k] += t - last;
      last = t;
    }
  }
  __device__ __forceinline__ void flush() {
    if (out && threadIdx.x == 0) {
      for (int k = 0; k < 14; ++k) out[k] += acc[k];
      out[14] += __builtin_amdgcn_s_memrealtime() - rt0;  // 100 MHz constant clock
      out[15] += last - first;                            // shader clock
    }
  }
};

#include "qp_block.h"

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
  // the block solve reads the right-hand side in whole blocks: zero the tail
  for (int j = n + tid; j < (int)(sizeof(s.rhs) / sizeof(double)); j += nt) s.rhs[j] = 0.0;
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
    if (pt.mode == 1 && pt.nblk == QP_NBLK_MPC20) {
      // x~ for the 3-DoF MPC at N = 20 (21 blocks): the G chain fully unrolled (wave 0),
      // the diagonal blocks eight a round on waves 0-1, the unrolled backward chain --
      // the fused chain's arithmetic in the same order (same bits), ~2.5x shorter
      blk_solve_dispatch<false, QP_NBLK_MPC20, 1>(pt, s, s.rhs, &T);
      __syncthreads();
      if (tid < 128) blk_solve_dispatch<false, QP_NBLK_MPC20, 2>(pt, s, s.rhs, &T);
      __syncthreads();
      blk_solve_dispatch<false, QP_NBLK_MPC20, 4>(pt, s, s.rhs, &T);
    } else if (pt.mode == 1) blk_solve_dispatch(pt, s, s.rhs, &T);  // x~
    else qp_band_solve(pt, s, s.rhs);
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
        // at max_iter the loop ends here: the new rho persists (the next solve
        // factors from scratch), so this factorisation would never be used
        if (it < st.max_iter) {
          f = qp_factor(pt, s, st.sigma);
          if (f) { res.factor_fail = f; return res; }
        }
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
