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
  double A[NNZMAX];
  double P[NMAX], q[NMAX], D[NMAX], x[NMAX], rhs[NMAX], dx[NMAX], aux[NMAX], invd[NMAX], tmpn[NMAX];
  double E[MMAX], l[MMAX], u[MMAX], rho[MMAX], y[MMAX], z[MMAX], zt[MMAX], dy[MMAX], tmpm[MMAX];
  double band[NMAX * (W + 1)];
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

// assemble M = P + sigma I + A' R A into the column band and factor it.
// band[j*(w+1)+t] = M[j+t][j] -> L[j+t][j]; invd[j] = 1/L[j][j].  Returns 0 or
// a 1-based failing column.
template <class S>
__device__ int qp_factor(const QPPattern &pt, S &s, double sigma) {
  const int n = pt.n, w = pt.w, nb = w + 1, tid = threadIdx.x, nt = blockDim.x;
  for (int e = tid; e < n * nb; e += nt) {
    const int j = e / nb, t = e - j * nb;
    double v = (t == 0) ? s.P[j] + sigma : 0.0;
    for (int k = pt.bandptr[e]; k < pt.bandptr[e + 1]; ++k) {
      const int r = pt.terms[3 * k], a = pt.terms[3 * k + 1], b = pt.terms[3 * k + 2];
      v += s.rho[r] * s.A[a] * s.A[b];
    }
    s.band[e] = v;
  }
  if (tid == 0) s.flag = 0;
  __syncthreads();
  const int nup = w * (w + 1) / 2;
  for (int j = 0; j < n; ++j) {
    double *col = s.band + j * nb;
    const double dj = col[0];
    double ct = 0.0, cs = 0.0;
    int t = 0, u = 0;
    const bool upd = tid < nup;
    if (upd) {  // map tid -> (t, u) with 1 <= u <= t <= w
      t = (int)((sqrt(8.0 * tid + 1.0) + 1.0) * 0.5);
      while (t * (t - 1) / 2 > tid) --t;
      while ((t + 1) * t / 2 <= tid) ++t;
      u = tid - t * (t - 1) / 2 + 1;
      ct = col[t];
      cs = col[u];
    }
    const double cw = (tid >= 1 && tid <= w) ? col[tid] : 0.0;
    __syncthreads();
    if (!(dj > 0.0)) {
      if (tid == 0) s.flag = j + 1;
      __syncthreads();
      return s.flag;
    }
    const double d = sqrt(dj);
    if (tid == 0) {
      col[0] = d;
      s.invd[j] = 1.0 / d;
    }
    if (tid >= 1 && tid <= w && j + tid < n) col[tid] = cw / d;
    if (upd && j + t < n) {
      // M[j+t][j+u] -= L[j+t][j] L[j+u][j]   (stored at band[(j+u)*nb + (t-u)])
      s.band[(j + u) * nb + (t - u)] -= (ct / d) * (cs / d);
    }
    __syncthreads();
  }
  return 0;
}

// b <- M^-1 b with M = L L' in the column band (wave 0 only; others idle)
template <class S>
__device__ void qp_band_solve(const QPPattern &pt, S &s, double *b) {
  if (threadIdx.x >= 64) return;
  const int n = pt.n, w = pt.w, nb = w + 1;
  const int lane = threadIdx.x;
  // forward: L y = b
  double win = (lane < n) ? b[lane] : 0.0;
#pragma unroll 2
  for (int j = 0; j < n; ++j) {
    const int pl = j & 63;
    const double yj = readlane_d(win, pl) * s.invd[j];
    const int t = 1 + ((lane - j - 1) & 63);  // row j + t owned by this lane
    const double lv = (t <= w && j + t < n) ? s.band[j * nb + t] : 0.0;
    if (lane == pl) {
      b[j] = yj;
      win = (j + 64 < n) ? b[j + 64] : 0.0;
    } else {
      win = fma(-lv, yj, win);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // backward: L' x = y
  {
    const int base = n - 64;
    const int i0 = base + ((lane - base) & 63);
    win = (i0 >= 0 && i0 < n) ? b[i0] : 0.0;
  }
#pragma unroll 2
  for (int i = n - 1; i >= 0; --i) {
    const int pl = i & 63;
    const double xi = readlane_d(win, pl) * s.invd[i];
    const int t = 1 + ((i - 1 - lane) & 63);  // row r = i - t owned by this lane
    const int r = i - t;
    const double lv = (t <= w && r >= 0) ? s.band[r * nb + t] : 0.0;
    if (lane == pl) {
      b[i] = xi;
      win = (i - 64 >= 0) ? b[i - 64] : 0.0;
    } else {
      win = fma(-lv, xi, win);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// residuals (auxil.c update_info) into s.zt = A x, s.aux = P x, s.dx-safe scratch
// returns pri, dua and the tolerance norms; scratch: zt <- Ax, aux <- Px, rhs <- A'y
template <class S>
__device__ void qp_update_info(const QPPattern &pt, S &s, double (&o)[8]) {
  const int n = pt.n, m = pt.m, tid = threadIdx.x, nt = blockDim.x;
  qp_spmv(pt, s, s.x, s.zt);
  qp_spmv_t(pt, s, s.y, s.rhs);
  for (int j = tid; j < n; j += nt) s.aux[j] = s.P[j] * s.x[j];
  __syncthreads();
  // o: 0 pri (unscaled)  1 |z/E|  2 |Ax/E|  3 dua*c  4 |q/D|  5 |A'y/D|  6 |Px/D|
  //    7 unused
  double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = tid; r < m; r += nt) {
    const double e = s.E[r];
    v[0] = fmax(v[0], fabs((s.zt[r] - s.z[r]) / e));
    v[1] = fmax(v[1], fabs(s.z[r] / e));
    v[2] = fmax(v[2], fabs(s.zt[r] / e));
  }
  for (int j = tid; j < n; j += nt) {
    const double d = s.D[j];
    v[3] = fmax(v[3], fabs((s.q[j] + s.aux[j] + s.rhs[j]) / d));
    v[4] = fmax(v[4], fabs(s.q[j] / d));
    v[5] = fmax(v[5], fabs(s.rhs[j] / d));
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
  qp_spmv_t(pt, s, s.dy, s.tmpn);
  __syncthreads();
  double mx[1] = {0.0};
  for (int j = tid; j < n; j += nt) mx[0] = fmax(mx[0], fabs(s.tmpn[j] / s.D[j]));
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
  qp_spmv(pt, s, s.dx, s.tmpm);
  __syncthreads();
  double bad[1] = {0.0};
  for (int r = tid; r < m; r += nt) {
    const double vv = s.tmpm[r] / s.E[r];
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

// compute_rho_estimate in the scaled space; scratch from qp_update_info still valid:
// zt = A x, aux = P x, rhs = A' y
template <class S>
__device__ double qp_rho_estimate(const QPPattern &pt, S &s) {
  const int n = pt.n, m = pt.m, tid = threadIdx.x, nt = blockDim.x;
  double v[6] = {0, 0, 0, 0, 0, 0};
  for (int r = tid; r < m; r += nt) {
    v[0] = fmax(v[0], fabs(s.zt[r] - s.z[r]));
    v[1] = fmax(v[1], fmax(fabs(s.z[r]), fabs(s.zt[r])));
  }
  for (int j = tid; j < n; j += nt) {
    v[2] = fmax(v[2], fabs(s.q[j] + s.aux[j] + s.rhs[j]));
    v[3] = fmax(v[3], fmax(fmax(fabs(s.q[j]), fabs(s.rhs[j])), fabs(s.aux[j])));
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
__device__ QPResult qp_solve(const QPPattern &pt, S &s, const QPSettingsDev &st) {
  const int n = pt.n, m = pt.m, tid = threadIdx.x, nt = blockDim.x;
  QPResult res{-10, 0, 0.0, 0};
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
  qp_set_rho(pt, s);
  int f = qp_factor(pt, s, st.sigma);
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
  bool can_check = false;
  int it;
  double o[8];
  for (it = 1; it <= st.max_iter; ++it) {
    // rhs = sigma x - q + A'(rho z - y)
    for (int r = tid; r < m; r += nt) s.zt[r] = s.rho[r] * s.z[r] - s.y[r];
    __syncthreads();
    qp_spmv_t(pt, s, s.zt, s.rhs);
    __syncthreads();
    for (int j = tid; j < n; j += nt) s.rhs[j] = sig * s.x[j] - s.q[j] + s.rhs[j];
    __syncthreads();
    qp_band_solve(pt, s, s.rhs);
    __syncthreads();
    qp_spmv(pt, s, s.rhs, s.zt);  // z~ = A x~
    for (int j = tid; j < n; j += nt) {
      const double xn = al * s.rhs[j] + (1.0 - al) * s.x[j];
      s.dx[j] = xn - s.x[j];
      s.x[j] = xn;
    }
    __syncthreads();
    for (int r = tid; r < m; r += nt) {
      const double zr = al * s.zt[r] + (1.0 - al) * s.z[r];
      double zn = zr + s.y[r] / s.rho[r];
      zn = fmin(fmax(zn, s.l[r]), s.u[r]);
      const double d = s.rho[r] * (zr - zn);
      s.dy[r] = d;
      s.y[r] += d;
      s.z[r] = zn;
    }
    __syncthreads();
    can_check = st.check_termination && (it % st.check_termination == 0);
    if (can_check) {
      res.iter = it;
      qp_update_info(pt, s, o);
      if (qp_check(pt, s, st, o, false, res.status)) break;
    }
    if (st.adaptive_rho && st.adaptive_rho_interval && (it % st.adaptive_rho_interval == 0)) {
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
