// chol.hip -- blocked right-looking fp64 Cholesky (single and batched), TRSM, POTRS.
//
// Replaces LAPACK dpotrf / dtrtrs / dpotrs reached from np.linalg.cholesky,
// scipy.linalg.solve_triangular and cho_solve (exact_gp.py:164-179, 251-260;
// sparse_gp.py:187-232, 293-296).
//
// potrf, per 32-wide panel k (all matrices of a batch in the same launches):
//   1. k_potrf_diag   one workgroup per matrix factors the 32x32 diagonal block
//                     in LDS (LAPACK pivot test: fail unless a_jj > 0), stores
//                     L_kk and its inverse;
//   2. k_potrf_panel  A[i,k] <- A[i,k] L_kk^-T for the rows below (as a GEMM
//                     with the precomputed inverse);
//   3. k_syrk_mfma    trailing lower update A[i,j] -= A[i,k] A[j,k]^T on
//                     v_mfma_f64_16x16x4_f64, 64x64 tiles, 4 waves x 32x32.
// A failed pivot sets info[b] (1-based column) and freezes that matrix.
#include "internal.h"
#include "mfma64.h"

#define NB 32
#define TP 34  // LDS pitch (doubles) for 32-wide tiles: conflict-free ds_read_b64

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_potrf_diag(int n, int k0, double *A, int64_t lda,
                                                    int64_t stride, int *info, double *Linv) {
  const int b = blockIdx.x;
  if (info[b]) return;
  double *M = A + (int64_t)b * stride;
  const int nb = min(NB, n - k0);
  __shared__ double s[NB][NB + 1];
  __shared__ double inv[NB][NB + 1];
  __shared__ int fail;
  const int tid = threadIdx.x;
  for (int e = tid; e < NB * NB; e += 256) {
    int i = e / NB, j = e % NB;
    s[i][j] = (i < nb && j <= i) ? M[(int64_t)(k0 + i) * lda + k0 + j] : 0.0;
  }
  if (tid == 0) fail = 0;
  __syncthreads();
  for (int j = 0; j < nb; ++j) {
    if (tid == 0) {
      double v = s[j][j];
      if (!(v > 0.0)) fail = j + 1;
      else s[j][j] = sqrt(v);
    }
    __syncthreads();
    if (fail) break;
    const double piv = s[j][j];
    for (int i = j + 1 + tid; i < nb; i += 256) s[i][j] /= piv;
    __syncthreads();
    const int w = nb - j - 1;
    for (int e = tid; e < w * w; e += 256) {
      int i = j + 1 + e / w, c = j + 1 + e % w;
      if (c <= i) s[i][c] -= s[i][j] * s[c][j];
    }
    __syncthreads();
  }
  if (fail) {
    if (tid == 0) info[b] = k0 + fail;
    return;
  }
  for (int e = tid; e < nb * nb; e += 256) {
    int i = e / nb, j = e % nb;
    if (j <= i) M[(int64_t)(k0 + i) * lda + k0 + j] = s[i][j];
  }
  // inverse of the lower-triangular block, one column per thread
  if (tid < NB) {
    const int c = tid;
    for (int r = 0; r < NB; ++r) {
      double v;
      if (r < c || r >= nb || c >= nb) v = (r == c) ? 1.0 : 0.0;
      else {
        double sum = (r == c) ? 1.0 : 0.0;
        for (int k = c; k < r; ++k) sum -= s[r][k] * inv[k][c];
        v = sum / s[r][r];
      }
      inv[r][c] = v;
    }
  }
  __syncthreads();
  double *Li = Linv + (int64_t)b * NB * NB;
  for (int e = tid; e < NB * NB; e += 256) Li[e] = inv[e / NB][e % NB];
}

// A[r, k0:k0+nb] <- A[r, k0:k0+nb] * Linv^T for rows r in [k0+nb, n)
__global__ __launch_bounds__(256) void k_potrf_panel(int n, int k0, double *A, int64_t lda,
                                                     int64_t stride, const int *info,
                                                     const double *Linv) {
  const int b = blockIdx.y;
  if (info[b]) return;
  double *M = A + (int64_t)b * stride;
  const int nb = min(NB, n - k0);
  const int r0 = k0 + nb + blockIdx.x * 64;
  __shared__ double sA[64][TP];
  __shared__ double sL[NB][TP];
  const int tid = threadIdx.x;
  for (int e = tid; e < 64 * NB; e += 256) {
    int r = e / NB, j = e % NB;
    sA[r][j] = (r0 + r < n && j < nb) ? M[(int64_t)(r0 + r) * lda + k0 + j] : 0.0;
  }
  const double *Li = Linv + (int64_t)b * NB * NB;
  for (int e = tid; e < NB * NB; e += 256) sL[e / NB][e % NB] = Li[e];
  __syncthreads();
  const int r = tid >> 2, cb = (tid & 3) * 8;
  if (r0 + r >= n) return;
  double out[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) out[q] = 0.0;
  for (int j = 0; j < NB; ++j) {
    const double a = sA[r][j];
#pragma unroll
    for (int q = 0; q < 8; ++q) out[q] = fma(a, sL[cb + q][j], out[q]);  // Linv[c][j], j<=c
  }
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (cb + q < nb) M[(int64_t)(r0 + r) * lda + k0 + cb + q] = out[q];
}

__device__ __forceinline__ void lower_tile_index(int t, int &ti, int &tj) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  ti = i;
  tj = t - i * (i + 1) / 2;
}

// trailing update on the lower triangle of [t0, n) x [t0, n) with panel columns [k0, k0+kw)
__global__ __launch_bounds__(256) void k_syrk_mfma(int n, int k0, int kw, int t0, double *A,
                                                   int64_t lda, int64_t stride, const int *info) {
  const int b = blockIdx.y;
  if (info && info[b]) return;
  double *M = A + (int64_t)b * stride;
  int ti, tj;
  lower_tile_index(blockIdx.x, ti, tj);
  const int ri = t0 + ti * 64, rj = t0 + tj * 64;
  __shared__ double sI[64][TP];
  __shared__ double sJ[64][TP];
  const int tid = threadIdx.x;
  for (int e = tid; e < 64 * NB; e += 256) {
    int r = e / NB, j = e % NB;
    bool ok = j < kw;
    sI[r][j] = (ok && ri + r < n) ? M[(int64_t)(ri + r) * lda + k0 + j] : 0.0;
    sJ[r][j] = (ok && rj + r < n) ? M[(int64_t)(rj + r) * lda + k0 + j] : 0.0;
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  const int qi = (wave >> 1) * 32, qj = (wave & 1) * 32;
  d4_t acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = (d4_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < NB; kk += 4) {
    const int kc = kk + (lane >> 4);
    double a0 = sI[qi + (lane & 15)][kc], a1 = sI[qi + 16 + (lane & 15)][kc];
    double b0 = sJ[qj + (lane & 15)][kc], b1 = sJ[qj + 16 + (lane & 15)][kc];
    acc[0][0] = mfma_f64(a0, b0, acc[0][0]);
    acc[0][1] = mfma_f64(a0, b1, acc[0][1]);
    acc[1][0] = mfma_f64(a1, b0, acc[1][0]);
    acc[1][1] = mfma_f64(a1, b1, acc[1][1]);
  }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = ri + qi + x * 16 + mf_row(lane, r);
        const int col = rj + qj + y * 16 + mf_col(lane);
        if (row < n && col <= row) M[(int64_t)row * lda + col] -= acc[x][y][r];
      }
}

hipError_t launch_potrf_batched(hipStream_t s, int n, int batch, double *A, int64_t lda,
                                int64_t stride, int *info, double *Linv_scratch) {
  hipError_t e = hipMemsetAsync(info, 0, sizeof(int) * batch, s);
  if (e != hipSuccess) return e;
  for (int k0 = 0; k0 < n; k0 += NB) {
    const int nb = min(NB, n - k0);
    hipLaunchKernelGGL(k_potrf_diag, dim3(batch), dim3(256), 0, s, n, k0, A, lda, stride, info,
                       Linv_scratch);
    const int t0 = k0 + nb;
    const int rest = n - t0;
    if (rest <= 0) break;
    hipLaunchKernelGGL(k_potrf_panel, dim3((rest + 63) / 64, batch), dim3(256), 0, s, n, k0, A,
                       lda, stride, info, Linv_scratch);
    const int nt = (rest + 63) / 64;
    hipLaunchKernelGGL(k_syrk_mfma, dim3(nt * (nt + 1) / 2, batch), dim3(256), 0, s, n, k0, nb,
                       t0, A, lda, stride, info);
  }
  return hipGetLastError();
}

hipError_t launch_potrf_batched(hipStream_t s, int n, int batch, double *A, int64_t lda,
                                int64_t stride, int *info) {
  double *Linv = (double *)gpmpc_scratch(1, sizeof(double) * NB * NB * (size_t)batch);
  if (!Linv) return hipErrorOutOfMemory;
  return launch_potrf_batched(s, n, batch, A, lda, stride, info, Linv);
}

// ---------------------------------------------------------------------------
// Triangular solves.  Inverses of the 32x32 diagonal blocks of L first, then
// one workgroup per 64-column panel of X walks the row blocks (forward for
// L X = B, backward for L^T X = B).
__global__ __launch_bounds__(64) void k_tri_inv_blocks(int n, const double *L, int64_t ldl,
                                                       double *Linv) {
  const int ib = blockIdx.x, r0 = ib * NB;
  const int nb = min(NB, n - r0);
  __shared__ double s[NB][NB + 1];
  __shared__ double inv[NB][NB + 1];
  const int tid = threadIdx.x;
  for (int e = tid; e < NB * NB; e += 64) {
    int i = e / NB, j = e % NB;
    s[i][j] = (i < nb && j <= i) ? L[(int64_t)(r0 + i) * ldl + r0 + j] : (i == j ? 1.0 : 0.0);
  }
  __syncthreads();
  if (tid < NB) {
    const int c = tid;
    for (int r = 0; r < NB; ++r) {
      double v = 0.0;
      if (r >= c) {
        double sum = (r == c) ? 1.0 : 0.0;
        for (int k = c; k < r; ++k) sum -= s[r][k] * inv[k][c];
        v = sum / s[r][r];
      }
      inv[r][c] = v;
    }
  }
  __syncthreads();
  for (int e = tid; e < NB * NB; e += 64) Linv[(int64_t)ib * NB * NB + e] = inv[e / NB][e % NB];
}

// Solved row blocks of X are stored to global memory and re-read by other waves
// of the same workgroup in later steps.  The vector L1 is not refreshed by those
// stores (a line cached by the step's first read would be served stale), so every
// X read goes round L1 (agent-scope relaxed load = global_load sc1) and every
// step drains its stores (s_waitcnt vmcnt(0)) before the barrier.
__device__ __forceinline__ double ld_l2(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// X (n x nrhs, ld ldx) <- op(L)^-1 X ; op = L (trans=0) or L^T (trans=1)
// rhs_lower: X is known lower-triangular (X[r][c] = 0 for r < c, e.g. identity):
// the forward walk starts at the panel's first column.
__global__ __launch_bounds__(256) void k_trsm_panel(int n, int nrhs, const double *L, int64_t ldl,
                                                    const double *Linv, double *X, int64_t ldx,
                                                    int trans, int rhs_lower) {
  const int c0 = blockIdx.x * 64;
  const int nblk = (n + NB - 1) / NB;
  __shared__ double sL[NB][TP];
  __shared__ double sX[NB][64 + 1];
  const int tid = threadIdx.x;
  const int rr = tid >> 3;        // 0..31 row within block
  const int cc = (tid & 7) * 8;   // 8 columns
  for (int step = 0; step < nblk; ++step) {
    const int ib = trans ? (nblk - 1 - step) : step;
    if (!trans && rhs_lower && (ib + 1) * NB <= c0) continue;
    const int r0 = ib * NB;
    const int nbi = min(NB, n - r0);
    double acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int c = c0 + cc + q;
      acc[q] = (rr < nbi && c < nrhs) ? ld_l2(X + (int64_t)(r0 + rr) * ldx + c) : 0.0;
    }
    // subtract contributions of already-solved blocks
    const int kb_lo = trans ? ib + 1 : ((rhs_lower) ? (c0 / NB) : 0);
    const int kb_hi = trans ? nblk : ib;
    for (int kb = kb_lo; kb < kb_hi; ++kb) {
      const int k0 = kb * NB;
      const int nbk = min(NB, n - k0);
      __syncthreads();
      for (int e = tid; e < NB * NB; e += 256) {
        int i = e / NB, j = e % NB;
        double v = 0.0;
        if (!trans) {  // L[r0+i][k0+j]
          if (i < nbi && j < nbk) v = L[(int64_t)(r0 + i) * ldl + k0 + j];
        } else {       // (L^T)[r0+i][k0+j] = L[k0+j][r0+i]
          if (i < nbi && j < nbk) v = L[(int64_t)(k0 + j) * ldl + r0 + i];
        }
        sL[i][j] = v;
      }
      for (int e = tid; e < NB * 64; e += 256) {
        int i = e / 64, j = e % 64;
        int c = c0 + j;
        sX[i][j] = (i < nbk && c < nrhs) ? ld_l2(X + (int64_t)(k0 + i) * ldx + c) : 0.0;
      }
      __syncthreads();
      for (int j = 0; j < NB; ++j) {
        const double l = sL[rr][j];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = fma(-l, sX[j][cc + q], acc[q]);
      }
    }
    // apply the inverse of the diagonal block: X_ib = inv(op(L_ii)) * acc
    __syncthreads();
    for (int e = tid; e < NB * NB; e += 256) {
      int i = e / NB, j = e % NB;
      // inv(L^T) = inv(L)^T
      sL[i][j] = trans ? Linv[(int64_t)ib * NB * NB + j * NB + i] : Linv[(int64_t)ib * NB * NB + e];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) sX[rr][cc + q] = acc[q];
    __syncthreads();
    double out[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) out[q] = 0.0;
    for (int j = 0; j < NB; ++j) {
      const double l = sL[rr][j];
#pragma unroll
      for (int q = 0; q < 8; ++q) out[q] = fma(l, sX[j][cc + q], out[q]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int c = c0 + cc + q;
      if (rr < nbi && c < nrhs) X[(int64_t)(r0 + rr) * ldx + c] = out[q];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

hipError_t launch_trsm_lower_ex(hipStream_t s, int n, int nrhs, const double *L, int64_t ldl,
                                double *X, int64_t ldx, int trans, int rhs_lower,
                                double *Linv_blocks /* may be null */) {
  const int nblk = (n + NB - 1) / NB;
  double *Linv = Linv_blocks;
  if (!Linv) Linv = (double *)gpmpc_scratch(0, sizeof(double) * NB * NB * (size_t)nblk);
  if (!Linv) return hipErrorOutOfMemory;
  hipLaunchKernelGGL(k_tri_inv_blocks, dim3(nblk), dim3(64), 0, s, n, L, ldl, Linv);
  hipLaunchKernelGGL(k_trsm_panel, dim3((nrhs + 63) / 64), dim3(256), 0, s, n, nrhs, L, ldl, Linv,
                     X, ldx, trans, rhs_lower);
  return hipGetLastError();
}

hipError_t launch_trsm_lower(hipStream_t s, int n, int nrhs, const double *L, int64_t ldl,
                             double *X, int64_t ldx, int transpose_L) {
  return launch_trsm_lower_ex(s, n, nrhs, L, ldl, X, ldx, transpose_L, 0, nullptr);
}

// ---------------------------------------------------------------------------
// C-ABI
extern "C" int gpmpc_potrf(gpmpc_ctx *ctx, int n, double *A, int lda, int *info) {
  GPMPC_CHECK_ARG(ctx && A && info && n >= 0 && lda >= n);
  *info = 0;
  if (n == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  DevBuf dA, dinfo;
  GPMPC_HIP(dA.alloc(sizeof(double) * (size_t)n * n));
  GPMPC_HIP(dinfo.alloc(sizeof(int)));
  GPMPC_HIP(hipMemcpy2DAsync(dA.p, sizeof(double) * n, A, sizeof(double) * lda,
                             sizeof(double) * n, n, hipMemcpyHostToDevice, s));
  GPMPC_HIP(launch_potrf_batched(s, n, 1, dA.as<double>(), n, 0, dinfo.as<int>()));
  GPMPC_HIP(hipMemcpyAsync(info, dinfo.p, sizeof(int), hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipMemcpy2DAsync(A, sizeof(double) * lda, dA.p, sizeof(double) * n,
                             sizeof(double) * n, n, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return *info > 0 ? *info : 0;
}

extern "C" int gpmpc_potrf_batched_dev(gpmpc_ctx *ctx, int n, int batch, double *dA, int lda,
                                       int64_t stride, int *dinfo) {
  GPMPC_CHECK_ARG(ctx && dA && dinfo && n >= 0 && batch >= 0 && lda >= n);
  if (n == 0 || batch == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  GPMPC_HIP(launch_potrf_batched(ctx->stream, n, batch, dA, lda, stride, dinfo));
  return 0;
}

static int trsm_host(gpmpc_ctx *ctx, int n, int nrhs, const double *L, int ldl, double *B, int ldb,
                     int both) {
  GPMPC_CHECK_ARG(ctx && L && B && n >= 0 && nrhs >= 0 && ldl >= n && ldb >= nrhs);
  if (n == 0 || nrhs == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  DevBuf dL, dB;
  GPMPC_HIP(dL.alloc(sizeof(double) * (size_t)n * n));
  GPMPC_HIP(dB.alloc(sizeof(double) * (size_t)n * nrhs));
  GPMPC_HIP(hipMemcpy2DAsync(dL.p, sizeof(double) * n, L, sizeof(double) * ldl,
                             sizeof(double) * n, n, hipMemcpyHostToDevice, s));
  GPMPC_HIP(hipMemcpy2DAsync(dB.p, sizeof(double) * nrhs, B, sizeof(double) * ldb,
                             sizeof(double) * nrhs, n, hipMemcpyHostToDevice, s));
  GPMPC_HIP(launch_trsm_lower(s, n, nrhs, dL.as<double>(), n, dB.as<double>(), nrhs, 0));
  if (both) GPMPC_HIP(launch_trsm_lower(s, n, nrhs, dL.as<double>(), n, dB.as<double>(), nrhs, 1));
  GPMPC_HIP(hipMemcpy2DAsync(B, sizeof(double) * ldb, dB.p, sizeof(double) * nrhs,
                             sizeof(double) * nrhs, n, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

extern "C" int gpmpc_trsm_lower(gpmpc_ctx *ctx, int n, int nrhs, const double *L, int ldl,
                                double *B, int ldb) {
  return trsm_host(ctx, n, nrhs, L, ldl, B, ldb, 0);
}

extern "C" int gpmpc_potrs(gpmpc_ctx *ctx, int n, int nrhs, const double *L, int ldl, double *B,
                           int ldb) {
  return trsm_host(ctx, n, nrhs, L, ldl, B, ldb, 1);
}
