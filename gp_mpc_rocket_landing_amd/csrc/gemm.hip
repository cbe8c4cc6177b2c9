// gemm.hip -- fp64 "NT" GEMM on v_mfma_f64_16x16x4_f64 with fused epilogues.
//
//   acc = A(M x K) * B(N x K)^T   (both row-major, K contiguous)
//   EPI_STORE : C = alpha*acc + beta*C  (optionally lower triangle only)
//   EPI_SUMSQ : part[tile_row][j] = sum over the tile's rows of acc^2
//
// The GP posterior uses it with A = W = L^-1 (lower-triangular: the K loop of
// row tile t stops at the tile's last row) and B = K* = k(X*, X): the sum of
// squares of v = L^-1 k*^T is reduced in the epilogue, so v is never stored
// (SURVEY 8d "Variance TRSM: N^2 P flops").  FITC uses EPI_STORE as SYRK.
//
// Tile 64 x 64 per 256-thread workgroup, each wave a 32 x 32 quadrant
// (2 x 2 MFMA blocks), K staged 16 at a time through LDS with an 18-double
// pitch (conflict-free ds_read_b64 for the 16-row x 4-k operand gathers).
#include "internal.h"
#include "mfma64.h"
#include "gemm.h"

#define GT 64
#define GK 16
#define GP 18

template <int EPI>
__global__ __launch_bounds__(256) void k_gemm_nt(int M, int N, int K, const double *__restrict__ A,
                                                 int64_t lda, const double *__restrict__ B,
                                                 int64_t ldb, double *__restrict__ C, int64_t ldc,
                                                 double alpha, double beta, int tri_a,
                                                 int lower_c, int64_t sA_, int64_t sB_,
                                                 int64_t sC_) {
  const int bz = blockIdx.z;
  A += bz * sA_;
  B += bz * sB_;
  C += bz * sC_;
  const int r0 = blockIdx.y * GT, c0 = blockIdx.x * GT;
  if (lower_c && c0 > r0 + GT - 1) return;
  __shared__ double sA[GT][GP];
  __shared__ double sB[GT][GP];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int qi = (wave >> 1) * 32, qj = (wave & 1) * 32;
  int kend = K;
  if (tri_a) kend = min(K, r0 + GT);
  d4_t acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = (d4_t){0.0, 0.0, 0.0, 0.0};
  // each thread loads 4 elements of A and 4 of B per K-step: row = tid/4, k = (tid%4)*4..+3
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  for (int k0 = 0; k0 < kend; k0 += GK) {
    double va[4], vb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k0 + lk + q;
      va[q] = (r0 + lr < M && k < kend) ? A[(int64_t)(r0 + lr) * lda + k] : 0.0;
      vb[q] = (c0 + lr < N && k < kend) ? B[(int64_t)(c0 + lr) * ldb + k] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sA[lr][lk + q] = va[q];
      sB[lr][lk + q] = vb[q];
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      const int kc = kk + (lane >> 4);
      const double a0 = sA[qi + (lane & 15)][kc], a1 = sA[qi + 16 + (lane & 15)][kc];
      const double b0 = sB[qj + (lane & 15)][kc], b1 = sB[qj + 16 + (lane & 15)][kc];
      acc[0][0] = mfma_f64(a0, b0, acc[0][0]);
      acc[0][1] = mfma_f64(a0, b1, acc[0][1]);
      acc[1][0] = mfma_f64(a1, b0, acc[1][0]);
      acc[1][1] = mfma_f64(a1, b1, acc[1][1]);
    }
  }
  if (EPI == EPI_STORE) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + qi + x * 16 + mf_row(lane, r);
          const int col = c0 + qj + y * 16 + mf_col(lane);
          if (row < M && col < N && (!lower_c || col <= row)) {
            double *p = C + (int64_t)row * ldc + col;
            *p = (beta == 0.0) ? alpha * acc[x][y][r] : alpha * acc[x][y][r] + beta * *p;
          }
        }
  } else {
    // sum of squares over rows (rows >= M contribute exact zeros)
    __shared__ double red[4][32];
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s0 = fma(acc[x][0][r], acc[x][0][r], s0);
        s1 = fma(acc[x][1][r], acc[x][1][r], s1);
      }
    s0 += __shfl_xor(s0, 16);
    s0 += __shfl_xor(s0, 32);
    s1 += __shfl_xor(s1, 16);
    s1 += __shfl_xor(s1, 32);
    if (lane < 16) {
      red[wave][lane] = s0;
      red[wave][16 + lane] = s1;
    }
    __syncthreads();
    if (tid < 64) {
      // column tid of the tile: quadrant column half qj = (tid >= 32) * 32
      const int half = tid >> 5, cc = tid & 31;
      const double v = red[half][cc] + red[2 + half][cc];  // waves (0,half) and (1,half)
      const int col = c0 + tid;
      if (col < N) C[(int64_t)blockIdx.y * ldc + col] = v;
    }
  }
}

hipError_t launch_gemm_nt(hipStream_t s, int epi, int M, int N, int K, const double *A,
                          int64_t lda, const double *B, int64_t ldb, double *C, int64_t ldc,
                          double alpha, double beta, int tri_a, int lower_c, int batch,
                          int64_t sA, int64_t sB, int64_t sC) {
  if (M <= 0 || N <= 0) return hipSuccess;
  dim3 g((N + GT - 1) / GT, (M + GT - 1) / GT, batch);
  if (epi == EPI_STORE)
    hipLaunchKernelGGL(k_gemm_nt<EPI_STORE>, g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc,
                       alpha, beta, tri_a, lower_c, sA, sB, sC);
  else
    hipLaunchKernelGGL(k_gemm_nt<EPI_SUMSQ>, g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc,
                       alpha, beta, tri_a, 0, sA, sB, sC);
  return hipGetLastError();
}
