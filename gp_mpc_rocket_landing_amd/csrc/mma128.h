// mma128.h -- the 128 x 128 FP64-MFMA tile loop shared by the GEMM kernels
// (gemm.hip) and the per-matrix Cholesky (chol.hip).  gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "mfma64.h"

#ifndef GK
#define GK 16  // K staged per LDS step
#endif
#ifndef GP
#define GP 18  // LDS pitch (doubles) of a 16-wide K slice
#endif
#define BT 128
// acc = A[r0.., k_lo:k_hi] B[c0.., k_lo:k_hi]^T for one 128 x 128 tile (wave w
// owns quadrant (w/2, w%2)); k_lo must be a multiple of GK.  Ends on a barrier,
// so the LDS can be reused by the caller straight away.
__device__ __forceinline__ void mma128_tile(const double *__restrict__ A, int64_t lda,
                                            const double *__restrict__ B, int64_t ldb, int M, int N,
                                            int r0, int c0, int k_lo, int k_hi,
                                            double (*sA)[BT][GP], double (*sB)[BT][GP],
                                            d4_t (&acc)[4][4]) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int qi = (wave >> 1) * 64, qj = (wave & 1) * 64;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = (d4_t){0.0, 0.0, 0.0, 0.0};
  const int lr = tid >> 1, lk = (tid & 1) * 8;
  const bool ra = r0 + lr < M, rb = c0 + lr < N;
  const double *pa = A + (int64_t)(ra ? r0 + lr : 0) * lda;
  const double *pb = B + (int64_t)(rb ? c0 + lr : 0) * ldb;
  const bool vec = ((lda | ldb) & 1) == 0 && ((((uintptr_t)A) | ((uintptr_t)B)) & 15) == 0;
  double va[8], vb[8];
  auto gload = [&](int k0) {
    const int k = k0 + lk;
    if (vec && k + 7 < k_hi) {
#pragma unroll
      for (int q = 0; q < 8; q += 2) {
        const double2 av = ra ? *(const double2 *)(pa + k + q) : make_double2(0.0, 0.0);
        const double2 bv = rb ? *(const double2 *)(pb + k + q) : make_double2(0.0, 0.0);
        va[q] = av.x; va[q + 1] = av.y;
        vb[q] = bv.x; vb[q + 1] = bv.y;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        va[q] = (ra && k + q < k_hi) ? pa[k + q] : 0.0;
        vb[q] = (rb && k + q < k_hi) ? pb[k + q] : 0.0;
      }
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sA[buf][lr][lk + q] = va[q];
      sB[buf][lr][lk + q] = vb[q];
    }
  };
  gload(k_lo);
  lstore(0);
  __syncthreads();
  int cur = 0;
  for (int k0 = k_lo; k0 < k_hi; k0 += GK) {
    const bool more = k0 + GK < k_hi;
    if (more) gload(k0 + GK);
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      const int kc = kk + (lane >> 4);
      double a[4], b[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) a[x] = sA[cur][qi + 16 * x + (lane & 15)][kc];
#pragma unroll
      for (int y = 0; y < 4; ++y) b[y] = sB[cur][qj + 16 * y + (lane & 15)][kc];
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = mfma_f64(a[x], b[y], acc[x][y]);
    }
    if (more) lstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
}

