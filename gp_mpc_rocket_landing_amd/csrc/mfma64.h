// mfma64.h -- fp64 MFMA helpers for gfx950 (v_mfma_f64_16x16x4_f64).
//
// Operand maps (cdna_hip_programming.md section 3, f64 row):
//   A: lane l holds A[i = l & 15][k = l >> 4]      (16 x 4 block)
//   B: lane l holds B[k = l >> 4][j = l & 15]      (4 x 16 block)
//   C/D: 4 doubles per lane, reg r holds C[row = (l >> 4) + 4 r][col = l & 15]
// One instruction = 16*16*4*2 = 2048 flop.
#pragma once
#include <hip/hip_runtime.h>

typedef double d4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4_t mfma_f64(double a, double b, d4_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int mf_row(int lane, int r) { return (lane >> 4) + 4 * r; }
__device__ __forceinline__ int mf_col(int lane) { return lane & 15; }
