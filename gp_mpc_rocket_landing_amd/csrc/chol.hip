#include <algorithm>
// chol.hip -- blocked right-looking fp64 Cholesky (single and batched), TRSM, POTRS.
//
// Replaces LAPACK dpotrf / dtrtrs / dpotrs reached from np.linalg.cholesky,
// scipy.linalg.solve_triangular and cho_solve (exact_gp.py:164-179, 251-260;
// sparse_gp.py:187-232, 293-296).
//
// potrf (all matrices of a batch in the same launches), default path
// (launch_potrf_batched128): per 128-column panel, k_potrf_diag128 factors the
// 128 x 128 diagonal block in LDS and emits its inverse, the panel below is
// solved in place by one MFMA GEMM with that inverse, and one lower SYRK
// (MFMA) updates the trailing matrix -- three launches per panel.  The older
// 32-column two-level path (k_potrf_diag + GEMMs, ~100 launches at n = 1000)
// stays behind GPMPC_POTRF128=0.  LAPACK pivot test (fail unless a_jj > 0); a
// failed pivot sets info[b] (1-based column) and freezes that matrix's
// diagonal steps.
#include "internal.h"
#include "mfma64.h"
#include "gemm.h"
#include "mma128.h"

#define NB 32
#define TP 34  // LDS pitch (doubles) for 32-wide tiles: conflict-free ds_read_b64

// ---------------------------------------------------------------------------
// 32x32 diagonal block: one wave per matrix, row i of the block in lane i's
// registers.  Right-looking: the pivot comes by readlane, column j is
// broadcast through LDS (one ds_write per lane, wave-ordered reads, no
// barrier).  Then L^-1 by column-parallel forward substitution (lane c
// computes column c; every lane reads the same L[r][k] -> LDS broadcast).
__global__ __launch_bounds__(64) void k_potrf_diag(int n, int k0, double *A, int64_t lda,
                                                   int64_t stride, int *info, double *Linv) {
  const int b = blockIdx.x;
  if (info[b]) return;
  double *M = A + (int64_t)b * stride;
  const int nb = min(NB, n - k0);
  const int lane = threadIdx.x;
  __shared__ double col[NB];
  __shared__ double sl[NB][NB + 2];
  double a[NB];
  const bool live = lane < nb;
#pragma unroll
  for (int j = 0; j < NB; ++j)
    a[j] = (live && j <= lane) ? M[(int64_t)(k0 + lane) * lda + k0 + j] : (j == lane ? 1.0 : 0.0);
  int fail = 0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    if (j < nb) {
      const double piv = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(a[j]), j),
                                          __builtin_amdgcn_readlane(__double2loint(a[j]), j));
      if (!(piv > 0.0)) {
        fail = j + 1;
        break;
      }
      const double d = sqrt(piv), id = 1.0 / d;
      a[j] = (lane == j) ? d : a[j] * id;
      if (lane < NB) col[lane] = a[j];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const double lij = a[j];
#pragma unroll
      for (int k = j + 1; k < NB; ++k) a[k] = fma(-lij, col[k], a[k]);  // upper part: unused
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (fail) {
    if (lane == 0) info[b] = k0 + fail;
    return;
  }
  if (live) {
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (j <= lane) M[(int64_t)(k0 + lane) * lda + k0 + j] = a[j];
  }
  // L (identity beyond nb) to LDS, then column c of L^-1 in lane c
  if (lane < NB) {
#pragma unroll
    for (int j = 0; j < NB; ++j) sl[lane][j] = (j <= lane) ? a[j] : 0.0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double x[NB];
  const int c = lane;
#pragma unroll
  for (int r = 0; r < NB; ++r) {
    double sum = (r == c) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < r; ++k) sum = fma(-sl[r][k], x[k], sum);  // x[k] = 0 for k < c
    x[r] = (r >= c) ? sum / sl[r][r] : 0.0;
  }
  if (lane < NB) {
    double *Li = Linv + (int64_t)b * NB * NB;
#pragma unroll
    for (int r = 0; r < NB; ++r) Li[r * NB + c] = x[r];
  }
}

// ---------------------------------------------------------------------------
// 128 x 128 diagonal block of the outer panel, factored and inverted in one
// workgroup per matrix with the whole block resident in LDS (128 x 130
// doubles = 130 KB; pitch = 2 mod 32 makes the 16-row x 2-k MFMA operand
// gathers conflict-free).  Four 32-column steps:
//   1. wave 0: L_jj (rows in lane registers, pivot by readlane -- the
//      k_potrf_diag algorithm) -> global memory; T_j = L_jj^-1 -> the
//      block's lower triangle in LDS;
//   2. panel below: X = A T_j^T (v_mfma_f64_16x16x4, K = 32), stored after a
//      barrier (it overwrites its own operand);
//   3. trailing lower update A -= X X^T (MFMA; disjoint from the operands).
// Then the off-diagonal L blocks go to global memory and the full inverse
// Linv = L^-1 (128 x 128, for the panel GEMM A[t0:n] <- A[t0:n] Linv^T) is
// assembled block-row by block-row: X_ij = -T_i sum_{k=j}^{i-1} L_ik X_kj,
// X_ij stored transposed in the (free) upper triangle.
#define DB 128
#define DP 130
// S, then 1 / L_jj for the 128 columns, then the fail flag and the sweep's flags
#define DIAG128_LDS (sizeof(double) * (DB * DP + DB + 4))
// LDS-only ordering.  A release fence (and __syncthreads, which carries one)
// waits for every outstanding global store (vmcnt(0)) -- here the L blocks
// streamed out behind the factor -- which put ~1-2 us of store latency on the
// serial chain at every sync.  The data exchanged between lanes and waves in
// k_potrf_diag128 is LDS only, so LDS completion (lgkmcnt(0)) is enough; the
// "memory" clobber keeps the compiler from moving accesses across.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ double rdlane(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}

// diagnostic phase cycles of workgroup 0 (GPMPC_DIAG128_STAMPS=1 builds the <true> launch)
__device__ unsigned long long g_d128_stamps[8];
// sweep timeline of workgroup 0, cycles since the sweep start: per wave, the
// start and end of its owner block; the per-wave sweep end
__device__ unsigned long long g_sw_stamps[12];
// owner-step phases of wave 0 (block 0), workgroup 0: pivots, stores, tiles
__device__ unsigned long long g_sw_step[3];

// T = L^-1 of the 32 x 32 diagonal block at (c0, c0) of S, by the calling wave: T11
// (lanes 0-15) and T22 (lanes 16-31) by column substitution, T21 = -T22 (L21 T11) by
// two K = 16 MFMA products; T goes to the block's lower triangle (dinv: 1 / L_jj of
// the block).  The block's upper-right 16 x 16 is used as scratch.
__device__ __forceinline__ void tinv32(double (*S)[DP], int c0, const double *dinv) {
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  // T11 (lanes 0-15) and T22 (lanes 16-31): column c of the half in lane c
  const int base = lane & 16, c = lane & 15;
  double x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    double sum = (r == c) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < r; ++k) sum = fma(-S[c0 + base + r][c0 + base + k], x[k], sum);
    x[r] = (r >= c) ? sum * dinv[base + r] : 0.0;
  }
  wave_lds_sync();
  if (lane < NB) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (r >= c) S[c0 + base + r][c0 + base + c] = x[r];
  }
  wave_lds_sync();
  // Y = L21 T11 -> upper-right 16 x 16 of the block (free space)
  d4_t y = d4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < 16; kk += 4) {
    const int m = kk + lk;
    y = mfma_f64(S[c0 + 16 + li][c0 + m], (m >= li) ? S[c0 + m][c0 + li] : 0.0, y);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) S[c0 + mf_row(lane, r)][c0 + 16 + li] = y[r];
  wave_lds_sync();
  // T21 = -T22 Y over L21
  d4_t t21 = d4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < 16; kk += 4) {
    const int m = kk + lk;
    t21 = mfma_f64((m <= li) ? S[c0 + 16 + li][c0 + 16 + m] : 0.0, S[c0 + m][c0 + 16 + li],
                   t21);
  }
  wave_lds_sync();
#pragma unroll
  for (int r = 0; r < 4; ++r) S[c0 + 16 + mf_row(lane, r)][c0 + li] = -t21[r];
}

// Linv = L^-1 of the factored 128 x 128 block in S (diagonal blocks already
// inverted in place, tinv32) to Li, all four waves.
__device__ __forceinline__ void inv_assemble(double (*S)[DP], double *Li, bool zero_upper) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
  // Linv's diagonal blocks (T_i, lower; zero above) now, its zero upper blocks
  // on the first panel only (the scratch keeps them: later panels write the
  // same lower part); the off-diagonal blocks go out from the registers as
  // they are formed below
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = tid + 256 * q, blk = e >> 10, rr = (e >> 5) & 31, cc = e & 31;
    const int i = blk * NB + rr, j = blk * NB + cc;
    Li[i * DB + j] = (cc > rr) ? 0.0 : S[i][j];
  }
  if (zero_upper) {
#pragma unroll 2
    for (int q = 0; q < 24; ++q) {
      // upper blocks (bi, bj), bj > bi: (0,1) (0,2) (0,3) (1,2) (1,3) (2,3)
      const int e = tid + 256 * q, ub = e >> 10, rr = (e >> 5) & 31, cc = e & 31;
      const int bi = ub < 3 ? 0 : ub < 5 ? 1 : 2, bj = ub < 3 ? ub + 1 : ub < 5 ? ub - 1 : 3;
      Li[(bi * NB + rr) * DB + bj * NB + cc] = 0.0;
    }
  }
  // ---- inverse, block row i = 1..3:  Y_j = sum_k L_ik X_kj -> upper block (j, i)
  // transposed; then X_ij = -T_i Y_j in place.  Jobs: (j, 16x16 tile) pairs.
  for (int i = 1; i < DB / NB; ++i) {
    const int njob = 4 * i;
    d4_t acc[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      acc[q] = d4_t{0.0, 0.0, 0.0, 0.0};
      const int jt = wave + 4 * q;
      if (jt < njob) {
        const int j = jt >> 2, rb = (jt >> 1 & 1) * 16, cb = (jt & 1) * 16;
        for (int k = j; k < i; ++k) {
#pragma unroll
          for (int mm = 0; mm < NB; mm += 4) {
            const int m = mm + lk, cc = cb + li;
            const double av = S[i * NB + rb + li][k * NB + m];            // L_ik[r][m]
            double bv;                                                      // X_kj[m][cc]
            if (k == j) bv = (cc <= m) ? S[j * NB + m][j * NB + cc] : 0.0;  // T_j lower
            else bv = S[j * NB + cc][k * NB + m];                           // transposed X_kj
            acc[q] = mfma_f64(av, bv, acc[q]);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int jt = wave + 4 * q;
      if (jt < njob) {
        const int j = jt >> 2, rb = (jt >> 1 & 1) * 16, cb = (jt & 1) * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) S[j * NB + cb + li][i * NB + rb + mf_row(lane, r)] = acc[q][r];
      }
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      acc[q] = d4_t{0.0, 0.0, 0.0, 0.0};
      const int jt = wave + 4 * q;
      if (jt < njob) {
        const int j = jt >> 2, rb = (jt >> 1 & 1) * 16, cb = (jt & 1) * 16;
#pragma unroll
        for (int mm = 0; mm < NB; mm += 4) {
          const int m = mm + lk, rr = rb + li;
          const double av = (m <= rr) ? S[i * NB + rr][i * NB + m] : 0.0;  // T_i[rr][m]
          const double bv = S[j * NB + cb + li][i * NB + m];                // Y_j[m][cb+li]
          acc[q] = mfma_f64(av, bv, acc[q]);
        }
      }
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int jt = wave + 4 * q;
      if (jt < njob) {
        const int j = jt >> 2, rb = (jt >> 1 & 1) * 16, cb = (jt & 1) * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * NB + rb + mf_row(lane, r);
          S[j * NB + cb + li][row] = -acc[q][r];
          Li[row * DB + j * NB + cb + li] = -acc[q][r];
        }
      }
    }
    lds_barrier();
  }
}

// LDS layouts of the 128 x 128 block for the column sweep.  Full: 128 rows at pitch DP
// (130 KB: one workgroup per CU).  Packed lower (PK): 16-row block ib stores columns
// 0 .. 16 ib + 15 (its rows' lower part and the full 16 x 16 diagonal tile) at pitch
// 16 ib + 18 (18 or 2 mod 32, so the 16-row MFMA operand gathers stay conflict-free):
// 74 KB, two workgroups per CU.  No upper triangle: the factor's owner stores no zeros
// above the diagonal, the 32 x 32 inverses keep their Y = L21 T11 in registers
// (tinv32_pk) and the inverse is assembled in place of L (inv_assemble_pk).
struct LdsFull {
  static constexpr bool PK = false;
  double *p;
  __device__ __forceinline__ double &operator()(int r, int c) const { return p[r * DP + c]; }
  __device__ __forceinline__ double (*rows() const)[DP] { return reinterpret_cast<double (*)[DP]>(p); }
};
struct LdsPk {
  static constexpr bool PK = true;
  double *p;
  __device__ __forceinline__ double &operator()(int r, int c) const {
    const int ib = r >> 4;
    return p[128 * ib * (ib + 1) + 32 * ib + (r & 15) * (16 * ib + 18) + c];
  }
};
#define DPK_ELEMS (128 * 8 * 9 + 32 * 8)  // 9472 doubles
#define DIAG128_LDS_PK (sizeof(double) * (DPK_ELEMS + DB + 4))
// does row r of the packed layout store column c
__device__ __forceinline__ bool pk_has(int r, int c) { return c < 16 * (r >> 4) + 16; }

// tinv32 on the packed layout: T11 / T22 by column substitution as tinv32, then
// T21 = -T22 (L21 T11) with Y = L21 T11 kept in the MFMA accumulators: the second
// product's k index is permuted so that lane l's k slot at step s is row
// (l >> 4) + 4 s of Y, which is exactly its own accumulator entry s.
__device__ __forceinline__ void tinv32_pk(LdsPk S, int c0, const double *dinv) {
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int base = lane & 16, c = lane & 15;
  double x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    double sum = (r == c) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < r; ++k) sum = fma(-S(c0 + base + r, c0 + base + k), x[k], sum);
    x[r] = (r >= c) ? sum * dinv[base + r] : 0.0;
  }
  wave_lds_sync();
  if (lane < NB) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (r >= c) S(c0 + base + r, c0 + base + c) = x[r];
  }
  wave_lds_sync();
  d4_t y = d4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < 16; kk += 4) {
    const int m = kk + lk;
    y = mfma_f64(S(c0 + 16 + li, c0 + m), (m >= li) ? S(c0 + m, c0 + li) : 0.0, y);
  }
  d4_t t21 = d4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    const int m = lk + 4 * s4;  // = mf_row(lane, s4): y[s4] is Y[m][li]
    t21 = mfma_f64((m <= li) ? S(c0 + 16 + li, c0 + 16 + m) : 0.0, y[s4], t21);
  }
  wave_lds_sync();
#pragma unroll
  for (int r = 0; r < 4; ++r) S(c0 + 16 + mf_row(lane, r), c0 + li) = -t21[r];
}

// inv_assemble on the packed layout, in place of L: block row i = 1..3 (32 rows), job
// (j, cb) (j < i, 16-column half cb) forms both 16-row tiles of
//   Y_j = sum_{k=j}^{i-1} L_ik X_kj       (X_jj = T_j; X_kj, k > j, already in place of L_kj)
// in its accumulators; after a barrier (every read of row i's L blocks done)
//   X_ij = -T_i Y_j                        (Y_j's 32 rows from the two accumulators, k permuted)
// goes in place of L_ij and to Li.
__device__ __forceinline__ void inv_assemble_pk(LdsPk S, double *Li, bool zero_upper) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = tid + 256 * q, blk = e >> 10, rr = (e >> 5) & 31, cc = e & 31;
    const int i = blk * NB + rr, j = blk * NB + cc;
    Li[i * DB + j] = (cc > rr) ? 0.0 : S(i, j);
  }
  if (zero_upper) {
#pragma unroll 2
    for (int q = 0; q < 24; ++q) {
      const int e = tid + 256 * q, ub = e >> 10, rr = (e >> 5) & 31, cc = e & 31;
      const int bi = ub < 3 ? 0 : ub < 5 ? 1 : 2, bj = ub < 3 ? ub + 1 : ub < 5 ? ub - 1 : 3;
      Li[(bi * NB + rr) * DB + bj * NB + cc] = 0.0;
    }
  }
  for (int i = 1; i < DB / NB; ++i) {
    const int njob = 2 * i;
    d4_t y[2][2];  // [job round][row tile]
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      y[q][0] = y[q][1] = d4_t{0.0, 0.0, 0.0, 0.0};
      const int jt = wave + 4 * q;
      if (jt < njob) {
        const int j = jt >> 1, cb = (jt & 1) * 16, cc = cb + li;
        for (int k = j; k < i; ++k) {
#pragma unroll
          for (int mm = 0; mm < NB; mm += 4) {
            const int m = mm + lk;
            double bv;  // X_kj[m][cc]
            if (k == j) bv = (cc <= m) ? S(j * NB + m, j * NB + cc) : 0.0;
            else bv = S(k * NB + m, j * NB + cc);
            y[q][0] = mfma_f64(S(i * NB + li, k * NB + m), bv, y[q][0]);
            y[q][1] = mfma_f64(S(i * NB + 16 + li, k * NB + m), bv, y[q][1]);
          }
        }
      }
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int jt = wave + 4 * q;
      if (jt < njob) {
        const int j = jt >> 1, cb = (jt & 1) * 16;
#pragma unroll
        for (int ro = 0; ro < 2; ++ro) {  // output row tile
          d4_t x = d4_t{0.0, 0.0, 0.0, 0.0};
          const int rr = ro * 16 + li;    // A row: T_i[rr][m]
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            if (rb > ro) continue;  // T_i lower: rows 0-15 see only m < 16
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
              const int m = rb * 16 + lk + 4 * s4;  // y[q][rb][s4] = Y_j[m][cb + li]
              const double av = (m <= rr) ? S(i * NB + rr, i * NB + m) : 0.0;
              x = mfma_f64(av, y[q][rb][s4], x);
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = i * NB + ro * 16 + mf_row(lane, r);
            S(row, j * NB + cb + li) = -x[r];
            Li[row * DB + j * NB + cb + li] = -x[r];
          }
        }
      }
    }
    lds_barrier();
  }
}

// The factor + inverse of a 128 x 128 diagonal block already in LDS (S: lower
// triangle, identity padding beyond pw, zero upper triangle; sfail = 0), for
// k_potrf_diag128 and the per-matrix k_potrf_persist.  Writes L (rows < pw) at
// M and, when Li is non-null and pw == 128, Linv (128 x 128, upper zero) at Li.
// Returns 1 (uniformly) when a pivot fails, after setting *infob.
template <bool ST>
__device__ __forceinline__ int diag128_core(double (*S)[DP], double *col, int &sfail, double *M,
                                            int64_t lda, int pw, int K0, int *infob, double *Li,
                                            bool stamp, bool zero_upper) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
  unsigned long long tl = 0;
  auto mark = [&](int k) {
    if (ST && stamp && threadIdx.x == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (k >= 0) atomicAdd(&g_d128_stamps[k], t - tl);
      tl = t;
    }
  };
  mark(-1);
  // 32-column blocks holding real rows; the identity padding beyond pw is its
  // own factor and inverse, so a short last panel (or a small matrix) skips it
  const int nblk = (pw + NB - 1) / NB;
  // trailing lower update A -= X X^T of panel pc's 32 columns over the 16 x 16
  // tiles of the region [org, nblk*32)^2, tile t in row-major lower order
  // (t = 0, 1, 2 are the region's first 32 x 32 diagonal block)
  auto trail_tile = [&](int t, int org, int pc) {
    int ti = 0;
    while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
    const int tj = t - ti * (ti + 1) / 2;
    const int rb = org + ti * 16, cb = org + tj * 16;
    d4_t acc = d4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < NB; kk += 4) {
      const int k = pc + kk + lk;
      acc = mfma_f64(S[rb + li][k], S[cb + li][k], acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) S[rb + mf_row(lane, r)][cb + li] -= acc[r];
  };
  for (int jb = 0; jb < nblk; ++jb) {
    const int c0 = jb * NB;
    // ---- 3 (of the previous block, deferred): wave 0 updates only this block's
    // diagonal 32 x 32 and goes on to factor it; waves 1-3 update the rest of
    // the trailing region meanwhile (the panel step below waits for them)
    if (jb > 0) {
      const int nr = (nblk * NB - c0) >> 4, ntile = nr * (nr + 1) / 2;
      if (wave == 0) {
        for (int t = 0; t < 3; ++t) trail_tile(t, c0, c0 - NB);
        wave_lds_sync();
        mark(3);
      } else {
        for (int t = 3 + wave - 1; t < ntile; t += 3) trail_tile(t, c0, c0 - NB);
      }
    }
    // ---- 1. diagonal 32 x 32 block (wave 0).  Every wave instruction costs
    // >= 4 cycles and this chain is serial, so the block is factored in 4-column
    // steps: the 4 panel columns right-looking in lane registers (row = lane,
    // readlane broadcasts of 3 + 2 + 1 entries), the rest of the block by one
    // K = 4 MFMA per 16 x 16 tile.  Then T = L^-1 by 16 x 16 halves: T11 and T22
    // at once (lanes 0-15 / 16-31, one column each, LDS-broadcast L rows) and
    // T21 = -T22 (L21 T11) with two K = 16 MFMA products.
    if (wave == 0) {
      double *dinv = col;  // 1 / L_jj
      int fail = 0;
      const bool lv = lane < NB;
#pragma unroll
      for (int j = 0; j < NB; j += 4) {
        double p[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = (lv && lane >= j) ? S[c0 + lane][c0 + j + q] : 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double piv = rdlane(p[q], j + q);
          if (fail == 0 && !(piv > 0.0)) fail = j + q + 1;
          if (fail) continue;
            // 1/sqrt by v_rsq_f64 + two Newton steps, sqrt = piv * rsq: ~8
          // dependent instructions on the serial chain instead of ~27 for the
          // correctly rounded sqrt and division (L agrees to a few ulp)
          double id = __builtin_amdgcn_rsq(piv);
          id = id * fma(-0.5 * piv * id, id, 1.5);
          id = id * fma(-0.5 * piv * id, id, 1.5);
          const double d = piv * id;
          if (lane == j + q) dinv[j + q] = id;
          p[q] = (lane < j + q) ? 0.0 : (lane == j + q ? d : p[q] * id);
#pragma unroll
          for (int q2 = q + 1; q2 < 4; ++q2) p[q2] = fma(-p[q], rdlane(p[q], j + q2), p[q2]);
        }
        if (fail) break;
        if (lv && lane >= j) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (lane >= j + q) {
              S[c0 + lane][c0 + j + q] = p[q];
              if (c0 + lane < pw) M[(int64_t)(c0 + lane) * lda + c0 + j + q] = p[q];
            }
        }
        // only wave 0 touches this block now and one wave's LDS operations execute
        // in order, so no lgkmcnt wait: a compiler fence is enough
        asm volatile("" ::: "memory");
        const int j4 = j + 4;
        if (j4 < NB) {
          // lower 16 x 16 tiles meeting rows/cols >= j4: (1,1) always, (1,0) and (0,0)
          // while j4 < 16 (j is a compile-time constant here).  The tiles' operands
          // are the panel columns' two 16-row halves; all reads first, the MFMAs
          // back to back, then the read-modify-writes: one LDS round trip per stage
          // instead of one per tile (the columns read and written are disjoint)
          const bool lo = j4 < 16;
          const double v16 = S[c0 + 16 + li][c0 + j + lk];
          const double v0 = lo ? S[c0 + li][c0 + j + lk] : 0.0;
          const double a16 = (16 + li >= j4) ? v16 : 0.0, a0 = (li >= j4) ? v0 : 0.0;
          const d4_t z4 = d4_t{0.0, 0.0, 0.0, 0.0};
          const d4_t t11 = mfma_f64(a16, a16, z4);
          const d4_t t10 = lo ? mfma_f64(a16, a0, z4) : z4;
          const d4_t t00 = lo ? mfma_f64(a0, a0, z4) : z4;
          double o11[4], o10[4], o00[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            o11[r] = S[c0 + 16 + mf_row(lane, r)][c0 + 16 + li];
            if (lo) {
              o10[r] = S[c0 + 16 + mf_row(lane, r)][c0 + li];
              o00[r] = S[c0 + mf_row(lane, r)][c0 + li];
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            S[c0 + 16 + mf_row(lane, r)][c0 + 16 + li] = o11[r] - t11[r];
            if (lo) {
              S[c0 + 16 + mf_row(lane, r)][c0 + li] = o10[r] - t10[r];
              S[c0 + mf_row(lane, r)][c0 + li] = o00[r] - t00[r];
            }
          }
          asm volatile("" ::: "memory");
        }
      }
      mark(7);
      if (fail) {
        if (lane == 0) {
          *infob = K0 + c0 + fail;
          sfail = 1;
        }
      } else {
        tinv32(S, c0, dinv);
      }
    }
    lds_barrier();
    mark(1);
    if (sfail) return 1;
    const int R = nblk * NB - c0 - NB;  // rows below the diagonal block (real blocks only)
    if (R == 0) break;
    // ---- 2. panel X = A T^T: (R/16) x 2 tiles of 16 x 16, K = 32
    {
      const int nt = (R >> 4) * 2;
      d4_t acc[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        acc[q] = d4_t{0.0, 0.0, 0.0, 0.0};
        const int t = wave + 4 * q;
        if (t < nt) {
          const int rb = c0 + NB + (t >> 1) * 16, cb = (t & 1) * 16;
#pragma unroll
          for (int kk = 0; kk < NB; kk += 4) {
            const int k = kk + lk, cc = cb + li;
            const double av = S[rb + li][c0 + k];
            const double bv = (k <= cc) ? S[c0 + cc][c0 + k] : 0.0;  // T[cc][k], lower
            acc[q] = mfma_f64(av, bv, acc[q]);
          }
        }
      }
      lds_barrier();
      // X is final L (later steps touch only columns beyond this block): it goes to
      // global memory from the registers as well (the diagonal blocks went out in step 1)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int t = wave + 4 * q;
        if (t < nt) {
          const int rb = c0 + NB + (t >> 1) * 16, cb = (t & 1) * 16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = rb + mf_row(lane, r);
            S[row][c0 + cb + li] = acc[q][r];
            if (row < pw) M[(int64_t)row * lda + c0 + cb + li] = acc[q][r];
          }
        }
      }
      lds_barrier();
      mark(2);
    }
  }
  mark(4);
  if (pw < DB || !Li) return 0;  // the last panel has no rows below: no inverse needed
  inv_assemble(S, Li, zero_upper);
  mark(5);
  mark(6);
  return 0;
}


// The same factor + inverse as a column sweep with the rows owned by the waves
// (wave w: rows 32w..32w+31 of the block, one per lane) -- no per-block inverse
// or panel GEMM on the serial path.  For 32-column block jb, wave jb (the owner)
// factors its diagonal block in 4-column steps as diag128_core's wave 0 does and
// publishes each step (LDS flag); every wave below it (followers) applies the
// step to its own rows -- the 4 x 4 triangular solve with the owner's pivots,
// then its rows x the block's remaining columns by K = 4 MFMAs -- one step
// behind.  At the end of the block each follower publishes its panel rows and
// updates its rows x the column blocks jb+1..w by K = 32 MFMAs (the other waves'
// panel rows behind their flags).  The owner never waits, and the next owner
// (wave jb+1) only needs its own rows.  Flags only rise, and a failed pivot
// raises them all (SW_BIG), so no wave waits forever.  Afterwards each wave
// inverts its own diagonal block (tinv32) and inv_assemble forms Linv.
#define SW_BIG (1 << 20)
template <bool ST, class LS>
__device__ __forceinline__ int diag128_sweep(LS S, double *dinv, int &sfail, int *fl,
                                             double *M, int64_t lda, int pw, int K0, int *infob,
                                             double *Li, bool stamp, bool zero_upper, bool tblk) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lk = lane >> 4;
  unsigned long long tl = 0;
  auto mark = [&](int k) {
    if (ST && stamp && threadIdx.x == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (k >= 0) atomicAdd(&g_d128_stamps[k], t - tl);
      tl = t;
    }
  };
  // flags by relaxed workgroup-scope atomics: unlike volatile accesses they stay
  // LDS operations (a volatile access goes through a flat address and waits for
  // every outstanding global store)
  auto ld_flag = [](int *f) { return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  auto st_flag = [](int *f, int v) { __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  if (tid < 5) st_flag(fl + tid, 0);
  lds_barrier();
  mark(-1);
  const unsigned long long tsw = ST ? __builtin_amdgcn_s_memtime() : 0;
  auto swmark = [&](int k) {
    if (ST && stamp && lane == 0) atomicAdd(&g_sw_stamps[k], __builtin_amdgcn_s_memtime() - tsw);
  };
  // bounded: a wait that never ends (a broken invariant) fails the matrix with
  // info = -1 instead of hanging the device
  auto wait_ge = [&](int i, int v) {
    for (int spin = 0; ld_flag(fl + i) < v; ++spin) {
      if (spin > (1 << 22)) {
        if (lane == 0) {
          *infob = -1;
          st_flag(&sfail, 1);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
  };
  // LDS operations of one wave execute in order: the data written before a flag
  // is in place when another wave sees the flag
  auto publish = [&](int i, int v) {
    asm volatile("" ::: "memory");
    if (lane == 0) st_flag(fl + i, v);
  };
  const int nblk = (pw + NB - 1) / NB;
  const bool lv = lane < NB;
  const int w0 = wave * NB;
  const int r = w0 + (lane & 31);  // this lane's row of the block
  const d4_t z4 = d4_t{0.0, 0.0, 0.0, 0.0};
  bool out = wave >= nblk;
  for (int jb = 0; jb <= wave && !out; ++jb) {
    const int cb0 = jb * NB;
    if (wave == jb) {
      // ---- owner
      swmark(wave);
      int fail = 0;
#pragma unroll
      for (int j = 0; j < NB; j += 4) {
        double p[4];
        unsigned long long ts0 = 0;
        if (ST && stamp && wave == 0 && lane == 0) ts0 = __builtin_amdgcn_s_memtime();
        // the step's four columns of this lane's row (two 16-byte reads; rows above
        // the step read as zero)
        {
          const double2 *rp = reinterpret_cast<const double2 *>(&S(r, cb0 + j));
          const double2 x01 = rp[0], x23 = rp[1];
          const bool on = lv && lane >= j;
          p[0] = on ? x01.x : 0.0;
          p[1] = on ? x01.y : 0.0;
          p[2] = on ? x23.x : 0.0;
          p[3] = on ? x23.y : 0.0;
        }
        // the 4 x 4 diagonal block by readlane, factored as uniform values: the
        // pivot chain is rsq + Newton + two ops per column, with the row updates
        // off it (the same operations, in the same order, as the per-lane form)
        const double a00 = rdlane(p[0], j), a10 = rdlane(p[0], j + 1), a11 = rdlane(p[1], j + 1);
        const double a20 = rdlane(p[0], j + 2), a21 = rdlane(p[1], j + 2), a22 = rdlane(p[2], j + 2);
        const double a30 = rdlane(p[0], j + 3), a31 = rdlane(p[1], j + 3), a32 = rdlane(p[2], j + 3);
        const double a33 = rdlane(p[3], j + 3);
        auto rsqn = [](double piv) {
          double id = __builtin_amdgcn_rsq(piv);
          id = id * fma(-0.5 * piv * id, id, 1.5);
          return id * fma(-0.5 * piv * id, id, 1.5);
        };
        int f = !(a00 > 0.0) ? 1 : 0;
        const double id0 = rsqn(a00);
        const double l10 = a10 * id0, l20 = a20 * id0, l30 = a30 * id0;
        const double piv1 = fma(-l10, l10, a11);
        if (!f && !(piv1 > 0.0)) f = 2;
        const double b21 = fma(-l20, l10, a21), b31 = fma(-l30, l10, a31);
        const double b22 = fma(-l20, l20, a22), b32 = fma(-l30, l20, a32), b33 = fma(-l30, l30, a33);
        const double id1 = rsqn(piv1);
        const double l21 = b21 * id1, l31 = b31 * id1;
        const double piv2 = fma(-l21, l21, b22);
        if (!f && !(piv2 > 0.0)) f = 3;
        const double c32 = fma(-l31, l21, b32), c33 = fma(-l31, l31, b33);
        const double id2 = rsqn(piv2);
        const double l32 = c32 * id2;
        const double piv3 = fma(-l32, l32, c33);
        if (!f && !(piv3 > 0.0)) f = 4;
        const double id3 = rsqn(piv3);
        if (f) {
          fail = j + f;
          break;
        }
        // rows: the per-lane form; the pivot rows take sqrt(piv) on the diagonal
        // and zero above it
        {
          const double v0 = p[0] * id0;
          double q1 = fma(-v0, l10, p[1]);
          const double v1 = q1 * id1;
          double q2 = fma(-v0, l20, p[2]);
          q2 = fma(-v1, l21, q2);
          const double v2 = q2 * id2;
          double q3 = fma(-v0, l30, p[3]);
          q3 = fma(-v1, l31, q3);
          q3 = fma(-v2, l32, q3);
          const double v3 = q3 * id3;
          const int d = lane - j;
          p[0] = d == 0 ? a00 * id0 : v0;
          p[1] = d < 1 ? 0.0 : d == 1 ? piv1 * id1 : v1;
          p[2] = d < 2 ? 0.0 : d == 2 ? piv2 * id2 : v2;
          p[3] = d < 3 ? 0.0 : d == 3 ? piv3 * id3 : v3;
        }
        unsigned long long ts1 = 0;
        if (ST && stamp && wave == 0 && lane == 0) ts1 = __builtin_amdgcn_s_memtime();
        // LDS only: the diagonal block goes to global memory at the end of the sweep
        if (lane == 0) {
          double2 *dp = reinterpret_cast<double2 *>(&dinv[cb0 + j]);
          dp[0] = make_double2(id0, id1);
          dp[1] = make_double2(id2, id3);
        }
        if (lv && (!LS::PK || lane >= j)) {  // (packed: no upper-triangle storage)
          double2 *rp = reinterpret_cast<double2 *>(&S(r, cb0 + j));
          rp[0] = make_double2(p[0], p[1]);
          rp[1] = make_double2(p[2], p[3]);
        }
        publish(0, jb * 8 + j / 4 + 1);
        unsigned long long ts2 = 0;
        if (ST && stamp && wave == 0 && lane == 0) ts2 = __builtin_amdgcn_s_memtime();
        const int j4 = j + 4;
        if (j4 < NB) {
          const bool lo = j4 < 16;
          const double v16 = S(cb0 + 16 + li, cb0 + j + lk);
          const double v0 = lo ? S(cb0 + li, cb0 + j + lk) : 0.0;
          const double a16 = (16 + li >= j4) ? v16 : 0.0, a0 = (li >= j4) ? v0 : 0.0;
          const d4_t t11 = mfma_f64(a16, a16, z4);
          const d4_t t10 = lo ? mfma_f64(a16, a0, z4) : z4;
          const d4_t t00 = lo ? mfma_f64(a0, a0, z4) : z4;
          double o11[4], o10[4], o00[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            o11[q] = S(cb0 + 16 + mf_row(lane, q), cb0 + 16 + li);
            if (lo) {
              o10[q] = S(cb0 + 16 + mf_row(lane, q), cb0 + li);
              o00[q] = S(cb0 + mf_row(lane, q), cb0 + li);
            }
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            S(cb0 + 16 + mf_row(lane, q), cb0 + 16 + li) = o11[q] - t11[q];
            if (lo) {
              S(cb0 + 16 + mf_row(lane, q), cb0 + li) = o10[q] - t10[q];
              S(cb0 + mf_row(lane, q), cb0 + li) = o00[q] - t00[q];
            }
          }
          asm volatile("" ::: "memory");
        }
        if (ST && stamp && wave == 0 && lane == 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const unsigned long long ts3 = __builtin_amdgcn_s_memtime();
          atomicAdd(&g_sw_step[0], ts1 - ts0);
          atomicAdd(&g_sw_step[1], ts2 - ts1);
          atomicAdd(&g_sw_step[2], ts3 - ts2);
        }
      }
      swmark(4 + wave);
      if (fail) {
        if (lane == 0) {
          *infob = K0 + cb0 + fail;
          st_flag(&sfail, 1);
        }
        publish(0, SW_BIG);
        out = true;
        break;
      }
      // the factored diagonal blocks go to global memory off the owners' path:
      // block 0 by wave 0 now, block w+1 by wave w (idle once it has owned block w)
      // column group by column group behind the owner's step flags
      if (wave == 0) {
#pragma unroll 4
        for (int k = 0; k < NB * NB / 64; ++k) {
          const int e = lane + 64 * k, rr = e >> 5, cc = e & 31;
          if (cc <= rr && rr < pw) M[(int64_t)rr * lda + cc] = S(rr, cc);
        }
      }
      if (wave + 1 < nblk) {
        const int n0 = (wave + 1) * NB, rr = n0 + (lane & 31), ch = (lane >> 5) * 2;
#pragma unroll 1
        for (int j = 0; j < NB; j += 4) {
          wait_ge(0, (wave + 1) * 8 + j / 4 + 1);
          if (ld_flag(&sfail)) break;
          const int cc = n0 + j + ch;
          const double2 v = *reinterpret_cast<const double2 *>(&S(rr, cc));
          if (rr < pw) {
            if (cc <= rr) M[(int64_t)rr * lda + cc] = v.x;
            if (cc + 1 <= rr) M[(int64_t)rr * lda + cc + 1] = v.y;
          }
        }
      }
    } else {
      // ---- follower: the owner's step on this wave's rows.  The panel's update of
      // this wave's own diagonal block accumulates step by step (K = 4 each), so a
      // wave that owns the next block starts without a K = 32 product
      d4_t d00 = z4, d10 = z4, d11 = z4;
#pragma unroll
      for (int j = 0; j < NB; j += 4) {
        wait_ge(0, jb * 8 + j / 4 + 1);
        if (ld_flag(&sfail)) {
          out = true;
          break;
        }
        const int c = cb0 + j;
        double p[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = lv ? S(r, c + q) : 0.0;
        const double l10 = S(c + 1, c), l20 = S(c + 2, c), l30 = S(c + 3, c);
        const double l21 = S(c + 2, c + 1), l31 = S(c + 3, c + 1), l32 = S(c + 3, c + 2);
        p[0] *= dinv[c];
        p[1] = fma(-p[0], l10, p[1]);
        p[2] = fma(-p[0], l20, p[2]);
        p[3] = fma(-p[0], l30, p[3]);
        p[1] *= dinv[c + 1];
        p[2] = fma(-p[1], l21, p[2]);
        p[3] = fma(-p[1], l31, p[3]);
        p[2] *= dinv[c + 2];
        p[3] = fma(-p[2], l32, p[3]);
        p[3] *= dinv[c + 3];
        if (lv) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            S(r, c + q) = p[q];
            if (r < pw) M[(int64_t)r * lda + c + q] = p[q];
          }
        }
        asm volatile("" ::: "memory");
        const double a0 = S(w0 + li, c + lk), a1 = S(w0 + 16 + li, c + lk);
        d00 = mfma_f64(a0, a0, d00);
        d10 = mfma_f64(a1, a0, d10);
        d11 = mfma_f64(a1, a1, d11);
        const int j4 = j + 4;
        if (j4 < NB) {
          // own rows (two 16-row tiles) x the block's columns >= j4
          const bool lo = j4 < 16;
          const double b1 = (16 + li >= j4) ? S(cb0 + 16 + li, c + lk) : 0.0;
          const double b0 = (lo && li >= j4) ? S(cb0 + li, c + lk) : 0.0;
          const d4_t t01 = mfma_f64(a0, b1, z4), t11 = mfma_f64(a1, b1, z4);
          const d4_t t00 = lo ? mfma_f64(a0, b0, z4) : z4;
          const d4_t t10 = lo ? mfma_f64(a1, b0, z4) : z4;
          double o01[4], o11[4], o00[4], o10[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            o01[q] = S(w0 + mf_row(lane, q), cb0 + 16 + li);
            o11[q] = S(w0 + 16 + mf_row(lane, q), cb0 + 16 + li);
            if (lo) {
              o00[q] = S(w0 + mf_row(lane, q), cb0 + li);
              o10[q] = S(w0 + 16 + mf_row(lane, q), cb0 + li);
            }
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            S(w0 + mf_row(lane, q), cb0 + 16 + li) = o01[q] - t01[q];
            S(w0 + 16 + mf_row(lane, q), cb0 + 16 + li) = o11[q] - t11[q];
            if (lo) {
              S(w0 + mf_row(lane, q), cb0 + li) = o00[q] - t00[q];
              S(w0 + 16 + mf_row(lane, q), cb0 + li) = o10[q] - t10[q];
            }
          }
          asm volatile("" ::: "memory");
        }
      }
      if (out) break;
      publish(1 + wave, jb + 1);
      // block end: the accumulated own diagonal block, then own rows x column blocks
      // v = jb+1..wave-1, K = 32 over block jb's columns (block v's rows are wave
      // v's: behind its flag)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        S(w0 + mf_row(lane, q), w0 + li) -= d00[q];
        S(w0 + 16 + mf_row(lane, q), w0 + li) -= d10[q];
        S(w0 + 16 + mf_row(lane, q), w0 + 16 + li) -= d11[q];
      }
      asm volatile("" ::: "memory");
      for (int v = jb + 1; v < wave; ++v) {
        wait_ge(1 + v, jb + 1);
        if (ld_flag(&sfail)) {
          out = true;
          break;
        }
        const int v0 = v * NB;
        d4_t t00 = z4, t01 = z4, t10 = z4, t11 = z4;
#pragma unroll
        for (int kk = 0; kk < NB; kk += 4) {
          const int k = cb0 + kk + lk;
          const double a0 = S(w0 + li, k), a1 = S(w0 + 16 + li, k);
          const double b0 = S(v0 + li, k), b1 = S(v0 + 16 + li, k);
          t00 = mfma_f64(a0, b0, t00);
          t10 = mfma_f64(a1, b0, t10);
          t11 = mfma_f64(a1, b1, t11);
          t01 = mfma_f64(a0, b1, t01);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          S(w0 + mf_row(lane, q), v0 + li) -= t00[q];
          S(w0 + 16 + mf_row(lane, q), v0 + li) -= t10[q];
          S(w0 + 16 + mf_row(lane, q), v0 + 16 + li) -= t11[q];
          S(w0 + mf_row(lane, q), v0 + 16 + li) -= t01[q];
        }
        asm volatile("" ::: "memory");
      }
    }
  }
  if (out && wave < nblk) publish(1 + wave, SW_BIG);
  swmark(8 + wave);
  lds_barrier();
  mark(7);
  if (sfail) return 1;
  if (pw < DB || !Li) return 0;  // the last panel has no rows below: no inverse needed
  if constexpr (LS::PK) tinv32_pk(S, w0, dinv + w0);
  else tinv32(S.rows(), w0, dinv + w0);
  if (tblk) {
    // the TRSM-form panel solve (k_potrf_psolve_lat) takes the four inverted
    // diagonal blocks (lower part; it masks the rest) instead of the full inverse
    wave_lds_sync();
#pragma unroll
    for (int q = 0; q < NB * NB / 64; ++q) {
      const int e = lane + 64 * q;
      Li[wave * NB * NB + e] = S(w0 + (e >> 5), w0 + (e & 31));
    }
    mark(1);
    return 0;
  }
  lds_barrier();
  mark(1);
  if constexpr (LS::PK) inv_assemble_pk(S, Li, zero_upper);
  else inv_assemble(S.rows(), Li, zero_upper);
  mark(5);
  return 0;
}

// Panel solve X L^T = A (in place) for few matrices, in the TRSM form: with T_w the
// inverted 32 x 32 diagonal blocks of L (k_potrf_diag128's tblk output),
//   X_w = (A_w - sum_{k<w} X_k L_wk^T) T_w^T,   w = 0..3 (32-column blocks).
// A workgroup owns 16 rows; wave w owns column block w and holds A_w in its MFMA
// accumulators from the start, with its operands of L and T_w prefetched into
// registers (one memory round trip).  Stage s: wave s forms X_s (accumulator ->
// LDS -> A operand, times T_s^T) and hands it to the later waves through LDS;
// after the barrier they subtract X_s L_ws^T.  Replaces the 128 x 128 inverse
// (its assembly was ~20% of the diagonal kernel) and the full 128 x 128 x 128
// product with a half-triangular one.
__global__ __launch_bounds__(256) void k_potrf_psolve_lat(int M, const double *L, int64_t lda,
                                                          const double *Tb, double *X,
                                                          int64_t sL, int64_t sT, int64_t sX) {
  const int bz = blockIdx.z;
  L += bz * sL;
  Tb += bz * sT;
  X += bz * sX;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r0 = blockIdx.x * 16, w0 = wave * NB;
  __shared__ double sx[4][16][NB + 2];  // X_w, row-major (A-operand reads)
  d4_t acc0, acc1;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = r0 + mf_row(lane, q);
    acc0[q] = row < M ? X[(int64_t)row * lda + w0 + li] : 0.0;
    acc1[q] = row < M ? X[(int64_t)row * lda + w0 + 16 + li] : 0.0;
  }
  // B operands: L_wk^T (k < w) and T_w^T (lower: kk <= c)
  double lb[3][2][8], tb[2][8];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int t = 0; t < 8; ++t)
        lb[k][y][t] = k < wave ? L[(int64_t)(w0 + 16 * y + li) * lda + k * NB + 4 * t + lk] : 0.0;
#pragma unroll
  for (int y = 0; y < 2; ++y)
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int c = 16 * y + li, kk = 4 * t + lk;
      tb[y][t] = kk <= c ? Tb[wave * NB * NB + c * NB + kk] : 0.0;
    }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (wave == s) {
      // R (accumulators) -> LDS, back as the A operand of R T_s^T
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sx[s][mf_row(lane, q)][li] = acc0[q];
        sx[s][mf_row(lane, q)][16 + li] = acc1[q];
      }
      wave_lds_sync();
      d4_t x0 = d4_t{0.0, 0.0, 0.0, 0.0}, x1 = x0;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const double a = sx[s][li][4 * t + lk];
        x0 = mfma_f64(a, tb[0][t], x0);
        x1 = mfma_f64(a, tb[1][t], x1);
      }
      wave_lds_sync();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = r0 + mf_row(lane, q);
        sx[s][mf_row(lane, q)][li] = x0[q];
        sx[s][mf_row(lane, q)][16 + li] = x1[q];
        if (row < M) {
          X[(int64_t)row * lda + w0 + li] = x0[q];
          X[(int64_t)row * lda + w0 + 16 + li] = x1[q];
        }
      }
    }
    if (s == 3) break;
    lds_barrier();
    if (wave > s) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const double a = -sx[s][li][4 * t + lk];
        acc0 = mfma_f64(a, lb[s][0][t], acc0);
        acc1 = mfma_f64(a, lb[s][1][t], acc1);
      }
    }
  }
}

template <bool ST, bool PK = false>
__global__ __launch_bounds__(256) void k_potrf_diag128(int n, int K0, double *A, int64_t lda,
                                                       int64_t stride, int *info, double *Linv,
                                                       int sweep) {
  const int b = blockIdx.x;
  if (info[b]) return;
  // one dynamic region (no static LDS in front of it): S, then col, then the fail flag
  extern __shared__ double S_[];
  constexpr int SN = PK ? DPK_ELEMS : DB * DP;
  double *col = S_ + SN;
  int &sfail = *reinterpret_cast<int *>(S_ + SN + DB);
  int *sflags = reinterpret_cast<int *>(S_ + SN + DB) + 1;
  double *M = A + (int64_t)b * stride + (int64_t)K0 * lda + K0;
  const int pw = min(DB, n - K0);
  const int tid = threadIdx.x;
  // lower triangle in, identity padding beyond pw, zero upper triangle (packed: the
  // diagonal tiles' upper parts only); 32 loads in flight per lane before the LDS
  // stores (a load-store loop waits out the HBM latency once per element)
#pragma unroll 1
  for (int q0 = 0; q0 < DB * DB / 256; q0 += 32) {
    double v[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int e = tid + 256 * (q0 + q), i = e >> 7, j = e & 127;
      v[q] = (j <= i && i < pw) ? M[(int64_t)i * lda + j] : (i == j ? 1.0 : 0.0);
    }
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int e = tid + 256 * (q0 + q), i = e >> 7, j = e & 127;
      if (!PK) S_[i * DP + j] = v[q];
      else if (pk_has(i, j)) LdsPk{S_}(i, j) = v[q];
    }
  }
  if (tid == 0) sfail = 0;
  lds_barrier();
  double *Li = Linv ? Linv + (int64_t)b * DB * DB : nullptr;
  if constexpr (PK) {
    diag128_sweep<ST>(LdsPk{S_}, col, sfail, sflags, M, lda, pw, K0, info + b, Li, b == 0, K0 == 0,
                      (sweep & 2) != 0);
  } else {
    double(*S)[DP] = reinterpret_cast<double(*)[DP]>(S_);
    if (sweep)
      diag128_sweep<ST>(LdsFull{S_}, col, sfail, sflags, M, lda, pw, K0, info + b, Li, b == 0, K0 == 0,
                        (sweep & 2) != 0);
    else
      diag128_core<ST>(S, col, sfail, M, lda, pw, K0, info + b, Li, b == 0, K0 == 0);
  }
}

// ---------------------------------------------------------------------------
// One workgroup per matrix for the whole factorisation (large batches: every CU
// owns a matrix, no launch-level serial chain).  Left-looking 128-column panels:
//   1. update: panel rows [J, n) -= L[rows, 0:J] L[J:J+128, 0:J]^T, one 128 x 128
//      MFMA tile at a time (mma128_tile, K = J); the row tiles below go back to
//      the matrix in place, the diagonal tile straight into the LDS block;
//   2. diag128_core factors and inverts the diagonal block (L_JJ out, Linv to a
//      per-matrix workspace);
//   3. panel solve: rows [J+128, n) <- X Linv^T, one K = 128 tile at a time.
// Data written by one wave and read by another in a later phase crosses the
// (per-CU, not store-refreshed) vector L1, so every phase boundary is a release
// fence + barrier + agent acquire (L1 invalidate).  The GEMM staging buffers
// alias the LDS block (they are never live at the same time).
__device__ __forceinline__ void wg_global_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

__global__ __launch_bounds__(256) void k_potrf_persist(int n, double *A, int64_t lda, int64_t stride,
                                                       int *info, double *Lws) {
  const int b = blockIdx.x;
  extern __shared__ double S_[];
  double(*S)[DP] = reinterpret_cast<double(*)[DP]>(S_);
  double *col = S_ + DB * DP;
  int &sfail = *reinterpret_cast<int *>(S_ + DB * DP + DB);
  int *sflags = reinterpret_cast<int *>(S_ + DB * DP + DB) + 1;
  double(*sA)[BT][GP] = reinterpret_cast<double(*)[BT][GP]>(S_);
  double(*sB)[BT][GP] = reinterpret_cast<double(*)[BT][GP]>(S_ + 2 * BT * GP);
  double *Mb = A + (int64_t)b * stride;
  double *Li = Lws + (int64_t)b * DB * DB;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int qi = (wave >> 1) * 64, qj = (wave & 1) * 64;
  for (int J = 0; J < n; J += DB) {
    const int pw = min(DB, n - J);
    const int nrt = (n - J + DB - 1) / DB;
    if (J > 0) {
      // 1. update, bottom row tile first: the diagonal tile (rt = 0) lands in LDS last
      for (int rt = nrt - 1; rt >= 0; --rt) {
        d4_t acc[4][4];
        const int r0 = J + rt * DB;
        mma128_tile<false, false, false, false, false, false>(Mb + (int64_t)r0 * lda, lda, Mb + (int64_t)J * lda,
                                                              lda, n - r0, pw, 0, 0, 0, J, sA, sB, acc);
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int i = qi + x * 16 + mf_row(lane, r), j = qj + y * 16 + mf_col(lane);
              if (rt > 0) {
                if (r0 + i < n && j < pw) {
                  double *p = Mb + (int64_t)(r0 + i) * lda + J + j;
                  *p = *p - acc[x][y][r];
                }
              } else {
                S[i][j] = (j <= i && i < pw) ? Mb[(int64_t)(J + i) * lda + J + j] - acc[x][y][r]
                                             : (i == j ? 1.0 : 0.0);
              }
            }
      }
    } else {
#pragma unroll 1
      for (int q0 = 0; q0 < DB * DB / 256; q0 += 32) {
        double v[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) {
          const int e = tid + 256 * (q0 + q), i = e >> 7, j = e & 127;
          v[q] = (j <= i && i < pw) ? Mb[(int64_t)i * lda + j] : (i == j ? 1.0 : 0.0);
        }
#pragma unroll
        for (int q = 0; q < 32; ++q) {
          const int e = tid + 256 * (q0 + q);
          S[e >> 7][e & 127] = v[q];
        }
      }
    }
    if (tid == 0) sfail = 0;
    lds_barrier();
    // 2. diagonal block: L_JJ to the matrix, Linv to the workspace
    if (diag128_core<false>(S, col, sfail, Mb + (int64_t)J * lda + J, lda, pw, J, info + b,
                            J + DB < n ? Li : nullptr, false, J == 0))
      return;
    if (J + DB >= n) break;
    wg_global_sync();
    // 3. panel solve, in place (each tile's reads end on mma128_tile's barrier)
    for (int rt = 1; rt < nrt; ++rt) {
      d4_t acc[4][4];
      const int r0 = J + rt * DB;
      mma128_tile<false, false, false, false, false, false>(Mb + (int64_t)r0 * lda + J, lda, Li, DB, n - r0, DB, 0,
                                                            0, 0, DB, sA, sB, acc);
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = qi + x * 16 + mf_row(lane, r), j = qj + y * 16 + mf_col(lane);
            if (r0 + i < n) Mb[(int64_t)(r0 + i) * lda + J + j] = acc[x][y][r];
          }
    }
    wg_global_sync();
  }
}

// Two-level blocking.  Outer panels of OB = 128 columns; inside a panel,
// 32-wide steps (left-looking within the panel):
//   1. A[k0:n, k0:k0+32] -= A[k0:n, K0:k0] A[k0:k0+32, K0:k0]^T   (MFMA GEMM, K <= 96)
//   2. k_potrf_diag: L_kk and L_kk^-1
//   3. A[k0+32:n, k0:k0+32] <- A[k0+32:n, k0:k0+32] L_kk^-T      (MFMA GEMM, K = 32, in place:
//      one column tile per row block, every read precedes the epilogue)
// then one trailing SYRK per outer panel, lower triangle only:
//   A[t0:n, t0:n] -= A[t0:n, K0:t0] A[t0:n, K0:t0]^T             (MFMA GEMM, K = 128)
// so the O(n^3) work runs as K = 128 GEMMs on v_mfma_f64_16x16x4.
#define OB 128
hipError_t launch_potrf_batched(hipStream_t s, int n, int batch, double *A, int64_t lda,
                                int64_t stride, int *info, double *Linv_scratch) {
  hipError_t e = hipMemsetAsync(info, 0, sizeof(int) * batch, s);
  if (e != hipSuccess) return e;
  auto at = [&](int r, int c) { return A + (int64_t)r * lda + c; };
  for (int K0 = 0; K0 < n; K0 += OB) {
    const int pw = min(OB, n - K0);
    for (int k0 = K0; k0 < K0 + pw; k0 += NB) {
      const int nb = min(NB, n - k0);
      if (k0 > K0) {
        e = launch_gemm_nt(s, EPI_STORE, n - k0, nb, k0 - K0, at(k0, K0), lda, at(k0, K0), lda,
                           at(k0, k0), lda, -1.0, 1.0, 0, 1, batch, stride, stride, stride);
        if (e != hipSuccess) return e;
      }
      hipLaunchKernelGGL(k_potrf_diag, dim3(batch), dim3(64), 0, s, n, k0, A, lda, stride, info,
                         Linv_scratch);
      if (k0 + nb < n) {
        e = launch_gemm_nt(s, EPI_STORE, n - k0 - nb, nb, nb, at(k0 + nb, k0), lda, Linv_scratch,
                           NB, at(k0 + nb, k0), lda, 1.0, 0.0, 0, 0, batch, stride,
                           (int64_t)NB * NB, stride);
        if (e != hipSuccess) return e;
      }
    }
    const int t0 = K0 + pw;
    if (t0 < n) {
      e = launch_gemm_nt(s, EPI_STORE, n - t0, n - t0, pw, at(t0, K0), lda, at(t0, K0), lda,
                         at(t0, t0), lda, -1.0, 1.0, 0, 1, batch, stride, stride, stride);
      if (e != hipSuccess) return e;
    }
  }
  return hipGetLastError();
}

// Outer panels of 128 with the fused diagonal kernel: per panel three launches
//   k_potrf_diag128            L_KK (global) and Linv = L_KK^-1 (scratch)
//   A[t0:n, K0:t0] <- A[t0:n, K0:t0] Linv^T      (MFMA, K = 128, in place)
//   A[t0:n, t0:n]  -= A[t0:n, K0:t0] A[t0:n, K0:t0]^T  (lower SYRK, K = 128)
static hipError_t launch_potrf_batched128(hipStream_t s, int n, int batch, double *A, int64_t lda,
                                          int64_t stride, int *info, double *Linv) {
  static const bool st = [] {
    const char *e = getenv("GPMPC_DIAG128_STAMPS");
    return e && atoi(e);
  }();
  static bool attr = [] {
    return hipFuncSetAttribute((const void *)k_potrf_diag128<false>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)DIAG128_LDS) == hipSuccess &&
           hipFuncSetAttribute((const void *)k_potrf_diag128<true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)DIAG128_LDS) == hipSuccess &&
           hipFuncSetAttribute((const void *)k_potrf_diag128<false, true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)DIAG128_LDS_PK) == hipSuccess &&
           hipFuncSetAttribute((const void *)k_potrf_diag128<true, true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)DIAG128_LDS_PK) == hipSuccess;
  }();
  if (!attr) return hipErrorInvalidConfiguration;
  hipError_t e = hipMemsetAsync(info, 0, sizeof(int) * batch, s);
  if (e != hipSuccess) return e;
  auto at = [&](int r, int c) { return A + (int64_t)r * lda + c; };
  // few matrices: the panel solve and the trailing SYRK in the latency form
  // (k_gemm_lat: one memory round trip per launch instead of K / 16);
  // GPMPC_POTRF_LAT = 0 / 1 forces it off / on, default for batch <= lat_max
  static const int lat_env = [] {
    const char *v = getenv("GPMPC_POTRF_LAT");
    return v ? atoi(v) : -1;
  }();
  const bool lat = lat_env >= 0 ? lat_env > 0 : batch <= 16;
  // diagonal kernel: the column sweep (default) or the per-block inverse form
  static const int sweep = [] {
    const char *v = getenv("GPMPC_DIAG_SWEEP");
    return v ? atoi(v) : 1;
  }();
  // panel solve in the TRSM form (k_potrf_psolve_lat) with the diagonal kernel's
  // inverted 32 x 32 blocks, for the latency path (GPMPC_POTRF_TRSM=0: the full
  // inverse and the latency GEMM)
  static const int trsm_env = [] {
    const char *v = getenv("GPMPC_POTRF_TRSM");
    return v ? atoi(v) : -1;
  }();
  // (measured: batch 32 0.99 -> 0.86 ms, 64 1.35 -> 1.28 ms, 256 3.64 -> 3.75 ms)
  const bool tblk = sweep && (trsm_env >= 0 ? trsm_env > 0 : batch <= 64);
  // the diagonal kernel on the packed lower layout (74 KB of LDS: two workgroups per CU)
  // where there are more matrices than CUs (GPMPC_DIAG_PK = 0 / 1: off / whenever the
  // sweep runs)
  static const int pk_env = [] {
    const char *v = getenv("GPMPC_DIAG_PK");
    return v ? atoi(v) : -1;
  }();
  const bool pk = sweep && (pk_env >= 0 ? pk_env > 0 : batch > 256);
  // panel solve A[c+128:n, c:c+128] <- A[c+128:n, c:c+128] Linv^T (in place)
  auto psolve = [&](int c) {
    const int r = c + DB;
    if (tblk) {
      hipLaunchKernelGGL(k_potrf_psolve_lat, dim3((n - r + 15) / 16, 1, batch), dim3(256), 0, s,
                         n - r, at(c, c), lda, Linv, at(r, c), stride, (int64_t)DB * DB, stride);
      return hipGetLastError();
    }
    if (lat)
      return launch_gemm_lat(s, 0, n - r, DB, DB, at(r, c), lda, Linv, DB, at(r, c), lda, 1.0, 0.0,
                             1, batch, stride, (int64_t)DB * DB, stride);
    return launch_gemm_nt_rowblock(s, n - r, DB, DB, at(r, c), lda, Linv, DB, at(r, c), lda, 1.0,
                                   0.0, batch, stride, (int64_t)DB * DB, stride);
  };
  // Outer panels of OB = 128 m columns.  Inside a panel, 128-column steps are
  // left-looking (a step's columns take the update of the panel's earlier
  // steps, K = c - K0); across panels, one lower SYRK with K = OB, so the
  // O(n^3) work runs as K = OB products (fewer C read-modify-writes, longer K).
  // Default: 128 (right-looking, K = 128 SYRKs) below batch 128, 1024 (left-looking:
  // each 128-column block takes the update of all earlier columns, K = c, with no
  // trailing SYRK) from 256 on and from 128 for multiples of 8 (the fused steps) --
  // measured at n = 1000 (round 3, unfused): 64: 1.34 vs 1.60 ms, 256: 3.62 vs 3.58 ms,
  // 1024: 13.6 vs 13.2 ms.  256-512: no better than either.
  static const int ob_env = [] {
    const char *v = getenv("GPMPC_POTRF_OB");
    if (!v) return 0;
    const int m = atoi(v) / DB;
    return DB * (m < 1 ? 1 : m > 8 ? 8 : m);
  }();
  // left-looking from batch 128 when the fused steps apply (a multiple of 8): measured at
  // n = 1000, 128: 2.13 -> 1.95 ms, 192: 2.89 -> 2.54 ms; 64 stays right-looking (1.25 vs 1.36)
  const int OBk = ob_env ? ob_env : ((batch >= 256 || (batch >= 128 && batch % 8 == 0)) ? 8 * DB : DB);
  static const int ksplit_env = [] {
    const char *v = getenv("GPMPC_POTRF_KSPLIT");
    return v ? atoi(v) : 0;
  }();
  // Left-looking block columns, fused: the diagonal block's update alone, the diagonal
  // kernel, then ONE pass over the rows below (update + panel solve, k_gemm128_updsolve)
  // instead of an update launch over all rows and a panel-solve launch; for batches that
  // are a multiple of 8 whose rows below fill >= 512 workgroups (GPMPC_POTRF_FUSE=0: off)
  static const int fuse_env = [] {
    const char *v = getenv("GPMPC_POTRF_FUSE");
    return v ? atoi(v) : 1;
  }();
  const bool fuse_ok = fuse_env && OBk > DB && !tblk && !lat && batch % 8 == 0;
  // look-ahead (GPMPC_POTRF_LA=1): a fused step's first row tile also applies the next
  // fused step's diagonal-block update (k_gemm128_updsolve<true>), so that launch goes.
  // Off: the first row tiles become the launch's stragglers (batch 1024: 11.6 -> 15.0 ms)
  static const int la_env = [] {
    const char *v = getenv("GPMPC_POTRF_LA");
    return v ? atoi(v) : 0;
  }();
  // the diagonal block's update by the balanced lower-triangle kernel (k_syrk128_diag,
  // 9 MFMA blocks per wave) instead of the 128-tile kernel's quadrants (GPMPC_SYRK_DIAG=0)
  static const int syrk_diag_env = [] {
    const char *v = getenv("GPMPC_SYRK_DIAG");
    return v ? atoi(v) : 1;
  }();
  // a block column fuses when its rows below fill >= GPMPC_POTRF_FUSE_MIN workgroups (512)
  static const int fuse_min_env = [] {
    const char *v = getenv("GPMPC_POTRF_FUSE_MIN");
    return v ? atoi(v) : 0;
  }();
  // (batch 128: 512 -> 1.88 ms, 1 -> 1.95 ms; 256-1024: no difference)
  const int fuse_min = fuse_min_env ? fuse_min_env : 512;
  auto fuses = [&](int c) {
    const int below = n - c - min(DB, n - c);
    return fuse_ok && below > 0 && (below + DB - 1) / DB * batch >= fuse_min;
  };
  for (int K0 = 0; K0 < n; K0 += OBk) {
    const int pw = min(OBk, n - K0);
    bool la_prev = false;  // this step's diagonal update was applied by the previous step
    for (int c = K0; c < K0 + pw; c += DB) {
      const int w = min(DB, n - c);
      const int below = n - c - w;
      const bool fuse = fuses(c);
      const bool la = la_env && fuse && w == DB && c + DB < K0 + pw && fuses(c + DB);
      if (c > K0 && fuse && la_prev) {
        // the diagonal block's update came with the previous step's first row tile
      } else if (c > K0 && fuse) {
        // the diagonal block's rows only (one tile per matrix), K split to fill the device
        const int K = c - K0;
        int ks = 1;
        if (ksplit_env != 1)
          while (ks < K / DB && batch * ks < 512) ++ks;
        e = syrk_diag_env ? launch_syrk128_diag(s, w, K, at(c, K0), lda, at(c, c), batch, stride, ks)
                          : launch_gemm_nt_rowblock(s, w, w, K, at(c, K0), lda, at(c, K0), lda, at(c, c), lda, -1.0,
                                                    1.0, batch, stride, stride, stride, 1, ks);
        if (e != hipSuccess) return e;
      } else if (c > K0) {
        // the block column's update by all earlier columns of the outer panel; K split
        // (atomic partial sums) when its row tiles give fewer than ~2 workgroups per CU,
        // >= 128 of K per split (GPMPC_POTRF_KSPLIT=1: never)
        const int K = c - K0, tiles = (n - c + DB - 1) / DB * batch;
        int ks = 1;
        if (ksplit_env != 1)
          while (ks < K / DB && tiles * ks < 512) ++ks;
        // the last block column of a left-looking panel has no rows below: its diagonal block alone
        e = (syrk_diag_env && OBk > DB && n - c == w)
                ? launch_syrk128_diag(s, w, K, at(c, K0), lda, at(c, c), batch, stride, ks)
                : launch_gemm_nt_rowblock(s, n - c, w, K, at(c, K0), lda, at(c, K0), lda, at(c, c), lda,
                                          -1.0, 1.0, batch, stride, stride, stride, 1, ks);
        if (e != hipSuccess) return e;
      }
      if (pk && st)
        hipLaunchKernelGGL((k_potrf_diag128<true, true>), dim3(batch), dim3(256), DIAG128_LDS_PK, s, n, c, A,
                           lda, stride, info, c + DB < n ? Linv : nullptr, sweep | (tblk ? 2 : 0));
      else if (pk)
        hipLaunchKernelGGL((k_potrf_diag128<false, true>), dim3(batch), dim3(256), DIAG128_LDS_PK, s, n, c, A,
                           lda, stride, info, c + DB < n ? Linv : nullptr, sweep | (tblk ? 2 : 0));
      else if (st)
        hipLaunchKernelGGL(k_potrf_diag128<true>, dim3(batch), dim3(256), DIAG128_LDS, s, n, c, A,
                           lda, stride, info, c + DB < n ? Linv : nullptr, sweep | (tblk ? 2 : 0));
      else
        hipLaunchKernelGGL(k_potrf_diag128<false>, dim3(batch), dim3(256), DIAG128_LDS, s, n, c,
                           A, lda, stride, info, c + DB < n ? Linv : nullptr, sweep | (tblk ? 2 : 0));
      if (fuse) {
        e = launch_gemm_updsolve(s, below, c - K0, at(c + w, K0), lda, at(c, K0), at(c + w, c), Linv, batch,
                                 stride, stride, (int64_t)DB * DB, la ? min(DB, below) : 0);
        if (e != hipSuccess) return e;
      } else if (c + DB < n && (e = psolve(c)) != hipSuccess) {
        return e;
      }
      la_prev = la;
    }
    const int t0 = K0 + pw;
    if (t0 < n) {
      if (lat && pw <= DB)
        e = launch_gemm_lat(s, 1, n - t0, n - t0, pw, at(t0, K0), lda, nullptr, lda, at(t0, t0),
                            lda, -1.0, 1.0, 0, batch, stride, stride, stride);
      else
        e = launch_gemm_nt(s, EPI_STORE, n - t0, n - t0, pw, at(t0, K0), lda, at(t0, K0), lda,
                           at(t0, t0), lda, -1.0, 1.0, 0, 1, batch, stride, stride, stride);
      if (e != hipSuccess) return e;
    }
  }
  if (st) {  // diagnostic: accumulated phase cycles of workgroup 0 over all panels
    unsigned long long h[8];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_d128_stamps), sizeof(h));
    fprintf(stderr, "diag128 cycles: load %llu diag %llu panel %llu trail0 %llu lout %llu inv %llu "
                    "linvout %llu fac4 %llu\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
    const unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_d128_stamps), z, sizeof(h));
    unsigned long long w[12];
    (void)hipMemcpyFromSymbol(w, HIP_SYMBOL(g_sw_stamps), sizeof(w));
    fprintf(stderr, "sweep (sum over panels) own start %llu %llu %llu %llu  own end %llu %llu %llu %llu  "
                    "wave end %llu %llu %llu %llu\n", w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7],
            w[8], w[9], w[10], w[11]);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sw_stamps), z, sizeof(z));
    (void)hipMemcpyFromSymbol(w, HIP_SYMBOL(g_sw_step), 3 * sizeof(w[0]));
    fprintf(stderr, "owner steps of block 0 (sum): pivots %llu stores %llu tiles %llu\n", w[0], w[1], w[2]);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sw_step), z, 3 * sizeof(z[0]));
  }
  return hipGetLastError();
}

hipError_t launch_potrf_batched(hipStream_t s, int n, int batch, double *A, int64_t lda,
                                int64_t stride, int *info) {
  static const int p128 = [] {
    const char *e = getenv("GPMPC_POTRF128");
    return e ? atoi(e) : 1;
  }();
  // one workgroup per matrix (GPMPC_POTRF_PERSIST=1; read per call, tests switch
  // it).  Off by default: measured 3.67 ms per round of <= 256 matrices of
  // n = 1000 (20.8% of FP64 peak at batch 256) against 3.9 ms (28%) for the
  // launch-per-panel path -- one wave per SIMD (130 KB of LDS per workgroup)
  // leaves the MFMA tile loop's LDS and barrier latency exposed, and the
  // diagonal chain idles the CU.
  const char *pe = getenv("GPMPC_POTRF_PERSIST");
  const bool persist = pe && atoi(pe) > 0;
  if (p128 && persist) {
    static bool attr = hipFuncSetAttribute((const void *)k_potrf_persist,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)DIAG128_LDS) == hipSuccess;
    if (!attr) return hipErrorInvalidConfiguration;
    double *Lws = (double *)gpmpc_scratch(s, 2, sizeof(double) * DB * DB * (size_t)batch);
    if (!Lws) return hipErrorOutOfMemory;
    hipError_t e = hipMemsetAsync(info, 0, sizeof(int) * batch, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_potrf_persist, dim3(batch), dim3(256), DIAG128_LDS, s, n, A, lda, stride,
                       info, Lws);
    return hipGetLastError();
  }
  if (p128) {
    double *Linv = (double *)gpmpc_scratch(s, 2, sizeof(double) * DB * DB * (size_t)batch);
    if (!Linv) return hipErrorOutOfMemory;
    return launch_potrf_batched128(s, n, batch, A, lda, stride, info, Linv);
  }
  double *Linv = (double *)gpmpc_scratch(s, 1, sizeof(double) * NB * NB * (size_t)batch);
  if (!Linv) return hipErrorOutOfMemory;
  return launch_potrf_batched(s, n, batch, A, lda, stride, info, Linv);
}

// ---------------------------------------------------------------------------
// Triangular solves.  Inverses of the 32x32 diagonal blocks of L first, then
// one workgroup per 64-column panel of X walks the row blocks (forward for
// L X = B, backward for L^T X = B).
#define TB 128  // row block of the blocked TRSM

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

// X (n x nrhs, ld ldx) <- op(L)^-1 X ; op = L (trans=0) or L^T (trans=1), n <= TB.
// rhs_lower: X is known lower-triangular (X[r][c] = 0 for r < c, e.g. identity):
// the forward walk starts at the panel's first column.
// The workgroup's 64-column panel of X stays in LDS for the whole walk: each 32-row
// block is solved from the blocks solved before it (read from LDS, not re-read through
// the L2 after a store drain) and written to X once at the end.  Same operations in the
// same order as the block-by-block walk (same bits).
__global__ __launch_bounds__(256) void k_trsm_panel(int n, int nrhs, const double *L, int64_t ldl,
                                                    const double *Linv, double *X, int64_t ldx,
                                                    int trans, int rhs_lower) {
  // blockIdx.y: the TB x TB diagonal block solved (launch_tri_inverse solves all the
  // diagonal blocks of L^-1 side by side; every other launch has gridDim.y = 1, n <= TB)
  {
    const int bq = blockIdx.y;
    L += (int64_t)bq * TB * (ldl + 1);
    X += (int64_t)bq * TB * (ldx + 1);
    Linv += (int64_t)bq * (TB / NB) * NB * NB;
    n = min(TB, n - bq * TB);
    if (bq) nrhs = n;
  }
  const int c0 = blockIdx.x * 64;
  const int nblk = (n + NB - 1) / NB;
  __shared__ double sL[NB][TP];
  __shared__ double sXp[TB][64 + 1];
  const int tid = threadIdx.x;
  const int rr = tid >> 3;        // 0..31 row within block
  const int cc = (tid & 7) * 8;   // 8 columns
  for (int e = tid; e < TB * 64; e += 256) {
    const int i = e >> 6, j = e & 63, c = c0 + j;
    sXp[i][j] = (i < n && c < nrhs) ? X[(int64_t)i * ldx + c] : 0.0;
  }
  for (int step = 0; step < nblk; ++step) {
    const int ib = trans ? (nblk - 1 - step) : step;
    if (!trans && rhs_lower && (ib + 1) * NB <= c0) continue;
    const int r0 = ib * NB;
    const int nbi = min(NB, n - r0);
    __syncthreads();  // the previous block's rows (and the panel load) before they are read
    double acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = sXp[r0 + rr][cc + q];
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
      __syncthreads();
      for (int j = 0; j < NB; ++j) {
        const double l = sL[rr][j];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = fma(-l, sXp[k0 + j][cc + q], acc[q]);
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
    for (int q = 0; q < 8; ++q) sXp[r0 + rr][cc + q] = acc[q];  // rows past n: zeros times zero columns
    __syncthreads();
    double out[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) out[q] = 0.0;
    for (int j = 0; j < NB; ++j) {
      const double l = sL[rr][j];
#pragma unroll
      for (int q = 0; q < 8; ++q) out[q] = fma(l, sXp[r0 + j][cc + q], out[q]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) sXp[r0 + rr][cc + q] = rr < nbi ? out[q] : 0.0;
  }
  __syncthreads();
  for (int e = tid; e < TB * 64; e += 256) {
    const int i = e >> 6, j = e & 63, c = c0 + j;
    if (i < n && c < nrhs) X[(int64_t)i * ldx + c] = sXp[i][j];
  }
}

hipError_t launch_trsm_lower_ex(hipStream_t s, int n, int nrhs, const double *L, int64_t ldl,
                                double *X, int64_t ldx, int trans, int rhs_lower,
                                double *Linv_blocks /* may be null */) {
  const int nblk = (n + NB - 1) / NB;
  double *Linv = Linv_blocks;
  if (!Linv) Linv = (double *)gpmpc_scratch(s, 0, sizeof(double) * NB * NB * (size_t)nblk);
  if (!Linv) return hipErrorOutOfMemory;
  hipLaunchKernelGGL(k_tri_inv_blocks, dim3(nblk), dim3(64), 0, s, n, L, ldl, Linv);
  if (n <= TB) {
    hipLaunchKernelGGL(k_trsm_panel, dim3((nrhs + 63) / 64), dim3(256), 0, s, n, nrhs, L, ldl, Linv,
                       X, ldx, trans, rhs_lower);
    return hipGetLastError();
  }
  // blocked right-looking L X = B (FITC L_uu^-1 K_uf, W = L^-1, and the alpha
  // solves, whose few columns used to walk all of L on one CU): per 128-row block, the panel walk against the block's own
  // diagonal (32 x 32 inverses above), then X[r1:, :] -= L[r1:, r0:r1] X[r0:r1, :]
  // as one MFMA GEMM.  With a lower-triangular right-hand side (identity) the
  // block's rows are zero beyond column r1, so only r1 columns are touched.
  if (trans) {
    // L^T X = B from the bottom: X[r0:r1] = L_blk^-T X[r0:r1], then
    // X[:r0, :] -= L[r0:r1, :r0]^T X[r0:r1, :]  (A^T B form of the GEMM)
    for (int r0 = ((n - 1) / TB) * TB; r0 >= 0; r0 -= TB) {
      const int nb = std::min(TB, n - r0);
      hipLaunchKernelGGL(k_trsm_panel, dim3((nrhs + 63) / 64), dim3(256), 0, s, nb, nrhs,
                         L + (int64_t)r0 * ldl + r0, ldl, Linv + (int64_t)(r0 / NB) * NB * NB,
                         X + (int64_t)r0 * ldx, ldx, 1, 0);
      if (r0 > 0) {
        hipError_t e = launch_gemm_tn(s, r0, nrhs, nb, L + (int64_t)r0 * ldl, ldl,
                                      X + (int64_t)r0 * ldx, ldx, X, ldx, -1.0, 1.0);
        if (e != hipSuccess) return e;
      }
    }
    return hipGetLastError();
  }
  for (int r0 = 0; r0 < n; r0 += TB) {
    const int nb = std::min(TB, n - r0), r1 = r0 + nb;
    const int cols = rhs_lower ? std::min(nrhs, r1) : nrhs;
    hipLaunchKernelGGL(k_trsm_panel, dim3((cols + 63) / 64), dim3(256), 0, s, nb, cols,
                       L + (int64_t)r0 * ldl + r0, ldl, Linv + (int64_t)(r0 / NB) * NB * NB,
                       X + (int64_t)r0 * ldx, ldx, 0, 0);
    if (r1 < n) {
      hipError_t e = launch_gemm_nn(s, n - r1, cols, nb, L + (int64_t)r1 * ldl + r0, ldl,
                                    X + (int64_t)r0 * ldx, ldx, X + (int64_t)r1 * ldx, ldx, -1.0, 1.0);
      if (e != hipSuccess) return e;
    }
  }
  return hipGetLastError();
}

// W = L^-1 (W preset to the identity, ldw >= n): the TB x TB diagonal blocks of W by
// one k_trsm_panel launch over all of them (blockIdx.y = block), then by doubling,
// for each pair of solved blocks A (rows s0..s0+b) and C (the next <= b rows):
//   W_CA = -C^-1 (L_CA A^-1)     (two MFMA GEMMs, tmp >= b x b doubles)
// 8 serial panel launches of the blocked TRSM (~0.8 ms at n = 1000) become one panel
// launch and 2 log2(n / TB) levels of GEMMs.
hipError_t launch_tri_inverse(hipStream_t s, int n, const double *L, int64_t ldl, double *W,
                              int64_t ldw, double *tmp) {
  const int nblk = (n + NB - 1) / NB;
  double *Linv = (double *)gpmpc_scratch(s, 0, sizeof(double) * NB * NB * (size_t)nblk);
  if (!Linv) return hipErrorOutOfMemory;
  hipLaunchKernelGGL(k_tri_inv_blocks, dim3(nblk), dim3(64), 0, s, n, L, ldl, Linv);
  const int nd = (n + TB - 1) / TB;
  hipLaunchKernelGGL(k_trsm_panel, dim3((std::min(n, TB) + 63) / 64, nd), dim3(256), 0, s, n,
                     std::min(n, TB), L, ldl, Linv, W, ldw, 0, 1);
  for (int b = TB; b < n; b *= 2) {
    // the pairs of a level whose C block is full (mc = b) are one batched launch per
    // GEMM (their operands sit (2b)(ld + 1) apart on the diagonal); a ragged last pair
    // goes alone
    const int full = (n / (2 * b)) > 0 ? ((n - b) / (2 * b) + 1) : 0;   // pairs with s0 + b < n
    int nf = 0;
    while (nf < full && (nf * 2 * b) + 2 * b <= n) ++nf;
    if (nf > 0) {
      const int64_t dL = (int64_t)2 * b * (ldl + 1), dW = (int64_t)2 * b * (ldw + 1), dT = (int64_t)b * b;
      hipError_t e = launch_gemm_nn_batched(s, b, b, b, L + (int64_t)b * ldl, ldl, dL, W, ldw, dW, tmp, b, dT,
                                            1.0, 0.0, nf);
      if (e != hipSuccess) return e;
      e = launch_gemm_nn_batched(s, b, b, b, W + (int64_t)b * ldw + b, ldw, dW, tmp, b, dT, W + (int64_t)b * ldw,
                                 ldw, dW, -1.0, 0.0, nf);
      if (e != hipSuccess) return e;
    }
    for (int s0 = nf * 2 * b; s0 + b < n; s0 += 2 * b) {
      const int c0 = s0 + b, mc = std::min(n, s0 + 2 * b) - c0;
      hipError_t e = launch_gemm_nn(s, mc, b, b, L + (int64_t)c0 * ldl + s0, ldl,
                                    W + (int64_t)s0 * ldw + s0, ldw, tmp, b, 1.0, 0.0);
      if (e != hipSuccess) return e;
      e = launch_gemm_nn(s, mc, b, mc, W + (int64_t)c0 * ldw + c0, ldw, tmp, b,
                         W + (int64_t)c0 * ldw + s0, ldw, -1.0, 0.0);
      if (e != hipSuccess) return e;
    }
  }
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
  GPMPC_HIP(dA.alloc(s, sizeof(double) * (size_t)n * n));
  GPMPC_HIP(dinfo.alloc(s, sizeof(int)));
  GPMPC_HIP(hipMemcpy2DAsync(dA.p, sizeof(double) * n, A, sizeof(double) * lda,
                             sizeof(double) * n, n, hipMemcpyHostToDevice, s));
  GPMPC_HIP(launch_potrf_batched(s, n, 1, dA.as<double>(), n, 0, dinfo.as<int>()));
  GPMPC_HIP(hipMemcpyAsync(info, dinfo.p, sizeof(int), hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipMemcpy2DAsync(A, sizeof(double) * lda, dA.p, sizeof(double) * n,
                             sizeof(double) * n, n, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  if (*info < 0) return gpmpc_potrf_info_error(*info, "potrf");
  return *info > 0 ? *info : 0;
}

// info > 0: the 1-based column of the first non-positive pivot (the reference's
// LinAlgError); info < 0: the diagonal kernel's sweep timed out -- an error of this
// library, reported as such and never as a pivot column
int gpmpc_potrf_info_error(int info, const char *what) {
  if (info < 0) {
    gpmpc_set_error("%s: Cholesky diagonal-factor sweep timed out (internal invariant broken, "
                    "factor unreliable)", what);
    return -1;
  }
  gpmpc_set_error("Matrix is not positive definite (%s, column %d)", what, info);
  return info;
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
  GPMPC_HIP(dL.alloc(s, sizeof(double) * (size_t)n * n));
  GPMPC_HIP(dB.alloc(s, sizeof(double) * (size_t)n * nrhs));
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

// C (n x n, lower) = alpha A A^T + beta C for batch matrices (device pointers):
// the trailing update of the blocked Cholesky as a standalone entry point.
extern "C" int gpmpc_syrk_batched_dev(gpmpc_ctx *ctx, int n, int k, int batch, const double *dA,
                                      int lda, int64_t strideA, double *dC, int ldc,
                                      int64_t strideC, double alpha, double beta) {
  GPMPC_CHECK_ARG(ctx && dA && dC && n >= 0 && k >= 0 && batch >= 1 && lda >= k && ldc >= n);
  GPMPC_HIP(launch_gemm_nt(ctx->stream, EPI_STORE, n, n, k, dA, lda, dA, lda, dC, ldc, alpha, beta,
                           0, 1, batch, strideA, strideA, strideC));
  return 0;
}
