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
// tri_rows >= 0: rows r < tri_rows of A are lower triangular (A[r][k] = 0 for
// k > r; 0: none is) and rows >= M are padding, so a 16-row MFMA block whose rows
// are all above the step's k, or all padding, multiplies exact zeros: it is
// skipped (the diagonal K block of a triangular row tile, the padded last tile).
// lower_out: only the lower triangle of the output is used, so a diagonal tile's
// blocks wholly above the diagonal are skipped.  Same bits.
// IL: wave w's four 16-row blocks interleaved with its partner's (rows 16 (w/2 + 2x),
// mma128_row) instead of a contiguous 64-row half, so the two row halves of a
// triangular tile carry the same mix of early- and late-dying blocks
__device__ __forceinline__ int mma128_row(int wave, int x, bool il) {
  return il ? 16 * ((wave >> 1) + 2 * x) : (wave >> 1) * 64 + 16 * x;
}

// ILC: the same interleave for the two column halves (columns 16 (w%2 + 2y),
// mma128_col), so a triangular B's dying column blocks are shared evenly (tri_b only)
__device__ __forceinline__ int mma128_col(int wave, int y, bool ilc) {
  return ilc ? 16 * ((wave & 1) + 2 * y) : (wave & 1) * 64 + 16 * y;
}

// L2A / L2B: the A / B operand is read with agent-scope loads (global_load sc1: round the
// vector L1), for an operand this workgroup has just written (the fused potrf steps).
// tri_b: B is lower triangular over the tile's columns (B[c0 + j][k] = 0 for k > c0 + j,
// the potrf's L_cc^-1), so a wave's 16-column MFMA block y dies once k is past its last row.
// Ci: the accumulators start from the tile of Ci (rows r0.., columns c0.., ldci) instead of
// zero; with NEGA (A staged negated) the tile computes Ci - A B^T.
#ifndef MMA_V2
#define MMA_V2 1
#endif
#ifndef MMA_V2_ALL
#define MMA_V2_ALL 1  // also the agent-scope (L2A / L2B) and column-interleaved (ILC) tiles
#endif

// whether mma128_tile takes the LDS-DMA loop
template <bool L2A, bool L2B, bool ILC, bool NEGA, bool DMA>
constexpr bool mma128_dma() { return MMA_V2 && DMA && (MMA_V2_ALL || (!L2A && !L2B && !ILC)); }

// The slot swizzle of row r: (r >> 1) & 5.  Over a lane group the even rows split into
// {0, 2, 12, 14} (k quad q) and {4, 6, 8, 10} (quad q ^ 1), likewise the odd rows; each set
// takes the swizzles {0, 1, 4, 5} and the other quad's chunk differs by 2, which maps them
// onto {2, 3, 6, 7}.  ((r >> 1) & 7, the consecutive-16-lane design, put the two quads on
// the same slots: every read 2-way conflicted, SQ_LDS_BANK_CONFLICT 0.49 of the LDS cycles.)
__device__ __forceinline__ int mma128_swz(int r) { return (r >> 1) & 5; }

// A zero 16-byte chunk: the LDS-DMA source of a tile's padding rows.
static __device__ __attribute__((aligned(16))) double g_mma_zero[2] = {0.0, 0.0};

// mma128_tile's loop with LDS-DMA staging (global_load_lds_dwordx4, no staging registers,
// no ds_write pass) and 16-byte fragment reads.  An operand's K step is 128 rows x 16
// doubles, 128 B a row, unpadded (one DMA wave-instruction fills 8 whole rows); the row's
// 16-byte chunk c (k = 2c, 2c + 1) sits in slot c ^ mma128_swz(r), so each of ds_read_b128's
// four lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32: lanes of two
// different k quads) hits 16 distinct (r & 1, slot) bank groups: conflict-free.
// The swizzle is applied on the DMA's per-lane global source address.  Substep q of a
// K step reads k = 4 (lane >> 4) + q (A and B alike), so one ds_read_b128 serves two
// substeps and a lane's four k's are two reads.  The step with a partial K slice (k_hi
// not a multiple of GK) and operands without 16-byte alignment are staged through
// registers in the same layout, zero filled.  NEGA: the A fragments are negated as they
// are read (fma(-a, b, c): the bits of staging -A).  Same tile semantics as mma128_tile; the
// sums run in another k order (not the same bits as the register-staged loop).
template <bool IL, bool ILC, bool NEGA, bool L2A, bool L2B>
__device__ __forceinline__ void mma128_tile_v2(const double *__restrict__ A, int64_t lda,
                                               const double *__restrict__ B, int64_t ldb, int M, int N,
                                               int r0, int c0, int k_lo, int k_hi, double *sA, double *sB,
                                               d4_t (&acc)[4][4], int tri_rows, bool lower_out, bool tri_b,
                                               const double *Ci, int64_t ldci) {
  constexpr int TS = BT * GK;  // doubles of one operand tile: two per operand fit the caller's sA / sB
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if (Ci) {
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + mma128_row(wave, x, IL) + mf_row(lane, r);
          const int col = c0 + mma128_col(wave, y, ILC) + mf_col(lane);
          acc[x][y][r] = (row < M && col < N) ? Ci[(int64_t)row * ldci + col] : 0.0;
        }
  } else {
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = (d4_t){0.0, 0.0, 0.0, 0.0};
  }
  const bool vec = ((lda | ldb) & 1) == 0 && ((((uintptr_t)A) | ((uintptr_t)B)) & 15) == 0;
  // staging map: instruction j of this wave fills tile row (4 wave + j) * 8 + lane / 8,
  // slot lane % 8, with the row's chunk (lane % 8) ^ mma128_swz(row)
  const int rs = (4 * wave) * 8 + (lane >> 3);
  auto st_row = [&](int j) { return rs + 8 * j; };
  auto st_chunk = [&](int j) { return (lane & 7) ^ mma128_swz(st_row(j)); };
  // The DMA is issued from inline asm: the compiler does not see it as an LDS write, so it
  // adds no wait before the fragment reads of the other buffer (which it cannot tell apart
  // from the DMA's); every step ends on an explicit vmcnt(0) + barrier instead.
  // (sc1: the agent-scope form of L2A / L2B, past the vector L1 that this workgroup's own
  // stores do not refresh)
  auto dma = [](const double *g, const double *l, bool sc1) {
    const uint32_t lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)l;
    int keep;
    if (sc1)
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\t"
                   "s_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds))
                   : "memory");
    else
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                   "s_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds))
                   : "memory");
  };
  auto stage = [&](int buf, int k0) {
    double *LA = sA + buf * TS, *LB = sB + buf * TS;
    if (vec && k0 + GK <= k_hi) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = st_row(j), c = st_chunk(j);
        const double *sa = r0 + r < M ? A + (int64_t)(r0 + r) * lda + k0 + 2 * c : g_mma_zero;
        const double *sb = c0 + r < N ? B + (int64_t)(c0 + r) * ldb + k0 + 2 * c : g_mma_zero;
        dma(sa, LA + (4 * wave + j) * 128, L2A);  // this instruction's 1 KB (wave-uniform)
        dma(sb, LB + (4 * wave + j) * 128, L2B);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = st_row(j), k = k0 + 2 * st_chunk(j);
        const bool ra = r0 + r < M, rb = c0 + r < N;
        const double *pa = A + (int64_t)(ra ? r0 + r : 0) * lda;
        const double *pb = B + (int64_t)(rb ? c0 + r : 0) * ldb;
        auto ld = [](const double *p, bool agent) {
          return agent ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
        };
        const double a0 = ra && k < k_hi ? ld(pa + k, L2A) : 0.0, a1 = ra && k + 1 < k_hi ? ld(pa + k + 1, L2A) : 0.0;
        const double b0 = rb && k < k_hi ? ld(pb + k, L2B) : 0.0, b1 = rb && k + 1 < k_hi ? ld(pb + k + 1, L2B) : 0.0;
        *(double2 *)(LA + (4 * wave + j) * 128 + 2 * lane) = make_double2(a0, a1);
        *(double2 *)(LB + (4 * wave + j) * 128 + 2 * lane) = make_double2(b0, b1);
      }
    }
  };
  // fragment reads: row R = (16-aligned block row) + lane % 16, so mma128_swz(R) = mma128_swz(lane % 16)
  const int sw = mma128_swz(lane & 15);
  const int foff0 = (lane & 15) * 16 + 2 * ((2 * (lane >> 4)) ^ sw);      // k = 4 (lane >> 4) + {0, 1}
  const int foff1 = (lane & 15) * 16 + 2 * ((2 * (lane >> 4) + 1) ^ sw);  // k = 4 (lane >> 4) + {2, 3}
  stage(0, k_lo);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int cur = 0;
  const int R0 = r0 + mma128_row(wave, 0, IL), R1 = r0 + mma128_row(wave, 1, IL);
  const int R2 = r0 + mma128_row(wave, 2, IL), R3 = r0 + mma128_row(wave, 3, IL);
  int k0 = k_lo;
#define MMA2_PHASE_M(MASK, KEND)                                                              \
  for (const int ke_ = (KEND); k0 < ke_; k0 += GK) {                                          \
    if (k0 + GK < k_hi) stage(cur ^ 1, k0 + GK);                                              \
    const double *la = sA + cur * TS, *lb = sB + cur * TS;                                    \
    double2 fa[2][4], fb[2][4];                                                               \
    _Pragma("unroll") for (int x = 0; x < 4; ++x) if (((MASK) >> (4 * x)) & 15) {             \
      fa[0][x] = *(const double2 *)(la + mma128_row(wave, x, IL) * 16 + foff0);               \
      fa[1][x] = *(const double2 *)(la + mma128_row(wave, x, IL) * 16 + foff1);               \
      if (NEGA) {                                                                             \
        fa[0][x].x = -fa[0][x].x; fa[0][x].y = -fa[0][x].y;                                   \
        fa[1][x].x = -fa[1][x].x; fa[1][x].y = -fa[1][x].y;                                   \
      }                                                                                       \
    }                                                                                         \
    _Pragma("unroll") for (int y = 0; y < 4; ++y) {                                           \
      fb[0][y] = *(const double2 *)(lb + mma128_col(wave, y, ILC) * 16 + foff0);              \
      fb[1][y] = *(const double2 *)(lb + mma128_col(wave, y, ILC) * 16 + foff1);              \
    }                                                                                         \
    _Pragma("unroll") for (int q = 0; q < 4; ++q)                                             \
      _Pragma("unroll") for (int x = 0; x < 4; ++x)                                           \
        _Pragma("unroll") for (int y = 0; y < 4; ++y)                                         \
          if (((MASK) >> (4 * x + y)) & 1) {                                                  \
            const double av = (q & 1) ? fa[q >> 1][x].y : fa[q >> 1][x].x;                    \
            const double bv = (q & 1) ? fb[q >> 1][y].y : fb[q >> 1][y].x;                    \
            acc[x][y] = mfma_f64(av, bv, acc[x][y]);                                          \
          }                                                                                   \
    __builtin_amdgcn_sched_barrier(0); /* the DMA wait and the barrier stay behind the MFMAs */ \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                          \
    __syncthreads();                                                                          \
    cur ^= 1;                                                                                 \
  }
#define MMA2_PHASE(XF, XL, KEND) MMA2_PHASE_M(((0xFFFF << (4 * (XF))) & (0xFFFF >> (4 * (4 - (XL))))), KEND)
  if (tri_b) {
    MMA2_PHASE_M(0xFFFF, min(k_hi, c0 + mma128_col(wave, 0, ILC) + 16))
    MMA2_PHASE_M(0xEEEE, min(k_hi, c0 + mma128_col(wave, 1, ILC) + 16))
    MMA2_PHASE_M(0xCCCC, min(k_hi, c0 + mma128_col(wave, 2, ILC) + 16))
    MMA2_PHASE_M(0x8888, min(k_hi, c0 + mma128_col(wave, 3, ILC) + 16))
  } else if (lower_out && r0 == c0) {
    const int wi = wave >> 1, wj = wave & 1;
    if (IL) {
      if (wj == 0 && wi == 0) { MMA2_PHASE_M(0xFF71, k_hi) }
      else if (wj == 0) { MMA2_PHASE_M(0xFFF3, k_hi) }
      else if (wi == 0) { MMA2_PHASE_M(0x7100, k_hi) }
      else { MMA2_PHASE_M(0xF300, k_hi) }
    } else {
      if (wi == wj) { MMA2_PHASE_M(0xF731, k_hi) }
      else if (wi == 1) { MMA2_PHASE_M(0xFFFF, k_hi) }
    }
  } else if (tri_rows >= 0 && R3 + 15 < tri_rows) {
    MMA2_PHASE(0, 4, min(k_hi, R0 + 16))
    MMA2_PHASE(1, 4, min(k_hi, R1 + 16))
    MMA2_PHASE(2, 4, min(k_hi, R2 + 16))
    MMA2_PHASE(3, 4, min(k_hi, R3 + 16))
  } else if (tri_rows < 0 || R3 < M) {
    MMA2_PHASE(0, 4, k_hi)
  } else if (R2 < M) {
    MMA2_PHASE(0, 3, k_hi)
  } else if (R1 < M) {
    MMA2_PHASE(0, 2, k_hi)
  } else if (R0 < M) {
    MMA2_PHASE(0, 1, k_hi)
  }
#undef MMA2_PHASE
#undef MMA2_PHASE_M
  for (; k0 < k_hi; k0 += GK) {  // dead steps: staging only
    if (k0 + GK < k_hi) stage(cur ^ 1, k0 + GK);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    cur ^= 1;
  }
}

// DMA: the LDS-DMA loop (mma128_tile_v2, in the caller's sA / sB) where the flags allow
// it; false keeps the register-staged loop
template <bool IL = false, bool L2A = false, bool L2B = false, bool ILC = false, bool NEGA = false,
          bool DMA = true>
__device__ __forceinline__ void mma128_tile(const double *__restrict__ A, int64_t lda,
                                            const double *__restrict__ B, int64_t ldb, int M, int N,
                                            int r0, int c0, int k_lo, int k_hi,
                                            double (*sA)[BT][GP], double (*sB)[BT][GP],
                                            d4_t (&acc)[4][4], int tri_rows = -1, bool lower_out = false,
                                            bool tri_b = false, const double *Ci = nullptr, int64_t ldci = 0) {
  if constexpr (mma128_dma<L2A, L2B, ILC, NEGA, DMA>()) {
    mma128_tile_v2<IL, ILC, NEGA, L2A, L2B>(A, lda, B, ldb, M, N, r0, c0, k_lo, k_hi, &sA[0][0][0], &sB[0][0][0], acc,
                                  tri_rows, lower_out, tri_b, Ci, ldci);
    return;
  }
  // the wave index through readfirstlane: the compiler then knows every per-wave
  // quantity (and the triangular skips below) is uniform
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if (Ci) {
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + mma128_row(wave, x, IL) + mf_row(lane, r);
          const int col = c0 + mma128_col(wave, y, ILC) + mf_col(lane);
          acc[x][y][r] = (row < M && col < N) ? Ci[(int64_t)row * ldci + col] : 0.0;
        }
  } else {
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = (d4_t){0.0, 0.0, 0.0, 0.0};
  }
  const int lr = tid >> 1, lk = (tid & 1) * 8;
  const bool ra = r0 + lr < M, rb = c0 + lr < N;
  const double *pa = A + (int64_t)(ra ? r0 + lr : 0) * lda;
  const double *pb = B + (int64_t)(rb ? c0 + lr : 0) * ldb;
  const bool vec = ((lda | ldb) & 1) == 0 && ((((uintptr_t)A) | ((uintptr_t)B)) & 15) == 0;
  double va[8], vb[8];
  // agent-scope 16-byte loads: raw buffer loads with the sc1 policy bit (aux 16 on gfx950),
  // whose completion the compiler tracks like any load; byte offsets must fit 31 bits
  const bool buf = (L2A || L2B) && vec && (int64_t)(max(r0, c0) + BT) * max(lda, ldb) * 8 < 0x7fffffff;
  // the operand's element (row, k) through an agent-scope 16-byte raw buffer load (sc1: aux 16
  // on gfx950), whose completion the compiler tracks like any load's
  auto ld_agent = [](const double *base, int64_t ld, int row, int k, double &x, double &y) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 0x7fffffff, 0x00020000);
    const double2 v = __builtin_bit_cast(
        double2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(row * ld + k) * 8, 0, 16));
    x = v.x; y = v.y;
  };
  auto gload = [&](int k0) {
    const int k = k0 + lk;
    if ((L2A || L2B) && buf && k + 7 < k_hi) {
#pragma unroll
      for (int q = 0; q < 8; q += 2) {
        if (!ra) { va[q] = 0.0; va[q + 1] = 0.0; }
        else if (L2A) ld_agent(A, lda, r0 + lr, k + q, va[q], va[q + 1]);
        else { const double2 v = *(const double2 *)(pa + k + q); va[q] = v.x; va[q + 1] = v.y; }
        if (!rb) { vb[q] = 0.0; vb[q + 1] = 0.0; }
        else if (L2B) ld_agent(B, ldb, c0 + lr, k + q, vb[q], vb[q + 1]);
        else { const double2 v = *(const double2 *)(pb + k + q); vb[q] = v.x; vb[q + 1] = v.y; }
      }
    } else if (L2A || L2B) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const bool ka = ra && k + q < k_hi, kb = rb && k + q < k_hi;
        va[q] = !ka ? 0.0 : L2A ? __hip_atomic_load(pa + k + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : pa[k + q];
        vb[q] = !kb ? 0.0 : L2B ? __hip_atomic_load(pb + k + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : pb[k + q];
      }
    } else if (vec && k + 7 < k_hi) {
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
      sA[buf][lr][lk + q] = NEGA ? -va[q] : va[q];
      sB[buf][lr][lk + q] = vb[q];
    }
  };
  gload(k_lo);
  lstore(0);
  __syncthreads();
  int cur = 0;
  // Skipped MFMA blocks (tri_rows >= 0).  A 16-row block x of this wave (rows
  // R_x = r0 + mma128_row(x), increasing in x) multiplies exact zeros from the K step
  // on whose first k is past R_x + 15 when all its rows are triangular, and always
  // when all are padding.  The live blocks of a step are then a range [XF, XL); each
  // range runs as a loop of its own over the steps it covers (a branch around the
  // MFMAs, even a uniform one, made the compiler spill the accumulators), and every
  // wave takes every step's barrier.
  const int R0 = r0 + mma128_row(wave, 0, IL), R1 = r0 + mma128_row(wave, 1, IL);
  const int R2 = r0 + mma128_row(wave, 2, IL), R3 = r0 + mma128_row(wave, 3, IL);
  int k0 = k_lo;
// MFMA block (x, y) runs when bit 4 x + y of MASK is set (a literal: the unrolled
// loops fold the tests away)
#define MMA_PHASE_M(MASK, KEND)                                                          \
  for (const int ke_ = (KEND); k0 < ke_; k0 += GK) {                                     \
    const bool more = k0 + GK < k_hi;                                                    \
    if (more) gload(k0 + GK);                                                            \
    _Pragma("unroll") for (int kk = 0; kk < GK; kk += 4) {                               \
      const int kc = kk + (lane >> 4);                                                   \
      double a[4], b[4];                                                                 \
      _Pragma("unroll") for (int x = 0; x < 4; ++x)                                      \
        if (((MASK) >> (4 * x)) & 15) a[x] = sA[cur][mma128_row(wave, x, IL) + (lane & 15)][kc]; \
      _Pragma("unroll") for (int y = 0; y < 4; ++y) b[y] = sB[cur][mma128_col(wave, y, ILC) + (lane & 15)][kc]; \
      _Pragma("unroll") for (int x = 0; x < 4; ++x)                                      \
        _Pragma("unroll") for (int y = 0; y < 4; ++y)                                    \
          if (((MASK) >> (4 * x + y)) & 1) acc[x][y] = mfma_f64(a[x], b[y], acc[x][y]);  \
    }                                                                                    \
    if (more) lstore(cur ^ 1);                                                           \
    __syncthreads();                                                                     \
    cur ^= 1;                                                                            \
  }
#define MMA_PHASE(XF, XL, KEND) MMA_PHASE_M(((0xFFFF << (4 * (XF))) & (0xFFFF >> (4 * (4 - (XL))))), KEND)
  if (tri_b) {
    // column blocks y of this wave (B rows c0 + mma128_col(y)) die one by one: live
    // blocks of a step are y >= YF (mask bits 4 x + y)
    MMA_PHASE_M(0xFFFF, min(k_hi, c0 + mma128_col(wave, 0, ILC) + 16))
    MMA_PHASE_M(0xEEEE, min(k_hi, c0 + mma128_col(wave, 1, ILC) + 16))
    MMA_PHASE_M(0xCCCC, min(k_hi, c0 + mma128_col(wave, 2, ILC) + 16))
    MMA_PHASE_M(0x8888, min(k_hi, c0 + mma128_col(wave, 3, ILC) + 16))
  } else if (lower_out && r0 == c0) {
    // a diagonal tile of a lower-triangular output: the blocks wholly above the
    // diagonal are never stored, so they are not computed (the live pattern of
    // wave (w/2, w%2) for its row mapping; one wave of the contiguous mapping has none)
    const int wi = wave >> 1, wj = wave & 1;
    if (IL) {
      if (wj == 0 && wi == 0) { MMA_PHASE_M(0xFF71, k_hi) }
      else if (wj == 0) { MMA_PHASE_M(0xFFF3, k_hi) }
      else if (wi == 0) { MMA_PHASE_M(0x7100, k_hi) }
      else { MMA_PHASE_M(0xF300, k_hi) }
    } else {
      if (wi == wj) { MMA_PHASE_M(0xF731, k_hi) }
      else if (wi == 1) { MMA_PHASE_M(0xFFFF, k_hi) }
    }
  } else if (tri_rows >= 0 && R3 + 15 < tri_rows) {  // all rows triangular: blocks die one by one
    MMA_PHASE(0, 4, min(k_hi, R0 + 16))
    MMA_PHASE(1, 4, min(k_hi, R1 + 16))
    MMA_PHASE(2, 4, min(k_hi, R2 + 16))
    MMA_PHASE(3, 4, min(k_hi, R3 + 16))
  } else if (tri_rows < 0 || R3 < M) {
    MMA_PHASE(0, 4, k_hi)
  } else if (R2 < M) {  // padding rows (>= M) from block 3, 2 or 1 on
    MMA_PHASE(0, 3, k_hi)
  } else if (R1 < M) {
    MMA_PHASE(0, 2, k_hi)
  } else if (R0 < M) {
    MMA_PHASE(0, 1, k_hi)
  }
#undef MMA_PHASE
#undef MMA_PHASE_M
  for (; k0 < k_hi; k0 += GK) {  // dead steps: staging only
    const bool more = k0 + GK < k_hi;
    if (more) {
      gload(k0 + GK);
      lstore(cur ^ 1);
    }
    __syncthreads();
    cur ^= 1;
  }
}

