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
#include <algorithm>
#include <cstdlib>
#include "internal.h"
#include "mfma64.h"
#include "gemm.h"

#define GT 64
#define GK 16
#define GP 18
static_assert(GK * (GT + 2) <= GT * GP, "k-major B tile must fit the row-major B buffer");

// lower-triangular tile t -> (row tile ti, col tile tj), tj <= ti
__device__ __forceinline__ void tri_tile(int t, int &ti, int &tj) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  ti = i;
  tj = t - i * (i + 1) / 2;
}

// BKN = 1: B is K x N row-major (C = alpha A B + beta C, the "NN" form); its
// tile is staged k-major (sBk[k][col]) so the MFMA fragment read stays
// contiguous.  Used by the blocked TRSM's trailing updates.
// AKM = 1: A is K x M row-major (C = alpha A^T B + ...), staged k-major the same way.
template <int EPI, int BKN = 0, int AKM = 0>
__global__ __launch_bounds__(256) void k_gemm_nt(int M, int N, int K, const double *__restrict__ A,
                                                 int64_t lda, const double *__restrict__ B,
                                                 int64_t ldb, double *__restrict__ C, int64_t ldc,
                                                 double alpha, double beta, int tri_a,
                                                 int lower_c, int64_t sA_, int64_t sB_,
                                                 int64_t sC_, int msum, double *__restrict__ Cm,
                                                 int64_t ldm, int remap_ty, int xcd_batch, int klast) {
  int bz = blockIdx.z;
  // klast > 0: the batch is the K chunks of a split product (launch_splitk): the last
  // chunk is klast long instead of K
  if (klast > 0 && !xcd_batch && (int)blockIdx.z == (int)gridDim.z - 1) K = klast;
  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd_batch) {
    // lower-triangular batch, one matrix per XCD at a time: workgroup i runs
    // on XCD i % 8, so matrix b's tiles all land on XCD b % 8 and its row and
    // column panels are re-read from that XCD's L2 instead of crossing all 8
    const int T = ((M + GT - 1) / GT) * ((M + GT - 1) / GT + 1) / 2;
    const int i = blockIdx.x, slot = i >> 3;
    bz = (i & 7) + 8 * (slot / T);
    if (bz >= xcd_batch) return;
    tri_tile(slot % T, by, bx);
  }
  A += bz * sA_;
  B += bz * sB_;
  C += bz * sC_;
  // optional XCD-aware order (1-D grid, GPMPC_GEMM_REMAP=1): workgroup i runs
  // on XCD i % 8; each XCD gets whole column blocks and walks their row tiles
  // back to back.  Off by default: for the posterior GEMM the plain order
  // (concurrent workgroups share a W row block, K* streams from the 256 MB
  // Infinity Cache) measured 0.46 ms vs 0.54 ms with the remap.
  if (xcd_batch) {
  } else if (remap_ty > 0) {
    const int i = blockIdx.x, slot = i >> 3;
    bx = (i & 7) + 8 * (slot / remap_ty);
    by = slot % remap_ty;
  } else if (remap_ty < 0) {  // 1-D grid over the lower-triangular tiles only
    tri_tile(blockIdx.x, by, bx);
  }
  const int r0 = by * GT, c0 = bx * GT;
  if (lower_c && c0 > r0 + GT - 1) return;
  __shared__ double sA[2][GT][GP];
  __shared__ double sB[2][GT][GP];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int qi = (wave >> 1) * 32, qj = (wave & 1) * 32;
  int kend = K;
  if (tri_a) kend = min(K, r0 + GT);
  d4_t acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = (d4_t){0.0, 0.0, 0.0, 0.0};
  // beta != 0: C is loaded here, before the K loop, so that its latency hides under
  // the loop instead of following it (the K = 128 Cholesky updates spent much of
  // their epilogue waiting for it); the epilogue arithmetic is unchanged
  const bool prec = EPI == EPI_STORE && beta != 0.0;
  d4_t cpre[2][2];
  if (prec) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + qi + x * 16 + mf_row(lane, r);
          const int col = c0 + qj + y * 16 + mf_col(lane);
          cpre[x][y][r] = (row < M && col < N && (!lower_c || col <= row)) ? C[(int64_t)row * ldc + col] : 0.0;
        }
  }
  // each thread moves 4 consecutive k of one row of A and of B per K-step:
  // row = tid/4, k = (tid%4)*4..+3.  The next step's operands are loaded into
  // registers while the current step's MFMAs run (LDS double buffer, one
  // barrier per K-step); rows are read as two 16-byte loads when aligned.
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  // BKN: thread loads k-row kb = tid/16 of B, columns c0 + (tid%16)*4 .. +3
  const int kb = tid >> 4, cb = (tid & 15) * 4;
  double (*sBk)[GK][GT + 2] = reinterpret_cast<double (*)[GK][GT + 2]>(&sB[0][0][0]);
  double (*sAk)[GK][GT + 2] = reinterpret_cast<double (*)[GK][GT + 2]>(&sA[0][0][0]);
  const bool ra = AKM ? true : r0 + lr < M, rb = BKN ? true : c0 + lr < N;
  const double *pa = AKM ? A + r0 + cb : A + (int64_t)(ra ? r0 + lr : 0) * lda;
  const bool veca = AKM ? (((lda | ldb) & 1) == 0 && ((((uintptr_t)A) | ((uintptr_t)B)) & 15) == 0 &&
                           r0 + cb + 3 < M)
                        : false;
  const double *pb = BKN ? B + c0 + cb : B + (int64_t)(rb ? c0 + lr : 0) * ldb;
  const bool vec = ((lda | ldb) & 1) == 0 && ((((uintptr_t)A) | ((uintptr_t)B)) & 15) == 0;
  const bool vecb = BKN ? (vec && c0 + cb + 3 < N) : vec;
  double va[4], vb[4];
  auto gload = [&](int k0) {
    const int k = k0 + lk;
    if (AKM) {
      const int kr = k0 + kb;
      const double *p = pa + (int64_t)kr * lda;
      if (kr < kend && veca) {
        const double2 a01 = *(const double2 *)p, a23 = *(const double2 *)(p + 2);
        va[0] = a01.x; va[1] = a01.y; va[2] = a23.x; va[3] = a23.y;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) va[q] = (kr < kend && r0 + cb + q < M) ? p[q] : 0.0;
      }
    } else if (vec && k + 3 < kend) {
      const double2 a01 = ra ? *(const double2 *)(pa + k) : make_double2(0.0, 0.0);
      const double2 a23 = ra ? *(const double2 *)(pa + k + 2) : make_double2(0.0, 0.0);
      va[0] = a01.x; va[1] = a01.y; va[2] = a23.x; va[3] = a23.y;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) va[q] = (ra && k + q < kend) ? pa[k + q] : 0.0;
    }
    if (BKN) {
      const int kr = k0 + kb;
      const double *p = pb + (int64_t)kr * ldb;
      if (kr < kend && vecb) {
        const double2 b01 = *(const double2 *)p, b23 = *(const double2 *)(p + 2);
        vb[0] = b01.x; vb[1] = b01.y; vb[2] = b23.x; vb[3] = b23.y;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) vb[q] = (kr < kend && c0 + cb + q < N) ? p[q] : 0.0;
      }
    } else if (vec && k + 3 < kend) {
      const double2 b01 = rb ? *(const double2 *)(pb + k) : make_double2(0.0, 0.0);
      const double2 b23 = rb ? *(const double2 *)(pb + k + 2) : make_double2(0.0, 0.0);
      vb[0] = b01.x; vb[1] = b01.y; vb[2] = b23.x; vb[3] = b23.y;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) vb[q] = (rb && k + q < kend) ? pb[k + q] : 0.0;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (AKM) sAk[buf][kb][cb + q] = va[q];
      else sA[buf][lr][lk + q] = va[q];
      if (BKN) sBk[buf][kb][cb + q] = vb[q];
      else sB[buf][lr][lk + q] = vb[q];
    }
  };
  gload(0);
  lstore(0);
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < kend; k0 += GK) {
    const bool more = k0 + GK < kend;
    if (more) gload(k0 + GK);
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      const int kc = kk + (lane >> 4);
      const double a0 = AKM ? sAk[cur][kc][qi + (lane & 15)] : sA[cur][qi + (lane & 15)][kc];
      const double a1 = AKM ? sAk[cur][kc][qi + 16 + (lane & 15)] : sA[cur][qi + 16 + (lane & 15)][kc];
      const double b0 = BKN ? sBk[cur][kc][qj + (lane & 15)] : sB[cur][qj + (lane & 15)][kc];
      const double b1 = BKN ? sBk[cur][kc][qj + 16 + (lane & 15)] : sB[cur][qj + 16 + (lane & 15)][kc];
      acc[0][0] = mfma_f64(a0, b0, acc[0][0]);
      acc[0][1] = mfma_f64(a0, b1, acc[0][1]);
      acc[1][0] = mfma_f64(a1, b0, acc[1][0]);
      acc[1][1] = mfma_f64(a1, b1, acc[1][1]);
    }
    if (more) lstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
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
            *p = prec ? alpha * acc[x][y][r] + beta * cpre[x][y][r] : alpha * acc[x][y][r];
          }
        }
  } else {
    // sum of squares over rows < msum (rows >= M contribute exact zeros);
    // rows msum..M-1 (alpha^T appended to W) are stored to Cm: the mean
    __shared__ double red[4][32];
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + qi + x * 16 + mf_row(lane, r);
        if (row < msum) {
          s0 = fma(acc[x][0][r], acc[x][0][r], s0);
          s1 = fma(acc[x][1][r], acc[x][1][r], s1);
        } else if (row < M) {
          const int col0 = c0 + qj + mf_col(lane);
          if (col0 < N) Cm[(int64_t)(row - msum) * ldm + col0] = acc[x][0][r];
          if (col0 + 16 < N) Cm[(int64_t)(row - msum) * ldm + col0 + 16] = acc[x][1][r];
        }
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
      if (col < N) C[(int64_t)by * ldc + col] = v;
    }
  }
}

// GPMPC_POST_XCD=1: the posterior GEMM's column-grouped XCD mapping (k_gemm128, tri_grid 2)
static int post_xcd() {
  static const int v = [] {
    const char *e = getenv("GPMPC_POST_XCD");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// ---------------------------------------------------------------------------
// Large-tile variant: 128 x 128 per workgroup, each wave a 64 x 64 quadrant
// (4 x 4 MFMA blocks: 8 fragment reads feed 16 MFMAs), K staged 16 at a time,
// LDS double buffer + register prefetch, 16-byte global loads (two threads per
// 16-double row segment).  Row tiles are dispatched longest-first when A is
// triangular.  Used when both M and N are large (posterior GEMM, trailing SYRK).
#include "mma128.h"

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_gemm128(int M, int N, int K, const double *__restrict__ A,
                                                    int64_t lda, const double *__restrict__ B,
                                                    int64_t ldb, double *__restrict__ C, int64_t ldc,
                                                    double alpha, double beta, int tri_a, int lower_c,
                                                    int64_t sA_, int64_t sB_, int64_t sC_, int msum,
                                                    double *__restrict__ Cm, int64_t ldm, int ksplit,
                                                    int tri_grid) {
  // grid z = batch x ksplit: split s of a matrix covers K range [s*kc, (s+1)*kc)
  // and accumulates alpha*acc into C with fp64 atomics (beta must be 1 then)
  int bz = blockIdx.z / ksplit, sp = blockIdx.z % ksplit;
  int ry = blockIdx.y;
  if (tri_grid == 3) {
    // XCD-batched row blocks (launch_gemm_nt_rowblock, batch a multiple of 8):
    // workgroup L runs on XCD L % 8; its m-th workgroup there takes matrix
    // 8 (m / (ny ks)) + L % 8, so all row tiles and K splits of a matrix share
    // one XCD and its B panel (the potrf's row block / inverse) is read from
    // that XCD's L2 instead of once per row tile across all eight
    const int ny = gridDim.y, L = blockIdx.x + blockIdx.y * gridDim.x + blockIdx.z * gridDim.x * gridDim.y;
    const int m = L >> 3, per = ny * ksplit, rem = m % per;
    bz = (L & 7) + 8 * (m / per);
    sp = rem / ny;
    ry = rem % ny;
  }
  A += bz * sA_;
  B += bz * sB_;
  C += bz * sC_;
  int by = tri_a ? (int)gridDim.y - 1 - ry : ry, bx = tri_grid == 3 ? 0 : (int)blockIdx.x;
  if (tri_grid == 1) tri_tile(blockIdx.x, by, bx);  // 1-D grid over the lower-triangular tiles
  if (tri_grid == 2) {
    // column-grouped: workgroup L runs on XCD L % 8; its m-th workgroup there
    // takes column tile 8 (m / ny) + L % 8, row tile m % ny (longest first), so
    // the ny row tiles of one K* column tile run together on one XCD and share
    // its L2 (as do the W row tiles of the 8 column tiles in flight)
    const int ny = gridDim.y, L = blockIdx.y * gridDim.x + blockIdx.x, m = L >> 3;
    bx = (L & 7) + 8 * (m / ny);
    by = tri_a ? ny - 1 - m % ny : m % ny;
  }
  const int r0 = by * BT, c0 = bx * BT;
  if (lower_c && c0 > r0 + BT - 1) return;
  int kbeg = 0;
  if (ksplit > 1) {
    const int kc = ((K + ksplit - 1) / ksplit + GK - 1) / GK * GK;
    kbeg = sp * kc;
    if (kbeg >= K) return;
    A += kbeg;
    B += kbeg;
    K = min(K - kbeg, kc);
  }
  __shared__ double sA[2][BT][GP];
  __shared__ double sB[2][BT][GP];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int qi = (wave >> 1) * 64, qj = (wave & 1) * 64;
  int kend = K;
  if (tri_a) kend = min(K, r0 + BT);
  d4_t acc[4][4];
  // triangular rows: all of W for a store, the W rows above the alpha rows for SUMSQ,
  // none for a plain A (0: only its padding rows are skipped)
  const int tri_rows = ksplit > 1 ? -1 : (tri_a ? (EPI == EPI_SUMSQ ? msum : M) : 0);
  mma128_tile<true>(A, lda, B, ldb, M, N, r0, c0, 0, kend, sA, sB, acc, tri_rows, lower_c != 0);
  if (EPI == EPI_STORE) {
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + mma128_row(wave, x, true) + mf_row(lane, r);
          const int col = c0 + qj + y * 16 + mf_col(lane);
          if (row < M && col < N && (!lower_c || col <= row)) {
            double *p = C + (int64_t)row * ldc + col;
            if (ksplit > 1) atomicAdd(p, alpha * acc[x][y][r]);
            else *p = (beta == 0.0) ? alpha * acc[x][y][r] : alpha * acc[x][y][r] + beta * *p;
          }
        }
  } else {
    __shared__ double red[4][64];
    double sq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + mma128_row(wave, x, true) + mf_row(lane, r);
        if (row < msum) {
#pragma unroll
          for (int y = 0; y < 4; ++y) sq[y] = fma(acc[x][y][r], acc[x][y][r], sq[y]);
        } else if (row < M) {
#pragma unroll
          for (int y = 0; y < 4; ++y) {
            const int col = c0 + qj + y * 16 + mf_col(lane);
            if (col < N) Cm[(int64_t)(row - msum) * ldm + col] = acc[x][y][r];
          }
        }
      }
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      sq[y] += __shfl_xor(sq[y], 16);
      sq[y] += __shfl_xor(sq[y], 32);
    }
    if (lane < 16) {
#pragma unroll
      for (int y = 0; y < 4; ++y) red[wave][y * 16 + lane] = sq[y];
    }
    __syncthreads();
    if (tid < 128) {
      const int half = tid >> 6, cc = tid & 63;        // column half qj = half * 64
      const double v = red[half][cc] + red[2 + half][cc];  // waves (0, half) and (1, half)
      const int col = c0 + tid;
      if (col < N) C[(int64_t)by * ldc + col] = v;
    }
  }
}


// The potrf's diagonal-block update C -= A A^T (C the w x w lower diagonal block, A its rows'
// K left columns; one workgroup per matrix and K split).  Of the 8 x 8 16-wide MFMA blocks
// of a 128 x 128 lower triangle 36 are live; the 128-tile kernel's quadrant waves own 12,
// 14, 4 and 6 of them, so every K step waits for the 14.  Here wave w owns column blocks w
// and 7 - w down to the last row block: 9 blocks each (8 - w + w + 1), fed by the A
// fragments of row blocks w..7 and B = A's fragments of the two column blocks.  A and B
// are the same rows, so one LDS tile is staged.  ks > 1: split s covers K range
// [s kc, (s + 1) kc) and adds its partial product with fp64 atomics.
template <int W>
__device__ __forceinline__ void syrk_diag_wave(const double *__restrict__ A, int64_t lda, int w, int k_lo,
                                               int k_hi, double (*sA)[BT][GP], double *__restrict__ C,
                                               int64_t ldc, bool atomic) {
  constexpr int C1 = W, C2 = 7 - W, N1 = 8 - C1, N2 = 8 - C2;  // column blocks and their live rows
  const int tid = threadIdx.x, lane = tid & 63;
  d4_t a1[N1], a2[N2];
#pragma unroll
  for (int i = 0; i < N1; ++i) a1[i] = (d4_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int i = 0; i < N2; ++i) a2[i] = (d4_t){0.0, 0.0, 0.0, 0.0};
  const int lr = tid >> 1, lk = (tid & 1) * 8;
  const bool ra = lr < w;
  const double *pa = A + (int64_t)(ra ? lr : 0) * lda;
  const bool vec = (lda & 1) == 0 && (((uintptr_t)A) & 15) == 0;
  double va[8];
  auto gload = [&](int k0) {
    const int k = k0 + lk;
    if (vec && k + 7 < k_hi) {
#pragma unroll
      for (int q = 0; q < 8; q += 2) {
        const double2 v = ra ? *(const double2 *)(pa + k + q) : make_double2(0.0, 0.0);
        va[q] = v.x; va[q + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) va[q] = (ra && k + q < k_hi) ? pa[k + q] : 0.0;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) sA[buf][lr][lk + q] = va[q];
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
      double fa[8];
#pragma unroll
      for (int r = C1; r < 8; ++r) fa[r] = sA[cur][16 * r + (lane & 15)][kc];
      const double b1 = fa[C1], b2 = fa[C2];  // B = A: the column blocks' own fragments
#pragma unroll
      for (int r = C1; r < 8; ++r) a1[r - C1] = mfma_f64(fa[r], b1, a1[r - C1]);
#pragma unroll
      for (int r = C2; r < 8; ++r) a2[r - C2] = mfma_f64(fa[r], b2, a2[r - C2]);
    }
    if (more) lstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  auto store = [&](const d4_t &acc, int rb, int cb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * rb + mf_row(lane, i), col = 16 * cb + mf_col(lane);
      if (row < w && col <= row) {
        double *p = C + (int64_t)row * ldc + col;
        if (atomic) atomicAdd(p, -acc[i]);
        else *p = -acc[i] + *p;
      }
    }
  };
#pragma unroll
  for (int r = C1; r < 8; ++r) store(a1[r - C1], r, C1);
#pragma unroll
  for (int r = C2; r < 8; ++r) store(a2[r - C2], r, C2);
}

__global__ __launch_bounds__(256, 2) void k_syrk128_diag(int w, int K, const double *__restrict__ A, int64_t lda,
                                                        double *__restrict__ C, int64_t stride, int ks) {
  const int b = blockIdx.x / ks, sp = blockIdx.x % ks;
  const int kc = ((K + ks - 1) / ks + GK - 1) / GK * GK, k_lo = sp * kc, k_hi = min(K, k_lo + kc);
  if (k_lo >= k_hi) return;
  __shared__ double sA[2][BT][GP];
  A += b * stride;
  C += b * stride;
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: syrk_diag_wave<0>(A, lda, w, k_lo, k_hi, sA, C, lda, ks > 1); break;
    case 1: syrk_diag_wave<1>(A, lda, w, k_lo, k_hi, sA, C, lda, ks > 1); break;
    case 2: syrk_diag_wave<2>(A, lda, w, k_lo, k_hi, sA, C, lda, ks > 1); break;
    default: syrk_diag_wave<3>(A, lda, w, k_lo, k_hi, sA, C, lda, ks > 1); break;
  }
}

hipError_t launch_syrk128_diag(hipStream_t s, int w, int K, const double *A, int64_t lda, double *C, int batch,
                               int64_t stride, int ks) {
  if (w <= 0 || K <= 0 || batch <= 0) return hipSuccess;
  if (w > BT) return hipErrorInvalidValue;
  if (ks < 1) ks = 1;
  hipLaunchKernelGGL(k_syrk128_diag, dim3(batch * ks), dim3(256), 0, s, w, K, A, lda, C, stride, ks);
  return hipGetLastError();
}

// The potrf's left-looking block-column step for the rows below the diagonal block,
// fused (one workgroup per 128-row tile r of matrix b, XCD-batched like the row-block GEMM):
//   Y = C - A_r B^T              C = the tile's 128 panel columns, A_r = its rows' K = c left
//                                columns, B = the diagonal block rows' left columns (K = c);
//                                the accumulators start from C and A is staged negated
//   X = Y Linv^T                 Linv = L_cc^-1 (128 x 128, lower) from the diagonal kernel
// Y goes to C in place and is read back by the second product through agent-scope loads
// (the vector L1 is not refreshed by this workgroup's own stores); X overwrites it.  The
// second product's column halves take interleaved 16-column blocks, so the blocks that
// die past Linv's triangle are shared evenly by the two wave columns.
// LA (look-ahead, tile 0 only, wn = the next block's width): tile 0's rows are the next
// diagonal block's, and with X stored they are final over all K + 128 left columns, so the
// same workgroup applies the next step's diagonal update D -= L L^T (lower, K + 128)
// instead of a separate launch: the diagonal kernel of the next step reads D.
// K = 0 (the first block column) is the plain in-place panel solve.
template <bool LA, bool K0 = false>
__global__ __launch_bounds__(256, 2) void k_gemm128_updsolve(int M, int K, const double *__restrict__ A,
                                                            int64_t lda, const double *__restrict__ B,
                                                            double *__restrict__ C, const double *__restrict__ Linv,
                                                            int64_t sA_, int64_t sC_, int64_t sL_, int wn) {
  const int ny = gridDim.y, L = blockIdx.y + blockIdx.z * ny;
  const int m = L >> 3;
  const int bz = (L & 7) + 8 * (m / ny), ry = m % ny;  // matrix b's row tiles on XCD b % 8
  A += bz * sA_;
  B += bz * sA_;
  C += bz * sC_;
  Linv += bz * sL_;
  const int r0 = ry * BT;
  __shared__ double sA[2][BT][GP];
  __shared__ double sB[2][BT][GP];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  d4_t acc[4][4];
  if (!K0 && K > 0) {
    mma128_tile<true, false, false, false, true>(A, lda, B, lda, M, BT, r0, 0, 0, K, sA, sB, acc, -1, false,
                                                 false, C, lda);
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + mma128_row(wave, x, true) + mf_row(lane, r);
          const int col = mma128_col(wave, y, false) + mf_col(lane);
          if (row < M) C[(int64_t)row * lda + col] = acc[x][y][r];
        }
    // every Y store complete at L2 before any wave reads the tile back
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  // K0 (the first block column: no update, nothing written yet): plain 16-byte loads
  mma128_tile<true, !K0, false, true>(C, lda, Linv, BT, M, BT, r0, 0, 0, BT, sA, sB, acc, -1, false, true);
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + mma128_row(wave, x, true) + mf_row(lane, r);
        const int col = mma128_col(wave, y, true) + mf_col(lane);
        if (row < M) C[(int64_t)row * lda + col] = acc[x][y][r];
      }
  if (LA && ry == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    // D = C + 128 columns: rows / columns 0 .. wn-1 of the next diagonal block
    mma128_tile<true, true, true>(A, lda, A, lda, wn, wn, 0, 0, 0, K + BT, sA, sB, acc, -1, true);
    double *D = C + BT;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = mma128_row(wave, x, true) + mf_row(lane, r);
          const int col = mma128_col(wave, y, false) + mf_col(lane);
          if (row < wn && col <= row) {
            double *p = D + (int64_t)row * lda + col;
            *p = -acc[x][y][r] + *p;
          }
        }
  }
}

hipError_t launch_gemm_updsolve(hipStream_t s, int M, int K, const double *A, int64_t lda, const double *B,
                                double *C, const double *Linv, int batch, int64_t sA, int64_t sC, int64_t sL,
                                int wn) {
  if (M <= 0) return hipSuccess;
  if (batch % 8 || wn > BT || wn > M) return hipErrorInvalidValue;
  const dim3 g(1, (M + BT - 1) / BT, batch);
  if (K == 0 && wn == 0)
    hipLaunchKernelGGL((k_gemm128_updsolve<false, true>), g, dim3(256), 0, s, M, K, A, lda, B, C, Linv, sA, sC, sL,
                       0);
  else if (wn > 0)
    hipLaunchKernelGGL(k_gemm128_updsolve<true>, g, dim3(256), 0, s, M, K, A, lda, B, C, Linv, sA, sC, sL, wn);
  else
    hipLaunchKernelGGL(k_gemm128_updsolve<false>, g, dim3(256), 0, s, M, K, A, lda, B, C, Linv, sA, sC, sL, 0);
  return hipGetLastError();
}

// Posterior pass with K* generated in the operand load (no K* in HBM):
//   part[t][j] = sum over the W rows of row tile t of ((W K*^T)_ij)^2,
//   meanT = alpha^T K*^T   (rows msum.. of A = [W; alpha^T])
// where K*[j][k] = k(q_j, x_k) is formed while the tile is staged, from the
// length-scaled query rows Qs (N x D) and training rows Xs (K x D) with the
// k_gram arithmetic (same fma order, same kernel_epilogue: the same bits).
// B-tile thread map: query row lr = tid & 127 (its D features in registers),
// k offset lk = 0 / 8 per wave pair, so each wave's training rows are uniform
// (scalar loads).  A (W) loads, LDS tiles, MFMA loop and epilogue as k_gemm128.
template <int D>
__global__ __launch_bounds__(256, 2) void k_gemm128_post(
    int M, int N, int K, const double *__restrict__ A, int64_t lda, const double *__restrict__ Qs,
    const double *__restrict__ Qn, const double *__restrict__ Xs, const double *__restrict__ Xn,
    int kind, double sigma2, double iso_scale, double *__restrict__ C, int64_t ldc, int msum,
    double *__restrict__ Cm, int64_t ldm) {
  const int by = (int)gridDim.y - 1 - (int)blockIdx.y, bx = blockIdx.x;  // longest row tiles first
  const int r0 = by * BT, c0 = bx * BT;
  const int kend = min(K, r0 + BT);  // W lower triangular; the alpha rows sit in the last tile
  __shared__ double sA[2][BT][GP];
  __shared__ double sB[2][BT][GP];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int qi = (wave >> 1) * 64, qj = (wave & 1) * 64;
  d4_t acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = (d4_t){0.0, 0.0, 0.0, 0.0};
  // A (W rows): row tid/2, k half (tid&1)*8
  const int lr = tid >> 1, lk = (tid & 1) * 8;
  const bool ra = r0 + lr < M;
  const double *pa = A + (int64_t)(ra ? r0 + lr : 0) * lda;
  const bool veca = (lda & 1) == 0 && (((uintptr_t)A) & 15) == 0;
  // B (K*): query row qr, wave-uniform k half
  const int qr = tid & 127;
  const int bk = __builtin_amdgcn_readfirstlane((tid >> 7) * 8);
  const int qrow = c0 + qr;
  const bool rq = qrow < N;
  double qv[D];
#pragma unroll
  for (int d = 0; d < D; ++d) qv[d] = rq ? Qs[(int64_t)qrow * D + d] : 0.0;
  const double qn = rq ? Qn[qrow] : 0.0;
  double va[8], vb[8];
  auto gload = [&](int k0) {
    const int k = k0 + lk;
    if (veca && k + 7 < kend) {
#pragma unroll
      for (int q = 0; q < 8; q += 2) {
        const double2 av = ra ? *(const double2 *)(pa + k + q) : make_double2(0.0, 0.0);
        va[q] = av.x; va[q + 1] = av.y;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) va[q] = (ra && k + q < kend) ? pa[k + q] : 0.0;
    }
    const int kb = k0 + bk;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int kq = kb + q;
      double v = 0.0;
      if (kq < kend) {  // wave-uniform
        const double *x = Xs + (int64_t)kq * D;
        double dot = 0.0;
#pragma unroll
        for (int d = 0; d < D; ++d) dot = fma(qv[d], x[d], dot);
        const double d2 = (qn + Xn[kq]) - 2.0 * dot;
        v = rq ? kernel_epilogue(kind, d2, sigma2, iso_scale) : 0.0;
      }
      vb[q] = v;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sA[buf][lr][lk + q] = va[q];
      sB[buf][qr][bk + q] = vb[q];
    }
  };
  gload(0);
  lstore(0);
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < kend; k0 += GK) {
    const bool more = k0 + GK < kend;
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
  // SUMSQ epilogue (k_gemm128<EPI_SUMSQ>)
  __shared__ double red[4][64];
  double sq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + qi + x * 16 + mf_row(lane, r);
      if (row < msum) {
#pragma unroll
        for (int y = 0; y < 4; ++y) sq[y] = fma(acc[x][y][r], acc[x][y][r], sq[y]);
      } else if (row < M) {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int col = c0 + qj + y * 16 + mf_col(lane);
          if (col < N) Cm[(int64_t)(row - msum) * ldm + col] = acc[x][y][r];
        }
      }
    }
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    sq[y] += __shfl_xor(sq[y], 16);
    sq[y] += __shfl_xor(sq[y], 32);
  }
  if (lane < 16) {
#pragma unroll
    for (int y = 0; y < 4; ++y) red[wave][y * 16 + lane] = sq[y];
  }
  __syncthreads();
  if (tid < 128) {
    const int half = tid >> 6, cc = tid & 63;
    const double v = red[half][cc] + red[2 + half][cc];
    const int col = c0 + tid;
    if (col < N) C[(int64_t)by * ldc + col] = v;
  }
}

hipError_t launch_gemm_post_fused(hipStream_t s, int n, int n_out, int P, const double *Wext,
                                  const double *Qs, const double *Qn, const double *Xs,
                                  const double *Xn, int d, int kind, double sigma2,
                                  double iso_scale, double *part, int64_t ldp, double *meanT,
                                  int64_t ldm) {
  const int M = n + n_out;
  if (P <= 0) return hipSuccess;
  dim3 g((P + BT - 1) / BT, (M + BT - 1) / BT, 1);
  switch (d) {
    case 11:
      hipLaunchKernelGGL(k_gemm128_post<11>, g, dim3(256), 0, s, M, P, n, Wext, (int64_t)n, Qs, Qn,
                         Xs, Xn, kind, sigma2, iso_scale, part, ldp, n, meanT, ldm);
      break;
    case 12:
      hipLaunchKernelGGL(k_gemm128_post<12>, g, dim3(256), 0, s, M, P, n, Wext, (int64_t)n, Qs, Qn,
                         Xs, Xn, kind, sigma2, iso_scale, part, ldp, n, meanT, ldm);
      break;
    case 13:
      hipLaunchKernelGGL(k_gemm128_post<13>, g, dim3(256), 0, s, M, P, n, Wext, (int64_t)n, Qs, Qn,
                         Xs, Xn, kind, sigma2, iso_scale, part, ldp, n, meanT, ldm);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Stream-K (C += alpha A B^T, STORE epilogue with beta = 1): the batch's
// (tile, K-step) units are cut into gridDim.x equal contiguous ranges, one per
// workgroup, so every resident slot does the same work whatever the tile count
// (no quantisation tail); each tile segment is added into C with fp64 atomics.
// Tiles are lower-triangular (tri) or the full tx x ty grid.
__global__ __launch_bounds__(256, 2) void k_gemm128_sk(int M, int N, int K,
                                                       const double *__restrict__ A, int64_t lda,
                                                       const double *__restrict__ B, int64_t ldb,
                                                       double *__restrict__ C, int64_t ldc,
                                                       double alpha, int tri, int tx, int T,
                                                       int64_t sA_, int64_t sB_, int64_t sC_,
                                                       int64_t total) {
  __shared__ double sA[2][BT][GP];
  __shared__ double sB[2][BT][GP];
  const int kiters = (K + GK - 1) / GK;
  int64_t u = (int64_t)blockIdx.x * total / gridDim.x;
  const int64_t u1 = (int64_t)(blockIdx.x + 1) * total / gridDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qi = (wave >> 1) * 64, qj = (wave & 1) * 64;
  while (u < u1) {
    const int64_t g = u / kiters;
    const int j0 = (int)(u - g * kiters);
    const int j1 = (int)min((int64_t)kiters, (int64_t)j0 + (u1 - u));
    const int bz = (int)(g / T), t = (int)(g % T);
    int by, bx;
    if (tri) tri_tile(t, by, bx);
    else by = t / tx, bx = t % tx;
    const int r0 = by * BT, c0 = bx * BT;
    d4_t acc[4][4];
    mma128_tile(A + bz * sA_, lda, B + bz * sB_, ldb, M, N, r0, c0, j0 * GK, min(K, j1 * GK), sA,
                sB, acc, 0, tri != 0);  // padding rows of the last row tile skipped
    double *Cb = C + bz * sC_;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = r0 + qi + x * 16 + mf_row(lane, r);
          const int col = c0 + qj + y * 16 + mf_col(lane);
          if (row < M && col < N && (!tri || col <= row))
            atomicAdd(Cb + (int64_t)row * ldc + col, alpha * acc[x][y][r]);
        }
    u += j1 - j0;
  }
}

// ---------------------------------------------------------------------------
// Latency form for short products (K <= 128) on few matrices: the Cholesky's
// panel solve and trailing SYRK at batch 1-16, where the pipelined tile kernels
// above spend their time in K / 16 dependent global-load round trips (13 us for
// a K = 128 SYRK of three workgroups, 29 us for a 128 x 128 x 128 panel tile on
// one CU).  Each wave owns a 16 x 32 block of C and loads its whole operand
// strip straight into registers -- 16 two-double loads per 16-row fragment,
// all in flight at once -- then runs the MFMAs: one memory round trip per
// launch.  Chunk t of 8 k's: lane l holds k = 8t + 2(l >> 4) + {0, 1} of row /
// column l & 15, used by two MFMAs (.x, .y); A and B share the permutation, so
// every k is summed once.
//   MODE 0 (rows, in place): a workgroup owns rows [16 bx, +16) x all N <= 128
//     columns (wave w: columns 32w..), so C may alias A: every wave's loads are
//     consumed before the barrier that precedes the stores.  tri_b: B is lower
//     triangular (B[c][k] = 0 for k > c), column block c0 stops at k < c0 + 32.
//   MODE 1 (lower): C = alpha A A^T + beta C over the lower 32 x 32 blocks of an
//     M x M matrix (B = A), two waves per block (row halves).
#define LAT_CH 16  // 16 chunks of 8 = K <= 128
template <int MODE>
__global__ __launch_bounds__(256) void k_gemm_lat(int M, int N, int K, const double *A, int64_t lda,
                                                  const double *B, int64_t ldb, double *C,
                                                  int64_t ldc, double alpha, double beta, int tri_b,
                                                  int64_t sA_, int64_t sB_, int64_t sC_) {
  const int bz = blockIdx.z;
  A += bz * sA_;
  B += bz * sB_;
  C += bz * sC_;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  int r0, c0, kend = K;
  bool live = true, upper_half = false;
  if (MODE == 0) {
    r0 = blockIdx.x * 16;
    c0 = wave * 32;
    live = c0 < N;
    if (tri_b) kend = min(K, c0 + 32);
  } else {
    const int nb = (M + 31) / 32, T = nb * (nb + 1) / 2;
    const int blk = blockIdx.x * 2 + (wave >> 1);
    int bi, bj;
    tri_tile(min(blk, T - 1), bi, bj);
    live = blk < T;
    r0 = bi * 32 + (wave & 1) * 16;
    c0 = bj * 32;
    upper_half = bi == bj && (wave & 1) == 0;  // its columns 16..31 lie above the diagonal
  }
  const int li = lane & 15, kq = (lane >> 4) * 2;
  const int ra = r0 + li, rb0 = c0 + li, rb1 = c0 + 16 + li;
  const bool va = live && ra < M, vb0 = live && rb0 < N, vb1 = live && rb1 < N && !upper_half;
  const double *pa = A + (int64_t)(va ? ra : 0) * lda;
  const double *pb0 = B + (int64_t)(vb0 ? rb0 : 0) * ldb;
  const double *pb1 = B + (int64_t)(vb1 ? rb1 : 0) * ldb;
  const bool vec = ((lda | ldb) & 1) == 0 && ((((uintptr_t)A) | ((uintptr_t)B)) & 15) == 0;
  auto ld2 = [&](const double *p, bool v, int k) -> double2 {
    if (!v || k >= kend) return make_double2(0.0, 0.0);
    if (k + 1 >= kend) return make_double2(p[k], 0.0);
    if (vec) return *(const double2 *)(p + k);
    return make_double2(p[k], p[k + 1]);
  };
  double2 a[LAT_CH], b0[LAT_CH], b1[LAT_CH];
#pragma unroll
  for (int t = 0; t < LAT_CH; ++t) {
    const int k = 8 * t + kq;
    a[t] = ld2(pa, va, k);
    b0[t] = ld2(pb0, vb0, k);
    b1[t] = ld2(pb1, vb1, k);
  }
  d4_t cpre[2];
  if (MODE == 1 && beta != 0.0) {
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + mf_row(lane, r), col = c0 + 16 * y + li;
        cpre[y][r] = (live && row < M && col <= row) ? C[(int64_t)row * ldc + col] : 0.0;
      }
  }
  d4_t acc0 = d4_t{0.0, 0.0, 0.0, 0.0}, acc1 = acc0;
#pragma unroll
  for (int t = 0; t < LAT_CH; ++t) {
    acc0 = mfma_f64(a[t].x, b0[t].x, acc0);
    acc1 = mfma_f64(a[t].x, b1[t].x, acc1);
    acc0 = mfma_f64(a[t].y, b0[t].y, acc0);
    acc1 = mfma_f64(a[t].y, b1[t].y, acc1);
  }
  if (MODE == 0) __syncthreads();  // every wave's operand reads are done: C may alias A
  if (!live) return;
#pragma unroll
  for (int y = 0; y < 2; ++y)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + mf_row(lane, r), col = c0 + 16 * y + li;
      const double v = y ? acc1[r] : acc0[r];
      if (MODE == 0) {
        if (row < M && col < N) {
          double *p = C + (int64_t)row * ldc + col;
          *p = beta == 0.0 ? alpha * v : alpha * v + beta * *p;
        }
      } else if (row < M && col <= row) {
        C[(int64_t)row * ldc + col] = beta == 0.0 ? alpha * v : alpha * v + beta * cpre[y][r];
      }
    }
}

hipError_t launch_gemm_lat(hipStream_t s, int mode, int M, int N, int K, const double *A,
                           int64_t lda, const double *B, int64_t ldb, double *C, int64_t ldc,
                           double alpha, double beta, int tri_b, int batch, int64_t sA, int64_t sB,
                           int64_t sC) {
  if (M <= 0 || N <= 0 || batch <= 0) return hipSuccess;
  if (K > 8 * LAT_CH || (mode == 0 && N > 128) || (mode == 1 && N != M)) return hipErrorInvalidValue;
  if (mode == 0) {
    hipLaunchKernelGGL(k_gemm_lat<0>, dim3((M + 15) / 16, 1, batch), dim3(256), 0, s, M, N, K, A,
                       lda, B, ldb, C, ldc, alpha, beta, tri_b, sA, sB, sC);
  } else {
    const int nb = (M + 31) / 32, T = nb * (nb + 1) / 2;
    hipLaunchKernelGGL(k_gemm_lat<1>, dim3((T + 1) / 2, 1, batch), dim3(256), 0, s, M, N, K, A, lda,
                       A, lda, C, ldc, alpha, beta, 0, sA, sA, sC);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Skinny products (M or N <= 32) with a long K -- the GEMVs of alpha = W^T (W y), the
// append's B^T = K21 W^T, S -= B^T B: on the 64-tile kernel they were a few workgroups
// each walking K / 16 dependent steps (70-90 us at K = 1000).  K is cut into S chunks
// (multiples of GK) whose partial products go to scratch slot 5 as a batch of the
// 64-tile kernel, then k_splitk_reduce forms C = alpha sum_s P_s + beta C in chunk order
// (deterministic; the sums run in another order than the one-pass product).
__global__ __launch_bounds__(256) void k_splitk_reduce(int M, int N, int S, const double *__restrict__ P,
                                                       double *__restrict__ C, int64_t ldc, double alpha,
                                                       double beta) {
  const int64_t MN = (int64_t)M * N;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < MN; e += (int64_t)gridDim.x * 256) {
    double acc = 0.0;
    for (int q = 0; q < S; ++q) acc += P[q * MN + e];
    const int i = (int)(e / N), j = (int)(e - (int64_t)i * N);
    double *c = C + (int64_t)i * ldc + j;
    *c = beta == 0.0 ? alpha * acc : alpha * acc + beta * *c;
  }
}

static bool splitk_env() {
  static const int v = [] {
    const char *e = getenv("GPMPC_SPLITK");
    return e ? atoi(e) : 1;
  }();
  return v != 0;
}

// form: 0 NT (A M x K, B N x K), 1 NN (B K x N), 2 TN (A K x M, B K x N).  Returns false
// (nothing launched) when the product is not skinny enough or scratch is unavailable.
static bool launch_splitk(hipStream_t s, int form, int M, int N, int K, const double *A, int64_t lda,
                          const double *B, int64_t ldb, double *C, int64_t ldc, double alpha, double beta,
                          hipError_t &err) {
  if (!splitk_env() || !(M <= 32 || N <= 32) || K < 256) return false;
  const int tiles = ((M + GT - 1) / GT) * ((N + GT - 1) / GT);
  int S = std::max(1, std::min(512 / tiles, K / 64));
  if (S < 2) return false;
  const int kc = ((K + S - 1) / S + GK - 1) / GK * GK;
  S = (K + kc - 1) / kc;
  const int64_t MN = (int64_t)M * N;
  double *P = (double *)gpmpc_scratch(s, 5, sizeof(double) * MN * S);
  if (!P) return false;
  // chunk q: A and B advance by kc along K
  const int64_t sA = form == 2 ? (int64_t)kc * lda : kc, sB = form == 0 ? kc : (int64_t)kc * ldb;
  const int klast = K - (S - 1) * kc;  // the last chunk's length (one launch for all chunks)
  const dim3 g((N + GT - 1) / GT, (M + GT - 1) / GT, S);
  if (form == 0)
    hipLaunchKernelGGL((k_gemm_nt<EPI_STORE, 0, 0>), g, dim3(256), 0, s, M, N, kc, A, lda, B, ldb, P, (int64_t)N,
                       1.0, 0.0, 0, 0, sA, sB, MN, M, nullptr, (int64_t)0, 0, 0, klast);
  else if (form == 1)
    hipLaunchKernelGGL((k_gemm_nt<EPI_STORE, 1, 0>), g, dim3(256), 0, s, M, N, kc, A, lda, B, ldb, P, (int64_t)N,
                       1.0, 0.0, 0, 0, sA, sB, MN, M, nullptr, (int64_t)0, 0, 0, klast);
  else
    hipLaunchKernelGGL((k_gemm_nt<EPI_STORE, 1, 1>), g, dim3(256), 0, s, M, N, kc, A, lda, B, ldb, P, (int64_t)N,
                       1.0, 0.0, 0, 0, sA, sB, MN, M, nullptr, (int64_t)0, 0, 0, klast);
  const int rb = (int)std::min<int64_t>((MN + 255) / 256, 1024);
  hipLaunchKernelGGL(k_splitk_reduce, dim3(rb), dim3(256), 0, s, M, N, S, P, C, ldc, alpha, beta);
  err = hipGetLastError();
  return true;
}

// The SUMSQ form of the same split for few columns (the posterior of one landing's 20
// queries, a predict of a few points): v = sum_s P_s per element, then per 64-row tile t
// part[t][j] = sum over its rows r < msum of v(r, j)^2 and the rows msum..M-1 to Cm -- the
// 64-tile SUMSQ kernel's output layout (gemm_row_tiles rows), so consumers are unchanged.
// Block (t, c): wave w takes column 4 c + w, lane = row of the tile; the S partials of an
// element are independent loads (in flight together), the column's sum of squares a wave
// reduction.
__global__ __launch_bounds__(256) void k_splitk_sumsq(int M, int N, int S, const double *__restrict__ P, int msum,
                                                      double *__restrict__ part, int64_t ldp,
                                                      double *__restrict__ Cm, int64_t ldm) {
  const int t = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = t * 64 + lane;
  const int64_t MN = (int64_t)M * N;
  for (int j = 4 * (int)blockIdx.y + w; j < N; j += 4 * (int)gridDim.y) {
    double v = 0.0;
    if (r < M) {
      const double *pe = P + (int64_t)r * N + j;
      double a[8];
      int q = 0;
      for (; q + 8 <= S; q += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = pe[(q + u) * MN];
#pragma unroll
        for (int u = 0; u < 8; ++u) v += a[u];
      }
      for (; q < S; ++q) v += pe[q * MN];
    }
    double sq = (r < msum) ? v * v : 0.0;
    if (r >= msum && r < M) Cm[(int64_t)(r - msum) * ldm + j] = v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
    if (lane == 0) part[(int64_t)t * ldp + j] = sq;
  }
}

static bool launch_splitk_sumsq(hipStream_t s, int M, int N, int K, const double *A, int64_t lda, const double *B,
                                int64_t ldb, double *part, int64_t ldp, int msum, double *Cm, int64_t ldm,
                                hipError_t &err) {
  if (!splitk_env() || N > GT || K < 256) return false;
  const int ty = (M + GT - 1) / GT;
  int S = std::max(1, std::min(512 / ty, K / 64));
  if (S < 2) return false;
  const int kc = ((K + S - 1) / S + GK - 1) / GK * GK;
  S = (K + kc - 1) / kc;
  const int64_t MN = (int64_t)M * N;
  double *P = (double *)gpmpc_scratch(s, 5, sizeof(double) * MN * S);
  if (!P) return false;
  hipLaunchKernelGGL((k_gemm_nt<EPI_STORE, 0, 0>), dim3(1, ty, S), dim3(256), 0, s, M, N, kc, A, lda, B, ldb, P,
                     (int64_t)N, 1.0, 0.0, 0, 0, (int64_t)kc, (int64_t)kc, MN, M, nullptr, (int64_t)0, 0, 0,
                     K - (S - 1) * kc);
  hipLaunchKernelGGL(k_splitk_sumsq, dim3(ty, (N + 3) / 4), dim3(256), 0, s, M, N, S, P, msum, part, ldp, Cm, ldm);
  err = hipGetLastError();
  return true;
}

static int gemm_big_env() {
  static const int v = [] {
    const char *e = getenv("GPMPC_GEMM128");
    return e ? atoi(e) : 1;
  }();
  return v;
}

static int gemm_kmin_env() {
  static const int v = [] {
    const char *e = getenv("GPMPC_GEMM128_KMIN");
    return e ? atoi(e) : 2 * BT;
  }();
  return v;
}

// The kernel launch_gemm_sumsq_mean picks for an (M x K) [W; alpha^T] against N query
// rows (batch 1, triangular A): the rules of launch_gemm_impl below.  A caller whose column
// count shrinks over time (the fleet's running prefix) fixes this at its planned size and
// passes it back, so every column sees the same kernel, hence the same bits.
int gemm_sumsq_kind(int M, int N, int K) {
  if (gemm_big_env() && M >= 2 * BT && N >= 2 * BT && K >= gemm_kmin_env()) return GEMM_SUMSQ_128;
  if (splitk_env() && N <= GT && K >= 256 && std::max(1, std::min(512 / ((M + GT - 1) / GT), K / 64)) >= 2)
    return GEMM_SUMSQ_SPLITK;
  return GEMM_SUMSQ_64;
}

static hipError_t launch_gemm_impl(hipStream_t s, int epi, int M, int N, int K, const double *A,
                                   int64_t lda, const double *B, int64_t ldb, double *C,
                                   int64_t ldc, double alpha, double beta, int tri_a, int lower_c,
                                   int batch, int64_t sA, int64_t sB, int64_t sC, int msum,
                                   double *Cm, int64_t ldm, int kind = -1) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const int big_env = gemm_big_env();
  // kind >= 0 (EPI_SUMSQ, batch 1): that kernel, whatever the size (gemm_sumsq_kind)
  if (epi != EPI_SUMSQ || batch != 1) kind = -1;
  const bool tg = lower_c && M == N && !tri_a;
  // a lower-triangular batch takes 128-tiles only when they fill >= 2 rounds
  // of 512 resident workgroups or K is long enough to split; otherwise they
  // quantise badly (1.1-1.25 rounds: 21-36% vs 44-50% for 64-tiles).  FITC
  // 2000 x 4000: 128-tiles + split-K 56% vs 39%
  const int t128 = ((M + BT - 1) / BT) * ((M + BT - 1) / BT + 1) / 2 * batch;
  static const int syrk128_env = [] {
    const char *e = getenv("GPMPC_SYRK128");
    return e ? atoi(e) : -1;
  }();
  const bool tri_ok = !tg || (syrk128_env >= 0 ? syrk128_env != 0 : t128 >= 1024 || K >= 1024);
  static const int sk_env = [] {
    const char *e = getenv("GPMPC_STREAMK");
    return e ? atoi(e) : -1;
  }();
  // stream-K for long accumulations into C on big tiles: measured 2000^2 x 4000
  // 60% (split-K 55%), 4000^2 x 4000 72%, 16 x 1000^2 x 1000 56% (64-tiles 52%);
  // smaller or shorter products (n ~ 500, K <= 256) keep the tiled kernels
  const bool sk_ok = epi == EPI_STORE && beta == 1.0 && !tri_a && M >= 2 * BT && N >= 2 * BT &&
                     K >= 2 * BT;
  const bool sk_auto = M >= 768 && N >= 768 && K >= 512;
  if (sk_ok && (sk_env >= 0 ? sk_env > 0 : sk_auto)) {
    const int tx = (N + BT - 1) / BT, ty = (M + BT - 1) / BT;
    const int T = tg ? ty * (ty + 1) / 2 : tx * ty;
    const int64_t total = (int64_t)T * batch * ((K + GK - 1) / GK);
    const int nwg = (int)std::min<int64_t>(512, total);
    hipLaunchKernelGGL(k_gemm128_sk, dim3(nwg), dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc,
                       alpha, (int)tg, tx, T, sA, sB, sC, total);
    return hipGetLastError();
  }
  const int kmin_env = gemm_kmin_env();
  const bool use128 = kind >= 0 ? kind == GEMM_SUMSQ_128 : big_env && tri_ok && M >= 2 * BT && N >= 2 * BT && K >= kmin_env;
  if (use128) {
    const int tx = (N + BT - 1) / BT, ty = (M + BT - 1) / BT;
    // split K when the tiles cannot give each CU ~4 workgroups to interleave (STORE
    // with beta = 1: partial products are added atomically); >= 512 of K per split
    const int tiles = (lower_c ? ty * (ty + 1) / 2 : tx * ty) * batch;
    // cost model: rounds of 512 resident workgroups (2 per CU) x (K per split
    // + ~256 of fixed cost: prologue, atomic C update).  Measured on 2000^2 x
    // 4000: ks 1/2/3/4/6/8 -> 30/38/53/43/49/45% (ks 4 leaves a 32-WG tail)
    int ksplit = 1;
    if (epi == EPI_STORE && beta == 1.0 && K >= 1024) {
      double best = 1e30;
      for (int ks = 1; ks <= K / 256 && ks <= 16; ++ks) {
        const double c = (double)((tiles * ks + 511) / 512) * ((double)K / ks + 256.0);
        if (c < best * 0.98) best = c, ksplit = ks;
      }
    }
    static const int ks_env = [] {
      const char *e = getenv("GPMPC_KSPLIT");
      return e ? atoi(e) : 0;
    }();
    if (ks_env > 0 && epi == EPI_STORE && beta == 1.0) ksplit = ks_env;
    // lower-triangular square products launch only their lower tiles, in a
    // 1-D order that interleaves them over the 8 XCDs (a 2-D grid whose
    // column count is a multiple of 8 pins columns to XCDs: 8x imbalance)
    dim3 g(tg ? ty * (ty + 1) / 2 : tx, tg ? 1 : ty, batch * ksplit);
    if (epi == EPI_STORE)
      hipLaunchKernelGGL(k_gemm128<EPI_STORE>, g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc,
                         alpha, beta, tri_a, lower_c, sA, sB, sC, M, nullptr, (int64_t)0, ksplit,
                         (int)tg);
    else
      hipLaunchKernelGGL(k_gemm128<EPI_SUMSQ>, g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc,
                         alpha, beta, tri_a, 0, sA, sB, sC, msum, Cm, ldm, 1,
                         (post_xcd() && batch == 1 && tx % 8 == 0) ? 2 : 0);
    return hipGetLastError();
  }
  if (epi == EPI_STORE && batch == 1 && !tri_a && !lower_c) {
    hipError_t e = hipSuccess;
    if (launch_splitk(s, 0, M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, e)) return e;
  }
  if (epi == EPI_SUMSQ && batch == 1 &&
      (kind >= 0 ? kind == GEMM_SUMSQ_SPLITK : gemm_row_tiles(M, N, K) == (M + GT - 1) / GT)) {
    hipError_t e = hipSuccess;  // (a triangular A's zero chunks are multiplied: the split is latency work)
    if (launch_splitk_sumsq(s, M, N, K, A, lda, B, ldb, C, ldc, msum, Cm, ldm, e)) return e;
  }
  const int tx = (N + GT - 1) / GT, ty = (M + GT - 1) / GT;
  static const int remap_env = [] {
    const char *e = getenv("GPMPC_GEMM_REMAP");
    return e ? atoi(e) : 0;  // measured slower for the posterior GEMM (W blocks thrash)
  }();
  const bool remap = remap_env && batch == 1 && ty > 1 && tx % 8 == 0;
  static const int xb_env = [] {
    const char *e = getenv("GPMPC_XCD_BATCH");
    return e ? atoi(e) : 1;
  }();
  const int T = ty * (ty + 1) / 2;
  const int xb = (tg && xb_env && batch >= 8) ? batch : 0;
  dim3 g = xb ? dim3(T * ((batch + 7) / 8) * 8, 1, 1)
         : tg ? dim3(T, 1, batch) : remap ? dim3(tx * ty, 1, 1) : dim3(tx, ty, batch);
  const int rt = tg ? -1 : remap ? ty : 0;
  if (epi == EPI_STORE)
    hipLaunchKernelGGL(k_gemm_nt<EPI_STORE>, g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc,
                       alpha, beta, tri_a, lower_c, sA, sB, sC, M, nullptr, (int64_t)0, rt, xb, 0);
  else
    hipLaunchKernelGGL(k_gemm_nt<EPI_SUMSQ>, g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc,
                       alpha, beta, tri_a, 0, sA, sB, sC, msum, Cm, ldm, rt, 0, 0);
  return hipGetLastError();
}

// C (M x N) = alpha A (M x K) B (K x N) + beta C, all row-major (64-tile kernel)
hipError_t launch_gemm_nn(hipStream_t s, int M, int N, int K, const double *A, int64_t lda,
                          const double *B, int64_t ldb, double *C, int64_t ldc, double alpha,
                          double beta) {
  if (M <= 0 || N <= 0) return hipSuccess;
  hipError_t e = hipSuccess;
  if (launch_splitk(s, 1, M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, e)) return e;
  dim3 g((N + GT - 1) / GT, (M + GT - 1) / GT, 1);
  hipLaunchKernelGGL((k_gemm_nt<EPI_STORE, 1, 0>), g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C,
                     ldc, alpha, beta, 0, 0, (int64_t)0, (int64_t)0, (int64_t)0, M, nullptr,
                     (int64_t)0, 0, 0, 0);
  return hipGetLastError();
}

// the same for batch products sA / sB / sC elements apart
hipError_t launch_gemm_nn_batched(hipStream_t s, int M, int N, int K, const double *A, int64_t lda, int64_t sA,
                                  const double *B, int64_t ldb, int64_t sB, double *C, int64_t ldc, int64_t sC,
                                  double alpha, double beta, int batch) {
  if (M <= 0 || N <= 0 || batch <= 0) return hipSuccess;
  dim3 g((N + GT - 1) / GT, (M + GT - 1) / GT, batch);
  hipLaunchKernelGGL((k_gemm_nt<EPI_STORE, 1, 0>), g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C,
                     ldc, alpha, beta, 0, 0, sA, sB, sC, M, nullptr, (int64_t)0, 0, 0, 0);
  return hipGetLastError();
}

// C (M x N) = alpha A^T B + beta C with A (K x M) and B (K x N) row-major ("TN")
hipError_t launch_gemm_tn(hipStream_t s, int M, int N, int K, const double *A, int64_t lda,
                          const double *B, int64_t ldb, double *C, int64_t ldc, double alpha,
                          double beta) {
  if (M <= 0 || N <= 0) return hipSuccess;
  hipError_t e = hipSuccess;
  if (launch_splitk(s, 2, M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, e)) return e;
  dim3 g((N + GT - 1) / GT, (M + GT - 1) / GT, 1);
  hipLaunchKernelGGL((k_gemm_nt<EPI_STORE, 1, 1>), g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C,
                     ldc, alpha, beta, 0, 0, (int64_t)0, (int64_t)0, (int64_t)0, M, nullptr,
                     (int64_t)0, 0, 0, 0);
  return hipGetLastError();
}

// C = alpha A B^T + beta C with N <= 128 on the 128 x 128 tile kernel: one
// workgroup owns whole rows of C, so C may alias A (every A read of a row
// block precedes its epilogue) -- the in-place panel solve of the potrf.
hipError_t launch_gemm_nt_rowblock(hipStream_t s, int M, int N, int K, const double *A,
                                   int64_t lda, const double *B, int64_t ldb, double *C,
                                   int64_t ldc, double alpha, double beta, int batch, int64_t sA,
                                   int64_t sB, int64_t sC, int lower_c, int ksplit) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (N > BT) return hipErrorInvalidValue;
  // split K (partial products added atomically): only with beta = 1 and C apart from A, B
  if (ksplit < 1 || beta != 1.0) ksplit = 1;
  dim3 g(1, (M + BT - 1) / BT, batch * ksplit);
  // a batch of >= 8 matrices (a multiple of 8): each matrix's row tiles on one XCD
  static const int xb_env = [] {
    const char *e = getenv("GPMPC_ROWBLOCK_XCD");
    return e ? atoi(e) : 1;
  }();
  const int tg = (xb_env && batch >= 8 && batch % 8 == 0) ? 3 : 0;
  hipLaunchKernelGGL(k_gemm128<EPI_STORE>, g, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc,
                     alpha, beta, 0, lower_c, sA, sB, sC, M, nullptr, (int64_t)0, ksplit, tg);
  return hipGetLastError();
}

hipError_t launch_gemm_nt(hipStream_t s, int epi, int M, int N, int K, const double *A,
                          int64_t lda, const double *B, int64_t ldb, double *C, int64_t ldc,
                          double alpha, double beta, int tri_a, int lower_c, int batch,
                          int64_t sA, int64_t sB, int64_t sC) {
  return launch_gemm_impl(s, epi, M, N, K, A, lda, B, ldb, C, ldc, alpha, beta, tri_a, lower_c,
                          batch, sA, sB, sC, M, nullptr, 0);
}

hipError_t launch_gemm_sumsq(hipStream_t s, int n, int P, const double *A, const double *Ks, double *part,
                             int64_t ldp, int kind) {
  return launch_gemm_impl(s, EPI_SUMSQ, n, P, n, A, n, Ks, n, part, ldp, 1.0, 0.0, 1, 0, 1, 0, 0, 0, n, nullptr,
                          0, kind);
}

hipError_t launch_gemm_sumsq_mean(hipStream_t s, int n, int n_out, int P, const double *Wext,
                                  const double *Ks, double *part, int64_t ldp, double *meanT,
                                  int64_t ldm, int kind) {
  return launch_gemm_impl(s, EPI_SUMSQ, n + n_out, P, n, Wext, n, Ks, n, part, ldp, 1.0, 0.0, 1, 0,
                          1, 0, 0, 0, n, meanT, ldm, kind);
}
