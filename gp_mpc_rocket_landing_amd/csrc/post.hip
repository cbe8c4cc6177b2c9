// post.hip -- the exact-GP posterior of many queries, column-stationary, with K* formed
// on the fly (ExactGP.predict, exact_gp.py:237-266: K* = k(X*, X), mean = K* alpha,
// var = sigma2 - |L^-1 K*^T|^2; kernels.py:205-262 for K*).
//
// One 512-thread workgroup owns 32 queries and HALF of the rows of [W; alpha^T]
// (W = L^-1, n <= 1008): the rows are cut into 16-row MFMA blocks b = 0 .. NB-1 plus the
// alpha block NB; block b belongs to wave b % 8 as its slot b / 8, and the workgroup of
// half h keeps the slots {0, 3, 4, 7} (h = 0) or {1, 2, 5, 6} (h = 1) -- the two halves
// then carry the same triangle area (1040 block-steps each at n = 1000) and inside a
// half every wave's live blocks at a K step differ by at most one (96% step balance).
// So a workgroup's accumulators hold its rows of W K*^T for all n columns of K at once:
// the 32-query K* slab of each 16-wide K step is formed ONCE per workgroup (each thread
// one value: the k_gram arithmetic, same bits) into a double-buffered 8 KB LDS ring,
// and K* never exists in HBM.  W is read straight into registers as MFMA A fragments
// from a packed fragment-order copy (k_post_pack: per K step j the blocks j .. NB, each
// 64 lanes x 4 doubles contiguous, the triangle above the diagonal not stored), one
// step ahead; each fragment feeds both 16-query column blocks.  A block stops at the
// last K step that touches its rows (W lower triangular); the alpha block runs all.
//
// Outputs per query: the sum of squares over this half's W rows (part[h]) and, from the
// workgroup holding the alpha block, the mean rows alpha^T K*^T (meanT) -- the layout
// k_post_finish / the fleet's fused finish already read (two partial rows).
// The MFMA sequence of the mean (k = 16 j + 4 s + lane / 16 per substep s, steps in
// order) is the 128-tile SUMSQ kernel's, and K* has the same bits, so the mean is
// bit-identical to the K*-in-HBM path.
#include "internal.h"
#include "mfma64.h"
#include "gemm.h"

namespace {
constexpr int PQ = 32;              // queries per workgroup
constexpr int NCW = 8;              // consumer (MFMA) waves
constexpr int NPW = 4;              // producer (K*) waves
constexpr int PT = 64 * (NCW + NPW);  // 768 threads: three waves per SIMD
constexpr int SLAB = 16 * PQ;       // K* values of one 16-wide K step
#ifndef POST_RING
#define POST_RING 8
#endif
#ifndef POST_PF
#define POST_PF 2  // training rows a producer thread keeps in flight
#endif
constexpr int RING = POST_RING;     // slabs in flight between producers and consumers

__host__ __device__ inline int64_t post_foff(int j, int NB) {  // first fragment of K step j
  return (int64_t)j * (NB + 1) - (int64_t)j * (j - 1) / 2;
}

// slot of the t-th block of a wave in half h
__device__ __forceinline__ int post_slot(int h, int t) {
  return h == 0 ? (t == 0 ? 0 : t == 1 ? 3 : t == 2 ? 4 : 7) : (t == 0 ? 1 : t == 1 ? 2 : t == 2 ? 5 : 6);
}
}  // namespace

int post_cs_blocks(int n) { return (n + 15) / 16; }

bool post_cs_ok(int n, int n_out, int d) {
  return n >= 1 && post_cs_blocks(n) <= 63 && n_out >= 1 && n_out <= 16 && d >= 11 && d <= 13;
}

size_t post_cs_frag_doubles(int n) {
  const int NB = post_cs_blocks(n);
  return (size_t)post_foff(NB, NB) * 256;
}

int post_cs_row_pitch(int d) { return (d + 2) & ~1; }  // scaled row | its squared norm, even

// Wf[(foff(j) + b - j) * 256 + lane * 4 + s] = A[16 b + lane % 16][16 j + 4 s + lane / 16]
// with A = [W (lower, rows < n); alpha^T (rows n .. n + n_out - 1) as block NB], zeros
// outside; Xp[k * DP + i] = Xs[k][i] (i < d), Xp[k * DP + d] = Xn[k], the rest zero.
__global__ void k_post_pack(int n, int NB, int n_out, const double *__restrict__ Wext, int64_t ldw,
                            const double *__restrict__ Xs, const double *__restrict__ Xn, int d, int DP,
                            double *__restrict__ Wf, double *__restrict__ Xp) {
  const int j = blockIdx.y, b = j + blockIdx.x, lane = threadIdx.x;
  if (b <= NB) {
    const int r = 16 * b + (lane & 15);
    double v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = 16 * j + 4 * s + (lane >> 4);
      double x = 0.0;
      if (b < NB) {
        if (r < n && k < n && k <= r) x = Wext[(int64_t)r * ldw + k];
      } else if ((lane & 15) < n_out && k < n) {
        x = Wext[(int64_t)(n + (lane & 15)) * ldw + k];
      }
      v[s] = x;
    }
    double *o = Wf + (post_foff(j, NB) + (b - j)) * 256 + lane * 4;
    *(double2 *)o = make_double2(v[0], v[1]);
    *(double2 *)(o + 2) = make_double2(v[2], v[3]);
  }
  // the padded training rows: one workgroup row per 64 rows (blockIdx.x == 0 column)
  if (blockIdx.x == 0) {
    const int k = 64 * (int)blockIdx.y + lane;
    for (int kk = k; kk < n; kk += 64 * (int)gridDim.y)
      for (int i = 0; i < DP; ++i)
        Xp[(int64_t)kk * DP + i] = i < d ? Xs[(int64_t)kk * d + i] : (i == d ? Xn[kk] : 0.0);
  }
}

hipError_t launch_post_pack(hipStream_t s, int n, int n_out, const double *Wext, int64_t ldw,
                            const double *Xs, const double *Xn, int d, double *Wf, double *Xp) {
  if (!post_cs_ok(n, n_out, d)) return hipErrorInvalidValue;
  const int NB = post_cs_blocks(n);
  hipLaunchKernelGGL(k_post_pack, dim3(NB + 1, NB), dim3(64), 0, s, n, NB, n_out, Wext, ldw, Xs, Xn, d,
                     post_cs_row_pitch(d), Wf, Xp);
  return hipGetLastError();
}

template <int D>
__global__ __launch_bounds__(PT, 1) void k_post_cs(int n, int NB, int P, int n_out, const double *__restrict__ Wf,
                                                   const double *__restrict__ Xp, const double *__restrict__ Qs,
                                                   const double *__restrict__ Qn, int kind, double sigma2,
                                                   double iso_scale, double *__restrict__ part, int64_t ldp,
                                                   double *__restrict__ meanT, int64_t ldm) {
  constexpr int DP = (D + 2) & ~1;
  const int h = blockIdx.x & 1, c0 = (int)(blockIdx.x >> 1) * PQ;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NS = NB;  // K steps of 16 over n (zero padded)
  __shared__ double sK[RING][SLAB];
  __shared__ double red[NCW][PQ];
  // per-wave progress words (one writer each): slabs formed by producer p, slabs released
  // by consumer w; a wait that expired (a broken invariant: the group's output goes NaN)
  __shared__ int s_ready[NPW], s_free[NCW], s_fail;
  if (tid < NPW) s_ready[tid] = 0;
  if (tid < NCW) s_free[tid] = 0;
  if (tid == 0) s_fail = 0;
  __syncthreads();
  auto ld = [](int *f) { return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  // bounded wait until every word of f[0 .. cnt) is >= v; returns their minimum, which the
  // caller keeps so that it reads the flags again only when it has caught up with them
  auto wait_all = [&](int *f, int cnt, int v) {
    int mn = 0;
    for (int it = 0;; ++it) {
      mn = 1 << 30;
      for (int i = 0; i < cnt; ++i) mn = min(mn, ld(f + i));
      if (mn >= v) break;
      if (it > (1 << 20)) {
        __hip_atomic_store(&s_fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        mn = 1 << 30;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");  // the slab accesses stay behind the flags
    return mn;
  };
  // publish this wave's progress after its LDS accesses of the slab have completed
  auto publish = [&](int *f, int v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  if (wave >= NCW) {
    // ---- producer waves: slab j (32 queries x 16 k) into ring slot j % RING.  Thread
    // (p, l) forms entries 128 p + 2 l + y (y = 0, 1): training row k = 16 j + 4 p + l / 16
    // against queries 16 y + l % 16 -- the B fragment of substep p, lane l, column block y
    const int p = wave - NCW;
    const int kk = 4 * p + (lane >> 4);
    double qv[2][D], qn[2];
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int qg = min(c0 + 16 * y + (lane & 15), P - 1);
#pragma unroll
      for (int i = 0; i < D; ++i) qv[y][i] = Qs[(int64_t)qg * D + i];
      qn[y] = Qn[qg];
    }
    // the training rows of the next PF slabs in flight (a register ring, PF-step unrolled)
    constexpr int PF = POST_PF;
    double xr[PF][DP];
    auto load_row = [&](int j, double (&x)[DP]) {
      const int k = min(16 * j + kk, n - 1);
      const double2 *src = (const double2 *)(Xp + (int64_t)k * DP);
#pragma unroll
      for (int i = 0; i < DP / 2; ++i) {
        const double2 v = src[i];
        x[2 * i] = v.x;
        x[2 * i + 1] = v.y;
      }
    };
#pragma unroll
    for (int q = 0; q < PF; ++q) load_row(q, xr[q]);
    int free_upto = RING;  // slots known free: slabs < free_upto may be written
    for (int j0 = 0; j0 < NS; j0 += PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int j = j0 + q;
        if (j < NS) {
          double v[2];
#pragma unroll
          for (int y = 0; y < 2; ++y) {  // the k_gram arithmetic (k_gram_rows): same bits
            double dot = 0.0;
#pragma unroll
            for (int i = 0; i < D; ++i) dot = fma(qv[y][i], xr[q][i], dot);
            const double d2 = (qn[y] + xr[q][D]) - 2.0 * dot;
            v[y] = 16 * j + kk < n ? kernel_epilogue(kind, d2, sigma2, iso_scale) : 0.0;
          }
          if (j + PF < NS) load_row(j + PF, xr[q]);
          if (j >= free_upto)  // every consumer must be done with slot j % RING
            free_upto = wait_all(s_free, NCW, j - RING + 1) + RING;
          *(double2 *)&sK[j % RING][p * 128 + 2 * lane] = make_double2(v[0], v[1]);
          publish(&s_ready[p], j + 1);
        }
      }
    }
  } else {
    // ---- consumer (MFMA) waves: this wave's blocks in slot order (increasing b): the
    // existing ones are a prefix
    int bt[4];
    int T = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bt[t] = wave + 8 * post_slot(h, t);
      if (bt[t] <= NB) T = t + 1;
    }
    const double *wl = Wf + lane * 4;
    // the A fragment of block b at K step j: substeps 2 h2 and 2 h2 + 1 (16 bytes)
    auto frag2 = [&](int j, int b, int h2, double &f0, double &f1) {
      const double2 a = *(const double2 *)(wl + (post_foff(j, NB) + (b - j)) * 256 + 2 * h2);
      f0 = a.x;
      f1 = a.y;
    };
    d4_t acc[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t][0] = acc[t][1] = (d4_t){0.0, 0.0, 0.0, 0.0};
    double fr[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (t < T) {
        frag2(0, bt[t], 0, fr[t][0], fr[t][1]);
        frag2(0, bt[t], 1, fr[t][2], fr[t][3]);
      }
    int j = 0, ready_upto = 0;  // slabs known formed: slabs < ready_upto may be read
// One K step with the live blocks [XF, XL) of this wave (literals: the unrolled loops
// hold no branch around the MFMAs): wait for slab j, its four B fragment reads, the
// MFMAs, slot j released.  A fragment register pair is reloaded with the next step's
// values as soon as its two substeps have issued (one set of fragment registers).  The
// last block XF may die at j + 1: its reload then reads the previous fragment of the
// packed array (in bounds, unused).
#define POST_PHASE(XF, XL, JEND)                                                     \
  for (const int je_ = (JEND); j < je_; ++j) {                                       \
    const double *sl = sK[j % RING];                                                 \
    const bool more = j + 1 < NS;                                                    \
    if (j >= ready_upto) ready_upto = wait_all(s_ready, NPW, j + 1);                 \
    double2 bv[4];                                                                   \
    _Pragma("unroll") for (int s = 0; s < 4; ++s)                                    \
      bv[s] = *(const double2 *)&sl[(s * 64 + lane) * 2];                            \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                  \
      _Pragma("unroll") for (int t = XF; t < XL; ++t) {                              \
        acc[t][0] = mfma_f64(fr[t][s], bv[s].x, acc[t][0]);                          \
        acc[t][1] = mfma_f64(fr[t][s], bv[s].y, acc[t][1]);                          \
      }                                                                              \
      if ((s & 1) && more) {                                                         \
        _Pragma("unroll") for (int t = XF; t < XL; ++t)                              \
          frag2(j + 1, bt[t], s >> 1, fr[t][s - 1], fr[t][s]);                       \
      }                                                                              \
    }                                                                                \
    publish(&s_free[wave], j + 1);                                                   \
  }
#define POST_END(t) min(bt[t] + 1, NS)
    switch (T) {
      case 4:
        POST_PHASE(0, 4, POST_END(0))
        POST_PHASE(1, 4, POST_END(1))
        POST_PHASE(2, 4, POST_END(2))
        POST_PHASE(3, 4, POST_END(3))
        break;
      case 3:
        POST_PHASE(0, 3, POST_END(0))
        POST_PHASE(1, 3, POST_END(1))
        POST_PHASE(2, 3, POST_END(2))
        break;
      case 2:
        POST_PHASE(0, 2, POST_END(0))
        POST_PHASE(1, 2, POST_END(1))
        break;
      case 1:
        POST_PHASE(0, 1, POST_END(0))
        break;
      default:
        break;
    }
#undef POST_END
#undef POST_PHASE
    if (j < NS) publish(&s_free[wave], NS);  // this wave's blocks are done: it releases the rest at once
    // epilogue: per query, the sum of squares over this half's W rows; the mean rows
    double ss[2] = {0.0, 0.0};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < T && bt[t] < NB) {
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r) ss[y] = fma(acc[t][y][r], acc[t][y][r], ss[y]);
      } else if (t < T) {  // the alpha block: row o = lane / 16 + 4 r
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int o = (lane >> 4) + 4 * r, q = c0 + 16 * y + (lane & 15);
            if (o < n_out && q < P) meanT[(int64_t)o * ldm + q] = acc[t][y][r];
          }
      }
    }
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      ss[y] += __shfl_xor(ss[y], 16);
      ss[y] += __shfl_xor(ss[y], 32);
    }
    if (lane < 16) {
      red[wave][lane] = ss[0];
      red[wave][16 + lane] = ss[1];
    }
  }
  __syncthreads();
  if (tid < PQ) {
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < NCW; ++w) v += red[w][tid];
    // an expired wait (never expected) makes the whole group's output NaN, not quietly wrong
    if (s_fail) v = __builtin_nan("");
    if (c0 + tid < P) part[(int64_t)h * ldp + c0 + tid] = v;
  }
}

hipError_t launch_post_cs(hipStream_t s, int n, int n_out, int P, const double *Wf, const double *Xp,
                          const double *Qs, const double *Qn, int d, int kind, double sigma2, double iso_scale,
                          double *part, int64_t ldp, double *meanT, int64_t ldm) {
  if (P <= 0) return hipSuccess;
  if (!post_cs_ok(n, n_out, d)) return hipErrorInvalidValue;
  const int NB = post_cs_blocks(n);
  const dim3 g(2 * ((P + PQ - 1) / PQ));
  switch (d) {
    case 11:
      hipLaunchKernelGGL(k_post_cs<11>, g, dim3(PT), 0, s, n, NB, P, n_out, Wf, Xp, Qs, Qn, kind, sigma2, iso_scale,
                         part, ldp, meanT, ldm);
      break;
    case 12:
      hipLaunchKernelGGL(k_post_cs<12>, g, dim3(PT), 0, s, n, NB, P, n_out, Wf, Xp, Qs, Qn, kind, sigma2, iso_scale,
                         part, ldp, meanT, ldm);
      break;
    default:
      hipLaunchKernelGGL(k_post_cs<13>, g, dim3(PT), 0, s, n, NB, P, n_out, Wf, Xp, Qs, Qn, kind, sigma2, iso_scale,
                         part, ldp, meanT, ldm);
  }
  return hipGetLastError();
}
