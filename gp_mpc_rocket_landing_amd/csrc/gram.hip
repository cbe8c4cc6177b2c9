// gram.hip -- kernel Gram matrices K(X1, X2) in fp64.
//
// Reference: SquaredExponentialARD._compute_scaled_distance_sq / __call__
// (kernels.py:205-262), Matern32/52 (kernels.py:516-545, 610-637) and the
// isotropic SE (kernels.py:417-432).  Like the reference we use the expansion
// form r^2 = |a|^2 + |b|^2 - 2 a.b of the length-scaled rows, clamped at 0.
//
// Layout: a 64 x 64 output tile per 256-thread workgroup.  The 64 a-rows of
// the tile are staged in LDS (read as wave-uniform broadcasts); each thread owns
// one output column (its b-row lives in registers) and 16 rows, so every wave
// stores 64 consecutive doubles (512 B) per row -- fully coalesced.  The
// kernel is HBM-store-bound for n1 = n2 = 1000 (8 MB out, 88 KB in).
#include "internal.h"
#include <cstdlib>

#define GRAM_TILE 64
#define GRAM_MAXD 32

__global__ void k_scale_rows(const double *__restrict__ X, int n, int d,
                             const double *__restrict__ ls, int iso, double *__restrict__ out,
                             double *__restrict__ norms) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int k = 0; k < d; ++k) {
    double v = iso ? X[(int64_t)i * d + k] : X[(int64_t)i * d + k] / ls[k];
    out[(int64_t)i * d + k] = v;
    s += v * v;
  }
  norms[i] = s;
}

hipError_t launch_scale_rows(hipStream_t s, const double *X, int n, int d, const double *ls,
                             int iso, double *out, double *norms) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scale_rows, dim3((n + 255) / 256), dim3(256), 0, s, X, n, d, ls, iso, out,
                     norms);
  return hipGetLastError();
}

template <int D>
__global__ __launch_bounds__(256) void k_gram(int kind, const double *__restrict__ a,
                                              const double *__restrict__ na, int n1,
                                              const double *__restrict__ b,
                                              const double *__restrict__ nb, int n2, int d,
                                              double sigma2, double iso_scale,
                                              double *__restrict__ K, int64_t ldk, int tr) {
  __shared__ double sa[GRAM_TILE][D + 1];
  __shared__ double sna[GRAM_TILE];
  const int r0 = blockIdx.y * GRAM_TILE, c0 = blockIdx.x * GRAM_TILE;
  const int tid = threadIdx.x;
  const int dd = (D > 0) ? D : d;
  for (int e = tid; e < GRAM_TILE * dd; e += 256) {
    int r = e / dd, k = e % dd;
    sa[r][k] = (r0 + r < n1) ? a[(int64_t)(r0 + r) * dd + k] : 0.0;
  }
  if (tid < GRAM_TILE) sna[tid] = (r0 + tid < n1) ? na[r0 + tid] : 0.0;
  const int col = c0 + (tid & 63);
  const int rg = tid >> 6;  // 4 row groups of 16
  double bj[(D > 0) ? D : GRAM_MAXD];
  double nbj = 0.0;
  if (col < n2) {
#pragma unroll
    for (int k = 0; k < ((D > 0) ? D : GRAM_MAXD); ++k)
      bj[k] = (k < dd) ? b[(int64_t)col * dd + k] : 0.0;
    nbj = nb[col];
  }
  __syncthreads();
  if (col >= n2) return;
#pragma unroll 4
  for (int rr = 0; rr < 16; ++rr) {
    const int r = rg * 16 + rr;
    const int row = r0 + r;
    if (row >= n1) break;
    double dot = 0.0;
#pragma unroll
    for (int k = 0; k < ((D > 0) ? D : GRAM_MAXD); ++k)
      if (k < dd) dot = fma(sa[r][k], bj[k], dot);
    double d2 = (sna[r] + nbj) - 2.0 * dot;
    double v = kernel_epilogue(kind, d2, sigma2, iso_scale);
    if (tr) K[(int64_t)col * ldk + row] = v;
    else K[(int64_t)row * ldk + col] = v;
  }
}

// Row-major K (no transpose), compile-time kernel kind and width: 64 columns x
// 128 rows per workgroup (each thread one column, 32 rows, 8 independent
// exponentials in flight), same arithmetic as k_gram (identical bits).
#ifndef GRAM_ROWS
#define GRAM_ROWS 128
#endif
#ifndef GRAM_UNROLL
#define GRAM_UNROLL 8
#endif
#ifndef GRAM_NT
#define GRAM_NT 1
#endif
template <int D, int KIND>
__global__ __launch_bounds__(256) void k_gram_rows(const double *__restrict__ a,
                                                   const double *__restrict__ na, int n1,
                                                   const double *__restrict__ b,
                                                   const double *__restrict__ nb, int n2,
                                                   double sigma2, double iso_scale,
                                                   double *__restrict__ K, int64_t ldk) {
  __shared__ double sa[GRAM_ROWS][D + 1];
  __shared__ double sna[GRAM_ROWS];
  const int r0 = blockIdx.y * GRAM_ROWS, c0 = blockIdx.x * GRAM_TILE;
  const int tid = threadIdx.x;
  for (int e = tid; e < GRAM_ROWS * D; e += 256) {
    const int r = e / D, k = e - r * D;
    sa[r][k] = (r0 + r < n1) ? a[(int64_t)(r0 + r) * D + k] : 0.0;
  }
  if (tid < GRAM_ROWS) sna[tid] = (r0 + tid < n1) ? na[r0 + tid] : 0.0;
  const int col = c0 + (tid & 63);
  constexpr int RPT = GRAM_ROWS / 4;  // rows per thread
  const int rb = (tid >> 6) * RPT;
  double bj[D];
  double nbj = 0.0;
  const bool cv = col < n2;
#pragma unroll
  for (int k = 0; k < D; ++k) bj[k] = cv ? b[(int64_t)col * D + k] : 0.0;
  if (cv) nbj = nb[col];
  __syncthreads();
  if (!cv) return;
  // K* is streamed: written once here, read once by the posterior GEMM from the Infinity
  // Cache / HBM (GRAM_NT: non-temporal stores, no L2 write-allocate).  A full row tile
  // (every tile but the last) stores without the per-row bound test.
  double *Kc = K + (int64_t)(r0 + rb) * ldk + col;
  auto put = [&](int rr, double v) {
#if GRAM_NT
    __builtin_nontemporal_store(v, Kc + (int64_t)rr * ldk);
#else
    Kc[(int64_t)rr * ldk] = v;
#endif
  };
  auto elem = [&](int r) {
    double dot = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) dot = fma(sa[r][k], bj[k], dot);
    const double d2 = (sna[r] + nbj) - 2.0 * dot;
    return kernel_epilogue(KIND, d2, sigma2, iso_scale);
  };
  if (r0 + GRAM_ROWS <= n1) {
#pragma unroll GRAM_UNROLL
    for (int rr = 0; rr < RPT; ++rr) put(rr, elem(rb + rr));
  } else {
#pragma unroll GRAM_UNROLL
    for (int rr = 0; rr < RPT; ++rr) {
      const double v = elem(rb + rr);
      if (r0 + rb + rr < n1) put(rr, v);
    }
  }
}

template <int D>
static hipError_t launch_gram_rows(hipStream_t s, int kind, const double *a, const double *na,
                                   int n1, const double *b, const double *nb, int n2,
                                   double sigma2, double iso_scale, double *K, int64_t ldk) {
  dim3 g((n2 + GRAM_TILE - 1) / GRAM_TILE, (n1 + GRAM_ROWS - 1) / GRAM_ROWS);
  switch (kind) {
    case GPMPC_SE_ARD:
      hipLaunchKernelGGL((k_gram_rows<D, GPMPC_SE_ARD>), g, dim3(256), 0, s, a, na, n1, b, nb, n2,
                         sigma2, iso_scale, K, ldk);
      break;
    case GPMPC_SE_ISO:
      hipLaunchKernelGGL((k_gram_rows<D, GPMPC_SE_ISO>), g, dim3(256), 0, s, a, na, n1, b, nb, n2,
                         sigma2, iso_scale, K, ldk);
      break;
    case GPMPC_MATERN32:
      hipLaunchKernelGGL((k_gram_rows<D, GPMPC_MATERN32>), g, dim3(256), 0, s, a, na, n1, b, nb,
                         n2, sigma2, iso_scale, K, ldk);
      break;
    default:
      hipLaunchKernelGGL((k_gram_rows<D, GPMPC_MATERN52>), g, dim3(256), 0, s, a, na, n1, b, nb,
                         n2, sigma2, iso_scale, K, ldk);
  }
  return hipGetLastError();
}

hipError_t launch_gram(hipStream_t s, int kind, const double *a, const double *na, int n1,
                       const double *b, const double *nb, int n2, int d, double sigma2,
                       double iso_scale, double *K, int64_t ldk, int transpose_out) {
  if (n1 <= 0 || n2 <= 0) return hipSuccess;
  if (d > GRAM_MAXD) return hipErrorInvalidValue;
  static const int rows_env = [] {
    const char *v = getenv("GPMPC_GRAM_ROWS");
    return v ? atoi(v) : 1;
  }();
  if (rows_env && !transpose_out && n1 >= 4 * GRAM_ROWS) {
    if (d == 11) return launch_gram_rows<11>(s, kind, a, na, n1, b, nb, n2, sigma2, iso_scale, K, ldk);
    if (d == 12) return launch_gram_rows<12>(s, kind, a, na, n1, b, nb, n2, sigma2, iso_scale, K, ldk);
    if (d == 13) return launch_gram_rows<13>(s, kind, a, na, n1, b, nb, n2, sigma2, iso_scale, K, ldk);
  }
  dim3 g((n2 + GRAM_TILE - 1) / GRAM_TILE, (n1 + GRAM_TILE - 1) / GRAM_TILE);
  switch (d) {
    case 11:
      hipLaunchKernelGGL(k_gram<11>, g, dim3(256), 0, s, kind, a, na, n1, b, nb, n2, d, sigma2,
                         iso_scale, K, ldk, transpose_out);
      break;
    case 12:
      hipLaunchKernelGGL(k_gram<12>, g, dim3(256), 0, s, kind, a, na, n1, b, nb, n2, d, sigma2,
                         iso_scale, K, ldk, transpose_out);
      break;
    case 13:
      hipLaunchKernelGGL(k_gram<13>, g, dim3(256), 0, s, kind, a, na, n1, b, nb, n2, d, sigma2,
                         iso_scale, K, ldk, transpose_out);
      break;
    default:
      hipLaunchKernelGGL(k_gram<0>, g, dim3(256), 0, s, kind, a, na, n1, b, nb, n2, d, sigma2,
                         iso_scale, K, ldk, transpose_out);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// C-ABI: host buffers in, host buffer out.
extern "C" int gpmpc_gram(gpmpc_ctx *ctx, int kind, const double *X1, int n1, const double *X2,
                          int n2, int d, const double *ls, double sigma2, double *K, int ldk) {
  GPMPC_CHECK_ARG(ctx && X1 && K && ls);
  GPMPC_CHECK_ARG(kind >= 0 && kind <= 3);
  GPMPC_CHECK_ARG(d >= 1 && d <= GRAM_MAXD);
  GPMPC_CHECK_ARG(n1 >= 0);
  if (!X2) n2 = n1;
  GPMPC_CHECK_ARG(n2 >= 0 && ldk >= n2);
  if (n1 == 0 || n2 == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const int iso = (kind == GPMPC_SE_ISO);
  const double iso_scale = iso ? 1.0 / (2.0 * ls[0] * ls[0]) : 0.0;
  DevBuf dX1, dX2, dls, da, db, dna, dnb, dK;
  GPMPC_HIP(dX1.alloc(s, sizeof(double) * n1 * d));
  GPMPC_HIP(dls.alloc(s, sizeof(double) * d));
  GPMPC_HIP(da.alloc(s, sizeof(double) * n1 * d));
  GPMPC_HIP(dna.alloc(s, sizeof(double) * n1));
  GPMPC_HIP(dK.alloc(s, sizeof(double) * (size_t)n1 * n2));
  GPMPC_HIP(hipMemcpyAsync(dX1.p, X1, sizeof(double) * n1 * d, hipMemcpyHostToDevice, s));
  // SE_ISO reads one lengthscale (ls[0]); the host array may hold just that one
  GPMPC_HIP(hipMemcpyAsync(dls.p, ls, sizeof(double) * (iso ? 1 : d), hipMemcpyHostToDevice, s));
  GPMPC_HIP(launch_scale_rows(s, dX1.as<double>(), n1, d, dls.as<double>(), iso, da.as<double>(),
                              dna.as<double>()));
  const double *pb = da.as<double>(), *pnb = dna.as<double>();
  if (X2) {
    GPMPC_HIP(dX2.alloc(s, sizeof(double) * n2 * d));
    GPMPC_HIP(db.alloc(s, sizeof(double) * n2 * d));
    GPMPC_HIP(dnb.alloc(s, sizeof(double) * n2));
    GPMPC_HIP(hipMemcpyAsync(dX2.p, X2, sizeof(double) * n2 * d, hipMemcpyHostToDevice, s));
    GPMPC_HIP(launch_scale_rows(s, dX2.as<double>(), n2, d, dls.as<double>(), iso,
                                db.as<double>(), dnb.as<double>()));
    pb = db.as<double>();
    pnb = dnb.as<double>();
  }
  GPMPC_HIP(launch_gram(s, kind, da.as<double>(), dna.as<double>(), n1, pb, pnb, n2, d, sigma2,
                        iso_scale, dK.as<double>(), n2, 0));
  GPMPC_HIP(hipMemcpy2DAsync(K, sizeof(double) * ldk, dK.p, sizeof(double) * n2,
                             sizeof(double) * n2, n1, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

// ---------------------------------------------------------------------------
// Hyperparameter gradients of the Gram (kernels.py:279-318 SE-ARD, 438-456
// isotropic SE): from K (already formed by launch_gram, so the same bits) and
//   SE-ARD: G_i = K (x1_i - x2_i)^2 / l_i^2   (direct differences, d matrices)
//   SE iso: G   = K r^2 / l^2                  (r^2 of the expansion form)
// one thread per (row, column); every matrix row-major n1 x n2, stacked.
__global__ __launch_bounds__(256) void k_gram_grad(int kind, const double *__restrict__ X1,
                                                   int n1, const double *__restrict__ X2, int n2,
                                                   int d, const double *__restrict__ ls,
                                                   const double *__restrict__ na,
                                                   const double *__restrict__ nb,
                                                   const double *__restrict__ K,
                                                   double *__restrict__ G) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x, row = blockIdx.y;
  if (col >= n2) return;
  const int64_t e = (int64_t)row * n2 + col, plane = (int64_t)n1 * n2;
  const double k = K[e];
  const double *a = X1 + (int64_t)row * d, *b = X2 + (int64_t)col * d;
  if (kind == GPMPC_SE_ARD) {
    for (int i = 0; i < d; ++i) {
      const double df = a[i] - b[i];
      G[i * plane + e] = k * ((df * df) / (ls[i] * ls[i]));
    }
  } else {  // isotropic: rows unscaled, r^2 as k_gram forms it
    double dot = 0.0;
    for (int i = 0; i < d; ++i) dot = fma(a[i], b[i], dot);
    double d2 = (na[row] + nb[col]) - 2.0 * dot;
    d2 = d2 > 0.0 ? d2 : 0.0;
    G[e] = (k * d2) / (ls[0] * ls[0]);
  }
}

extern "C" int gpmpc_gram_grad(gpmpc_ctx *ctx, int kind, const double *X1, int n1, const double *X2,
                               int n2, int d, const double *ls, double sigma2, double *K, double *G) {
  GPMPC_CHECK_ARG(ctx && X1 && ls && G);
  GPMPC_CHECK_ARG(kind == GPMPC_SE_ARD || kind == GPMPC_SE_ISO);
  GPMPC_CHECK_ARG(d >= 1 && d <= GRAM_MAXD && n1 >= 0);
  if (!X2) n2 = n1;
  GPMPC_CHECK_ARG(n2 >= 0);
  if (n1 == 0 || n2 == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const int iso = (kind == GPMPC_SE_ISO);
  const double iso_scale = iso ? 1.0 / (2.0 * ls[0] * ls[0]) : 0.0;
  const int ng = iso ? 1 : d;
  const size_t nn = (size_t)n1 * n2;
  DevBuf dX1, dX2, dls, da, db, dna, dnb, dK, dG;
  GPMPC_HIP(dX1.alloc(s, sizeof(double) * n1 * d));
  GPMPC_HIP(dls.alloc(s, sizeof(double) * d));
  GPMPC_HIP(da.alloc(s, sizeof(double) * n1 * d));
  GPMPC_HIP(dna.alloc(s, sizeof(double) * n1));
  GPMPC_HIP(dK.alloc(s, sizeof(double) * nn));
  GPMPC_HIP(dG.alloc(s, sizeof(double) * nn * ng));
  GPMPC_HIP(hipMemcpyAsync(dX1.p, X1, sizeof(double) * n1 * d, hipMemcpyHostToDevice, s));
  // SE_ISO reads one lengthscale (ls[0]); the host array may hold just that one
  GPMPC_HIP(hipMemcpyAsync(dls.p, ls, sizeof(double) * (iso ? 1 : d), hipMemcpyHostToDevice, s));
  GPMPC_HIP(launch_scale_rows(s, dX1.as<double>(), n1, d, dls.as<double>(), iso, da.as<double>(),
                              dna.as<double>()));
  const double *pX2 = dX1.as<double>(), *pb = da.as<double>(), *pnb = dna.as<double>();
  if (X2) {
    GPMPC_HIP(dX2.alloc(s, sizeof(double) * n2 * d));
    GPMPC_HIP(db.alloc(s, sizeof(double) * n2 * d));
    GPMPC_HIP(dnb.alloc(s, sizeof(double) * n2));
    GPMPC_HIP(hipMemcpyAsync(dX2.p, X2, sizeof(double) * n2 * d, hipMemcpyHostToDevice, s));
    GPMPC_HIP(launch_scale_rows(s, dX2.as<double>(), n2, d, dls.as<double>(), iso,
                                db.as<double>(), dnb.as<double>()));
    pX2 = dX2.as<double>(); pb = db.as<double>(); pnb = dnb.as<double>();
  }
  GPMPC_HIP(launch_gram(s, kind, da.as<double>(), dna.as<double>(), n1, pb, pnb, n2, d, sigma2,
                        iso_scale, dK.as<double>(), n2, 0));
  hipLaunchKernelGGL(k_gram_grad, dim3((n2 + 255) / 256, n1), dim3(256), 0, s, kind,
                     dX1.as<double>(), n1, pX2, n2, d, dls.as<double>(), dna.as<double>(), pnb,
                     dK.as<double>(), dG.as<double>());
  GPMPC_HIP(hipGetLastError());
  if (K) GPMPC_HIP(hipMemcpyAsync(K, dK.p, sizeof(double) * nn, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipMemcpyAsync(G, dG.p, sizeof(double) * nn * ng, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

// ---------------------------------------------------------------------------
// Composite kernels (kernels.py:676-844: SumKernel, ProductKernel, WhiteNoise over the
// stationary kernels) as a postfix program of (code, parameter offset) pairs:
//   GPMPC_SE_ARD / _MATERN32 / _MATERN52: par[off] = sigma2, par[off + 1 ..] = the d
//     lengthscales (expansion-form distance of the scaled rows, clamped at 0, as k_gram)
//   GPMPC_SE_ISO: par[off] = sigma2, par[off + 1] = l (distance of the raw rows)
//   GPMPC_KP_WHITE: par[off] = sigma2 on the diagonal of a Gram of one row set (X2 None
//     in the reference), zero between two sets
//   GPMPC_KP_SUM / GPMPC_KP_PROD: the two values on top of the stack
// Rows are raw.  One thread per entry: the composite Grams are fit/predict-time work.
__device__ double kprog_leaf(int code, const double *__restrict__ p, const double *__restrict__ a,
                             const double *__restrict__ b, int d, bool diag_entry) {
  if (code == GPMPC_KP_WHITE) return diag_entry ? p[0] : 0.0;
  double na = 0.0, nb = 0.0, dot = 0.0;
  if (code == GPMPC_SE_ISO) {
    for (int i = 0; i < d; ++i) {
      na = fma(a[i], a[i], na);
      nb = fma(b[i], b[i], nb);
      dot = fma(a[i], b[i], dot);
    }
    const double l = p[1];
    return kernel_epilogue(GPMPC_SE_ISO, (na + nb) - 2.0 * dot, p[0], 1.0 / (2.0 * l * l));
  }
  for (int i = 0; i < d; ++i) {
    const double x = a[i] / p[1 + i], y = b[i] / p[1 + i];
    na = fma(x, x, na);
    nb = fma(y, y, nb);
    dot = fma(x, y, dot);
  }
  return kernel_epilogue(code, (na + nb) - 2.0 * dot, p[0], 0.0);
}

__global__ void k_gram_prog(const int *__restrict__ ops, int nops, const double *__restrict__ par,
                            const double *__restrict__ X1, int n1, const double *__restrict__ X2, int n2, int d,
                            int same, double *__restrict__ K, int64_t ldk) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x, row = blockIdx.y;
  if (col >= n2 || row >= n1) return;
  const double *a = X1 + (int64_t)row * d, *b = X2 + (int64_t)col * d;
  double st[GPMPC_KP_MAXSTACK];
  int sp = 0;
  for (int o = 0; o < nops; ++o) {
    const int code = ops[2 * o], off = ops[2 * o + 1];
    if (code == GPMPC_KP_SUM) { st[sp - 2] = st[sp - 2] + st[sp - 1]; --sp; }
    else if (code == GPMPC_KP_PROD) { st[sp - 2] = st[sp - 2] * st[sp - 1]; --sp; }
    else st[sp++] = kprog_leaf(code, par + off, a, b, d, same && row == col);
  }
  K[(int64_t)row * ldk + col] = st[0];
}

hipError_t launch_gram_prog(hipStream_t s, const int *ops, int nops, const double *par, const double *X1, int n1,
                            const double *X2, int n2, int d, int same, double *K, int64_t ldk) {
  if (n1 <= 0 || n2 <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gram_prog, dim3((n2 + 127) / 128, n1), dim3(128), 0, s, ops, nops, par, X1, n1,
                     same ? X1 : X2, n2, d, same, K, ldk);
  return hipGetLastError();
}

// Host checks of a program (stack depth, operand counts, offsets in range, d lengthscales
// > 0); its diagonal k(x, x): every leaf's is its sigma2 (stationary kernels, white noise),
// so the diagonal of a composite is one constant (kernels.py diagonal methods)
int kprog_check(const int *ops, int nops, int npar, int d, const double *par, double *diag) {
  if (!ops || !par || nops < 1 || nops > GPMPC_KP_MAXOPS) return -2;
  double st[GPMPC_KP_MAXSTACK];
  int sp = 0;
  for (int o = 0; o < nops; ++o) {
    const int code = ops[2 * o], off = ops[2 * o + 1];
    if (code == GPMPC_KP_SUM || code == GPMPC_KP_PROD) {
      if (sp < 2) return -2;
      st[sp - 2] = code == GPMPC_KP_SUM ? st[sp - 2] + st[sp - 1] : st[sp - 2] * st[sp - 1];
      --sp;
      continue;
    }
    const int np = code == GPMPC_KP_WHITE ? 1 : code == GPMPC_SE_ISO ? 2
                 : (code == GPMPC_SE_ARD || code == GPMPC_MATERN32 || code == GPMPC_MATERN52) ? 1 + d : -1;
    if (np < 0 || off < 0 || off + np > npar || sp >= GPMPC_KP_MAXSTACK) return -2;
    if (!(par[off] >= 0.0)) return -2;
    for (int i = 1; i < np; ++i)
      if (!(par[off + i] > 0.0)) return -2;
    st[sp++] = par[off];
  }
  if (sp != 1) return -2;
  if (diag) *diag = st[0];
  return 0;
}
