// gp.hip -- exact GP and FITC sparse GP on the device.
//
// Exact GP (MultiOutputExactGP.fit -> ExactGP.fit, exact_gp.py:118-204, 476-499):
// the n_out outputs share one kernel and one X, so a single Gram, a single
// Cholesky (with the exact_gp.py:163-175 jitter ladder) and a single
// W = L^-1 serve every output.  alpha = cho_solve(L, y_c) for all
// outputs at once (n x n_out right-hand sides).
//
// Posterior (ExactGP.predict, exact_gp.py:213-268):
//   K*   = k(X*, X)                          (gram kernel, P x n)
//   mean = K* alpha * y_std + y_mean          (NT GEMM, alpha^T as A)
//   var  = max(sigma2 - colsum((W K*^T)^2), 1e-10) * y_std^2
// where the sum of squares is fused into the GEMM epilogue (gemm.hip).
#include "internal.h"
#include "gemm.h"
#include <cmath>
#include <vector>

struct GpCore {
  int kind = 0, n = 0, d = 0, n_out = 0;
  double sigma2 = 1.0, iso_scale = 0.0;
  DevBuf ls, Xs, Xn;   // scaled training rows, squared norms
  DevBuf W;            // n x n, L^-1 (lower)
  DevBuf alphaT;       // n_out x n
  DevBuf ymean, ystd;  // n_out
  std::vector<double> h_ymean, h_ystd;
  // the column-stationary posterior's operands (post.hip, exact GPs with n <= 1008):
  // [W; alpha^T] in packed MFMA-fragment order and the scaled rows padded with their norms
  DevBuf Wf, Xp;
  // composite kernel (kind == GPMPC_KPROG): the postfix program (gpmpc.h GPMPC_KP_*);
  // Xs then holds the raw rows, Xn zeros, and sigma2 the program's diagonal constant
  DevBuf ops, par;
  int nops = 0;
};

// a composite kernel program as the entry points receive it (host arrays)
struct KProgArg {
  const int *ops;
  int nops;
  const double *par;
  int npar;
};

struct gpmpc_gp {
  GpCore core;
  DevBuf L;  // n x n lower Cholesky factor
  double noise = 1e-4;
  int jitter_steps = 0;
};

struct gpmpc_fitc {
  GpCore core;  // core.Xs = scaled inducing rows (m), W = L_uu^-1, alphaT, ...
  DevBuf W2;    // m x m, L_B^-1 L_uu^-1 (lower): w = L_B^-1 v = W2 k*
  int m = 0;
};

// ---------------------------------------------------------------------------
__global__ void k_eye(int n, double *A) {
  int j = blockIdx.x * blockDim.x + threadIdx.x, i = blockIdx.y;
  if (j < n) A[(int64_t)i * n + j] = (i == j) ? 1.0 : 0.0;
}

// finish the posterior: var (P x n_out), mean (P x n_out) from partials
__global__ void k_post_finish(int P, int n_out, int nrt, const double *__restrict__ part,
                              int64_t ldp, const double *__restrict__ meanT, int64_t ldm,
                              const double *__restrict__ ymean, const double *__restrict__ ystd,
                              double sigma2, double *__restrict__ mean, double *__restrict__ var) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= P) return;
  double ss = 0.0;
  for (int t = 0; t < nrt; ++t) ss += part[(int64_t)t * ldp + j];
  double lat = sigma2 - ss;
  lat = lat > 1e-10 ? lat : 1e-10;
  for (int c = 0; c < n_out; ++c) {
    if (mean) mean[(int64_t)j * n_out + c] = meanT[(int64_t)c * ldm + j] * ystd[c] + ymean[c];
    if (var) var[(int64_t)j * n_out + c] = lat * ystd[c] * ystd[c];
  }
}

hipError_t launch_post_finish(hipStream_t s, int P, int n_out, int nrt, const double *part,
                              int64_t ldp, const double *meanT, int64_t ldm, const double *ymean,
                              const double *ystd, double sigma2, double *mean, double *var) {
  hipLaunchKernelGGL(k_post_finish, dim3((P + 255) / 256), dim3(256), 0, s, P, n_out, nrt, part,
                     ldp, meanT, ldm, ymean, ystd, sigma2, mean, var);
  return hipGetLastError();
}

// FITC: pv / pw hold per-row-tile column sums of v^2 (v = Luu^-1 k*) and w^2 (w = W2 k*).
__global__ void k_fitc_finish(int P, int n_out, int nrv, int nrw, const double *__restrict__ pv,
                              const double *__restrict__ pw, int64_t ldp,
                              const double *__restrict__ meanT, int64_t ldm,
                              const double *__restrict__ ymean, const double *__restrict__ ystd,
                              double sigma2, double *__restrict__ mean, double *__restrict__ var) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= P) return;
  double sv = 0.0, sw = 0.0;
  for (int t = 0; t < nrv; ++t) sv += pv[(int64_t)t * ldp + j];
  for (int t = 0; t < nrw; ++t) sw += pw[(int64_t)t * ldp + j];
  double lat = sigma2 - sv + sw;
  lat = lat > 1e-10 ? lat : 1e-10;
  for (int c = 0; c < n_out; ++c) {
    mean[(int64_t)j * n_out + c] = meanT[(int64_t)c * ldm + j] * ystd[c] + ymean[c];
    var[(int64_t)j * n_out + c] = lat * ystd[c] * ystd[c];
  }
}

// column scaling: A[i][j] *= s[j]
__global__ void k_scale_cols(int rows, int cols, double *A, int64_t lda, const double *s) {
  int j = blockIdx.x * blockDim.x + threadIdx.x, i = blockIdx.y;
  if (j < cols) A[(int64_t)i * lda + j] *= s[j];
}

// ---------------------------------------------------------------------------
// small device reductions (all GP arithmetic stays on the device)
__device__ double block_sum(double v, double *red) {
  const int tid = threadIdx.x;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
  return t;
}

// exact_gp.py:141-150: per output column, mean / population std (std < 1e-10 -> 1)
__global__ __launch_bounds__(256) void k_normalise(int n, int n_out, const double *Y, double *yn,
                                                   double *ymean, double *ystd) {
  __shared__ double red[4];
  const int c = blockIdx.x;
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += Y[(int64_t)i * n_out + c];
  const double m = block_sum(s, red) / n;
  double q = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    double t = Y[(int64_t)i * n_out + c] - m;
    q += t * t;
  }
  double sd = sqrt(block_sum(q, red) / n);
  if (sd < 1e-10) sd = 1.0;
  for (int i = threadIdx.x; i < n; i += 256) yn[(int64_t)i * n_out + c] = (Y[(int64_t)i * n_out + c] - m) / sd;
  if (threadIdx.x == 0) { ymean[c] = m; ystd[c] = sd; }
}

// exact_gp.py:186-204: lml_c = -1/2 y_c.alpha_c - sum log L_ii - n/2 log 2 pi; also alpha^T
__global__ __launch_bounds__(256) void k_lml_exact(int n, int n_out, const double *L,
                                                   const double *yn, const double *alpha,
                                                   double *alphaT, double *lml) {
  __shared__ double red[4];
  const int c = blockIdx.x;
  double ld = 0.0, fit = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    ld += log(L[(int64_t)i * n + i]);
    const double a = alpha[(int64_t)i * n_out + c];
    fit += yn[(int64_t)i * n_out + c] * a;
    alphaT[(int64_t)c * n + i] = a;
  }
  ld = block_sum(ld, red);
  fit = block_sum(fit, red);
  if (threadIdx.x == 0) lml[c] = -0.5 * fit - ld - 0.5 * n * log(2.0 * M_PI);
}

// FITC Lambda (sparse_gp.py:193-199): lam_j = max(sigma2 - sum_i A_ij^2 + noise, 1e-10)
__global__ void k_fitc_lambda(int m, int n, const double *A, double sigma2, double noise,
                              double *lam, double *isq) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double q = 0.0;
  for (int i = 0; i < m; ++i) q += A[(int64_t)i * n + j] * A[(int64_t)i * n + j];
  double v = sigma2 - q + noise;
  v = v > 1e-10 ? v : 1e-10;
  lam[j] = v;
  isq[j] = 1.0 / sqrt(v);
}

// yl[c][j] = yn[j][c] / lam[j]
__global__ void k_fitc_yl(int n, int n_out, const double *yn, const double *lam, double *yl) {
  int j = blockIdx.x * blockDim.x + threadIdx.x, c = blockIdx.y;
  if (j < n) yl[(int64_t)c * n + j] = yn[(int64_t)j * n_out + c] / lam[j];
}

// FITC lml (sparse_gp.py:212-218) and alpha^T
__global__ __launch_bounds__(256) void k_lml_fitc(int m, int n, int n_out, const double *LB,
                                                  const double *yn, const double *lam,
                                                  const double *cvec, const double *alpha,
                                                  double *alphaT, double *lml) {
  __shared__ double red[4];
  const int c = blockIdx.x;
  double ldb = 0.0, ca = 0.0, yly = 0.0, ll = 0.0;
  for (int i = threadIdx.x; i < m; i += 256) {
    ldb += log(LB[(int64_t)i * m + i]);
    const double a = alpha[(int64_t)i * n_out + c];
    ca += cvec[(int64_t)i * n_out + c] * a;
    alphaT[(int64_t)c * m + i] = a;
  }
  for (int j = threadIdx.x; j < n; j += 256) {
    const double y = yn[(int64_t)j * n_out + c];
    yly += y * y / lam[j];
    ll += log(lam[j]);
  }
  ldb = block_sum(ldb, red);
  ca = block_sum(ca, red);
  yly = block_sum(yly, red);
  ll = block_sum(ll, red);
  if (threadIdx.x == 0) lml[c] = -0.5 * (yly - ca) - ldb - 0.5 * ll - 0.5 * n * log(2.0 * M_PI);
}

static int core_setup(gpmpc_ctx *ctx, GpCore &g, int kind, const double *X, int n, int d,
                      const double *ls, double sigma2, const KProgArg *prog = nullptr) {
  hipStream_t s = ctx->stream;
  g.kind = prog ? GPMPC_KPROG : kind;
  g.n = n;
  g.d = d;
  g.sigma2 = sigma2;
  if (prog) {
    double diag = 0.0;
    if (kprog_check(prog->ops, prog->nops, prog->npar, d, prog->par, &diag)) {
      gpmpc_set_error("composite kernel program is malformed (codes, offsets, stack, parameters)");
      return -2;
    }
    g.sigma2 = diag;  // k(x, x) of the program: the posterior's and FITC's prior variance
    g.iso_scale = 0.0;
    g.nops = prog->nops;
    GPMPC_HIP(g.ops.alloc(s, sizeof(int) * 2 * prog->nops));
    GPMPC_HIP(g.par.alloc(s, sizeof(double) * prog->npar));
    GPMPC_HIP(g.Xs.alloc(s, sizeof(double) * n * d));
    GPMPC_HIP(g.Xn.alloc(s, sizeof(double) * n));
    GPMPC_HIP(hipMemcpyAsync(g.ops.p, prog->ops, sizeof(int) * 2 * prog->nops, hipMemcpyHostToDevice, s));
    GPMPC_HIP(hipMemcpyAsync(g.par.p, prog->par, sizeof(double) * prog->npar, hipMemcpyHostToDevice, s));
    GPMPC_HIP(hipMemcpyAsync(g.Xs.p, X, sizeof(double) * n * d, hipMemcpyHostToDevice, s));
    GPMPC_HIP(hipMemsetAsync(g.Xn.p, 0, sizeof(double) * n, s));
    GPMPC_HIP(hipStreamSynchronize(s));
    return 0;
  }
  const int iso = (kind == GPMPC_SE_ISO);
  g.iso_scale = iso ? 1.0 / (2.0 * ls[0] * ls[0]) : 0.0;
  DevBuf dX;
  GPMPC_HIP(dX.alloc(s, sizeof(double) * n * d));
  GPMPC_HIP(g.ls.alloc(s, sizeof(double) * d));
  GPMPC_HIP(g.Xs.alloc(s, sizeof(double) * n * d));
  GPMPC_HIP(g.Xn.alloc(s, sizeof(double) * n));
  GPMPC_HIP(hipMemcpyAsync(dX.p, X, sizeof(double) * n * d, hipMemcpyHostToDevice, s));
  // SE_ISO reads one lengthscale (ls[0]); the host array may hold just that one
  GPMPC_HIP(hipMemcpyAsync(g.ls.p, ls, sizeof(double) * (iso ? 1 : d), hipMemcpyHostToDevice, s));
  GPMPC_HIP(launch_scale_rows(s, dX.as<double>(), n, d, g.ls.as<double>(), iso, g.Xs.as<double>(),
                              g.Xn.as<double>()));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

// the core's form of device rows (p x d, raw in) for its Grams: scaled by the lengthscales
// with squared norms, or raw (norms zero) for a composite program
static hipError_t core_rows(hipStream_t s, const GpCore &g, const double *Xraw, int p, double *A, double *NA) {
  if (g.kind == GPMPC_KPROG) {
    hipError_t e = hipMemcpyAsync(A, Xraw, sizeof(double) * p * g.d, hipMemcpyDeviceToDevice, s);
    return e == hipSuccess ? hipMemsetAsync(NA, 0, sizeof(double) * p, s) : e;
  }
  return launch_scale_rows(s, Xraw, p, g.d, g.ls.as<double>(), g.kind == GPMPC_SE_ISO, A, NA);
}

// K (n1 x n2, ldk) between core-form rows; same = 1: one row set (B ignored for a program,
// whose WhiteNoise leaves then sit on the diagonal -- kernel(X) vs kernel(X1, X2))
static hipError_t core_gram(hipStream_t s, const GpCore &g, const double *A, const double *NA, int n1,
                            const double *B, const double *NB, int n2, int same, double *K, int64_t ldk) {
  if (g.kind == GPMPC_KPROG)
    return launch_gram_prog(s, g.ops.as<int>(), g.nops, g.par.as<double>(), A, n1, B, n2, g.d, same, K, ldk);
  return launch_gram(s, g.kind, A, NA, n1, B, NB, n2, g.d, g.sigma2, g.iso_scale, K, ldk, 0);
}

// GPMPC_POST_CS=1: the column-stationary posterior (post.hip) instead of K* in HBM (gram +
// 128-tile SUMSQ GEMM).  Off by default: measured slower at the bench workload (DESIGN.md
// section 3).  Read at every fit and predict, so a process can switch it between handles.
bool post_cs_env() {
  const char *e = getenv("GPMPC_POST_CS");
  return e && atoi(e) != 0;
}

// Wf / Xp for the column-stationary posterior (post.hip) from the current [W; alpha^T],
// Xs, Xn; released when the GP is outside the kernel's range
static hipError_t core_pack(hipStream_t s, GpCore &g) {
  if (g.kind == GPMPC_KPROG || !post_cs_env() || !post_cs_ok(g.n, g.n_out, g.d)) {
    g.Wf.release();
    g.Xp.release();
    return hipSuccess;
  }
  hipError_t e = g.Wf.alloc(s, sizeof(double) * post_cs_frag_doubles(g.n));
  if (e == hipSuccess) e = g.Xp.alloc(s, sizeof(double) * (size_t)g.n * post_cs_row_pitch(g.d));
  if (e == hipSuccess)
    e = launch_post_pack(s, g.n, g.n_out, g.W.as<double>(), g.n, g.Xs.as<double>(), g.Xn.as<double>(), g.d,
                         g.Wf.as<double>(), g.Xp.as<double>());
  return e;
}

// K* = k(Xq, X_core) (p x n) on device from host queries; returns scaled queries too
static int core_cross(gpmpc_ctx *ctx, const GpCore &g, const double *dXq_raw, int p, DevBuf &Ks,
                      DevBuf *qs = nullptr, DevBuf *qn = nullptr) {
  hipStream_t s = ctx->stream;
  DevBuf a, na;
  DevBuf &A = qs ? *qs : a;
  DevBuf &NA = qn ? *qn : na;
  GPMPC_HIP(A.alloc(s, sizeof(double) * p * g.d));
  GPMPC_HIP(NA.alloc(s, sizeof(double) * p));
  GPMPC_HIP(core_rows(s, g, dXq_raw, p, A.as<double>(), NA.as<double>()));
  GPMPC_HIP(Ks.alloc(s, sizeof(double) * (size_t)p * g.n));
  GPMPC_HIP(core_gram(s, g, A.as<double>(), NA.as<double>(), p, g.Xs.as<double>(), g.Xn.as<double>(), g.n, 0,
                      Ks.as<double>(), g.n));
  return 0;
}

// ---------------------------------------------------------------------------
// bump allocator over a persistent scratch slot (gp_append temporaries)
struct ScratchCarve {
  double *base;
  size_t off = 0;
  double *take(size_t count) { double *p = base + off; off += (count + 31) & ~(size_t)31; return p; }
};
struct ScratchPtr {
  double *p;
  template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

// alpha = L^-T L^-1 y for the few output columns of an exact fit (exact_gp.py:179,
// cho_solve): one workgroup per column with the vector in LDS, by 32-row blocks.
// Forward: wave 0 solves the block's triangle in registers (readlane broadcasts),
// then all 256 threads subtract L[r, blk] x_blk from the rows below (each row's 32
// block entries contiguous).  Backward (L^T): wave 0 back-substitutes the block with
// L_bb^T, then x[r] -= sum_j L[r0 + j][r] x_j for the rows above (consecutive threads,
// consecutive r: coalesced).  The blocked TRSM it replaces walked 2 x 8 panel
// launches of ~70 us each for 3 columns (fit breakdown).
#define POTRS_COLS_MAXN 16384
__global__ __launch_bounds__(256) void k_potrs_cols(int n, const double *__restrict__ L,
                                                    int64_t ldl, double *__restrict__ Y,
                                                    int n_out) {
  const int c = blockIdx.x;
  extern __shared__ double x[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int i = tid; i < n; i += 256) x[i] = Y[(int64_t)i * n_out + c];
  __syncthreads();
  for (int r0 = 0; r0 < n; r0 += 32) {
    const int nb = min(32, n - r0);
    if (wave == 0) {
      double a[32];
#pragma unroll
      for (int j = 0; j < 32; ++j)
        a[j] = (lane < nb && j <= lane) ? L[(int64_t)(r0 + lane) * ldl + r0 + j] : 1.0;
      double sv = lane < nb ? x[r0 + lane] : 0.0;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        if (j < nb) {
          if (lane == j) sv = sv / a[j];
          const double xj = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(sv), j),
                                             __builtin_amdgcn_readlane(__double2loint(sv), j));
          if (lane > j) sv = fma(-a[j], xj, sv);
        }
      }
      if (lane < nb) x[r0 + lane] = sv;
    }
    __syncthreads();
    const int r1 = r0 + nb;
    if (r1 < n) {
      double xb[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) xb[j] = x[r0 + j];  // nb = 32 whenever rows remain below
      for (int r = r1 + tid; r < n; r += 256) {
        const double *row = L + (int64_t)r * ldl + r0;
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < 32; ++j) acc = fma(row[j], xb[j], acc);
        x[r] -= acc;
      }
    }
    __syncthreads();
  }
  for (int r0 = ((n - 1) / 32) * 32; r0 >= 0; r0 -= 32) {
    const int nb = min(32, n - r0);
    if (wave == 0) {
      double a[32];  // a[j] = (L_bb^T)[lane][j] = L[r0 + j][r0 + lane], j >= lane
#pragma unroll
      for (int j = 0; j < 32; ++j)
        a[j] = (lane < nb && j < nb && j >= lane) ? L[(int64_t)(r0 + j) * ldl + r0 + lane] : 1.0;
      double sv = lane < nb ? x[r0 + lane] : 0.0;
#pragma unroll
      for (int j = 31; j >= 0; --j) {
        if (j < nb) {
          if (lane == j) sv = sv / a[j];
          const double xj = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(sv), j),
                                             __builtin_amdgcn_readlane(__double2loint(sv), j));
          if (lane < j) sv = fma(-a[j], xj, sv);
        }
      }
      if (lane < nb) x[r0 + lane] = sv;
    }
    __syncthreads();
    if (r0 > 0) {
      double xb[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) xb[j] = j < nb ? x[r0 + j] : 0.0;
      for (int r = tid; r < r0; r += 256) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if (j < nb) acc = fma(L[(int64_t)(r0 + j) * ldl + r], xb[j], acc);
        x[r] -= acc;
      }
    }
    __syncthreads();
  }
  for (int i = tid; i < n; i += 256) Y[(int64_t)i * n_out + c] = x[i];
}

// ---------------------------------------------------------------------------
// cho_solve through the inverse the fit forms anyway (exact fits, W = L^-1):
//   alpha1 = W^T (W y);  r = y - L (L^T alpha1);  alpha = alpha1 + W^T (W r)
// One step of iterative refinement against the factor makes the explicit-inverse
// solve as accurate as the two substitutions (exact_gp.py:179, cho_solve); six
// triangular matrix x (n x nc) products that fill the device instead of one
// serial substitution per output column on one CU (k_potrs_cols, ~0.77 ms at n = 1000).
// Both forms sum in a fixed order (no atomics): results are bit-reproducible.

// y = base + sgn * T x   (T lower n x n, row-major; x, y, base n x nc row-major, nc <= 16):
// one wave per row, lanes striding the row's columns, then a wave reduction
__global__ __launch_bounds__(256) void k_trmv_n(int n, int nc, const double *__restrict__ T, int64_t ldt,
                                                const double *__restrict__ x, const double *__restrict__ base,
                                                double sgn, double *__restrict__ y) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n) return;
  double acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = 0.0;
  const double *tr = T + (int64_t)row * ldt;
  for (int j = lane; j <= row; j += 64) {
    const double t = tr[j];
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (c < nc) acc[c] = fma(t, x[(int64_t)j * nc + c], acc[c]);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    if (c < nc) {
      double v = acc[c];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      acc[c] = v;
    }
  }
  if (lane < nc) {
    double v = 0.0;
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (c == lane) v = acc[c];
    y[(int64_t)row * nc + lane] = (base ? base[(int64_t)row * nc + lane] : 0.0) + sgn * v;
  }
}

// partial sums of T^T x over 32-row blocks: part[rb][j][c] = sum_{i in rb, i >= j} T[i][j] x[i][c]
#define TRMV_T_RB 32
__global__ __launch_bounds__(256) void k_trmv_t_part(int n, int nc, const double *__restrict__ T, int64_t ldt,
                                                     const double *__restrict__ x, double *__restrict__ part) {
  const int j = blockIdx.x * 256 + threadIdx.x, rb = blockIdx.y;
  const int i0 = rb * TRMV_T_RB, i1 = min(n, i0 + TRMV_T_RB);
  if (j >= n) return;
  double acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = 0.0;
  for (int i = max(i0, j); i < i1; ++i) {
    const double t = T[(int64_t)i * ldt + j];
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (c < nc) acc[c] = fma(t, x[(int64_t)i * nc + c], acc[c]);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c)
    if (c < nc) part[((int64_t)rb * n + j) * nc + c] = acc[c];
}

// y = base + sgn * sum_rb part[rb]   (row blocks summed in order)
__global__ void k_trmv_t_sum(int n, int nc, int nrb, const double *__restrict__ part,
                             const double *__restrict__ base, double sgn, double *__restrict__ y) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n * nc) return;
  const int j = e / nc;
  double v = 0.0;
  for (int rb = j / TRMV_T_RB; rb < nrb; ++rb) v += part[(int64_t)rb * n * nc + e];
  y[e] = (base ? base[e] : 0.0) + sgn * v;
}

static hipError_t launch_trmv(hipStream_t s, int trans, int n, int nc, const double *T, int64_t ldt,
                              const double *x, const double *base, double sgn, double *y, double *part) {
  if (!trans) {
    hipLaunchKernelGGL(k_trmv_n, dim3((n + 3) / 4), dim3(256), 0, s, n, nc, T, ldt, x, base, sgn, y);
  } else {
    const int nrb = (n + TRMV_T_RB - 1) / TRMV_T_RB;
    hipLaunchKernelGGL(k_trmv_t_part, dim3((n + 255) / 256, nrb), dim3(256), 0, s, n, nc, T, ldt, x, part);
    hipLaunchKernelGGL(k_trmv_t_sum, dim3((n * nc + 255) / 256), dim3(256), 0, s, n, nc, nrb, part, base,
                       sgn, y);
  }
  return hipGetLastError();
}

// Y (n x nc, in place) <- (L L^T)^-1 Y with W = L^-1 formed; scratch from the stream pool
static hipError_t cho_solve_inv(hipStream_t s, int n, int nc, const double *L, const double *W, double *Y) {
  const int nrb = (n + TRMV_T_RB - 1) / TRMV_T_RB;
  DevBuf v, a1, t, part;
  hipError_t e;
  if ((e = v.alloc(s, sizeof(double) * n * nc)) || (e = a1.alloc(s, sizeof(double) * n * nc)) ||
      (e = t.alloc(s, sizeof(double) * n * nc)) || (e = part.alloc(s, sizeof(double) * (size_t)nrb * n * nc)))
    return e;
  double *pv = v.as<double>(), *pa = a1.as<double>(), *pt = t.as<double>(), *pp = part.as<double>();
  if ((e = launch_trmv(s, 0, n, nc, W, n, Y, nullptr, 1.0, pv, pp)) ||       // v = W y
      (e = launch_trmv(s, 1, n, nc, W, n, pv, nullptr, 1.0, pa, pp)) ||      // alpha1 = W^T v
      (e = launch_trmv(s, 1, n, nc, L, n, pa, nullptr, 1.0, pt, pp)) ||      // t = L^T alpha1
      (e = launch_trmv(s, 0, n, nc, L, n, pt, Y, -1.0, pv, pp)) ||           // r = y - L t
      (e = launch_trmv(s, 0, n, nc, W, n, pv, nullptr, 1.0, pt, pp)) ||      // w = W r
      (e = launch_trmv(s, 1, n, nc, W, n, pt, pa, 1.0, Y, pp)))              // alpha = alpha1 + W^T w
    return e;
  return hipSuccess;
}

static bool potrs_cols_ok(int n) {
  static const int env = [] {
    const char *e = getenv("GPMPC_POTRS_COLS");
    return e ? atoi(e) : 1;
  }();
  static const bool attr = hipFuncSetAttribute((const void *)k_potrs_cols,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)(sizeof(double) * POTRS_COLS_MAXN)) == hipSuccess;
  return env && attr && n <= POTRS_COLS_MAXN;
}

static int exact_fit(gpmpc_ctx *ctx, int kind, const double *X, int n, int d, const double *Y, int n_out,
                     const double *ls, double sigma2, double noise, const KProgArg *prog, gpmpc_gp **out,
                     double *y_mean, double *y_std, double *lml, int *jitter_steps) {
  GPMPC_CHECK_ARG(ctx && X && Y && (ls || prog) && out && n >= 1 && d >= 1 && d <= 32);
  GPMPC_CHECK_ARG(n_out >= 1 && n_out <= 16 && (prog || (kind >= 0 && kind <= 3)));
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  auto *gp = new gpmpc_gp();
  GpCore &g = gp->core;
  gp->noise = noise;
  int rc = core_setup(ctx, g, kind, X, n, d, ls, sigma2, prog);
  if (rc) { delete gp; return rc; }
  DevBuf Kn, dinfo;
  auto fail = [&](int code) { delete gp; return code; };
  if (Kn.alloc(s, sizeof(double) * (size_t)n * n) != hipSuccess ||
      gp->L.alloc(s, sizeof(double) * (size_t)n * n) != hipSuccess ||
      dinfo.alloc(s, sizeof(int)) != hipSuccess) {
    gpmpc_set_error("gp_fit_exact: out of device memory");
    return fail(-1);
  }
  // K + noise I   (exact_gp.py:156-160)
  if (core_gram(s, g, g.Xs.as<double>(), g.Xn.as<double>(), n, g.Xs.as<double>(), g.Xn.as<double>(), n, 1,
                Kn.as<double>(), n) != hipSuccess ||
      launch_add_diag(s, n, Kn.as<double>(), n, noise, 1, 0) != hipSuccess) {
    gpmpc_set_error("gp_fit_exact: gram launch failed");
    return fail(-1);
  }
  // Cholesky with the jitter ladder (exact_gp.py:163-175): first no jitter,
  // then j = 1e-6 and j *= 10 while j < 1.
  int info = 0, steps = 0;
  double jit = 0.0;
  for (;;) {
    if (hipMemcpyAsync(gp->L.p, Kn.p, sizeof(double) * (size_t)n * n, hipMemcpyDeviceToDevice,
                       s) != hipSuccess)
      return fail(-1);
    if (steps > 0 && launch_add_diag(s, n, gp->L.as<double>(), n, jit, 1, 0) != hipSuccess)
      return fail(-1);
    if (launch_potrf_batched(s, n, 1, gp->L.as<double>(), n, 0, dinfo.as<int>()) != hipSuccess ||
        hipMemcpyAsync(&info, dinfo.p, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      gpmpc_set_error("gp_fit_exact: potrf failed: %s", hipGetErrorString(hipGetLastError()));
      return fail(-1);
    }
    if (info == 0) break;
    if (info < 0) return fail(gpmpc_potrf_info_error(info, "gp_fit_exact"));
    jit = (steps == 0) ? 1e-6 : jit * 10;
    if (!(jit < 1.0)) {
      gpmpc_set_error("Kernel matrix is not positive definite even with jitter");
      return fail(GPMPC_ERR_NOT_PD);
    }
    ++steps;
  }
  if (jitter_steps) *jitter_steps = steps;
  gp->jitter_steps = steps;
  // normalised targets, alpha = L^-T L^-1 y for all outputs (exact_gp.py:141-150, 179)
  DevBuf dYraw, dY, dyn, dlml;
  if (dYraw.alloc(s, sizeof(double) * n * n_out) || dY.alloc(s, sizeof(double) * n * n_out) ||
      dyn.alloc(s, sizeof(double) * n * n_out) || dlml.alloc(s, sizeof(double) * n_out) ||
      g.ymean.alloc(s, sizeof(double) * n_out) || g.ystd.alloc(s, sizeof(double) * n_out) ||
      g.alphaT.alloc(s, sizeof(double) * n_out * n) ||
      g.W.alloc(s, sizeof(double) * (size_t)(n + n_out) * n))  // [W; alpha^T]
    return fail(-1);
  g.n_out = n_out;
  hipMemcpyAsync(dYraw.p, Y, sizeof(double) * n * n_out, hipMemcpyHostToDevice, s);
  hipLaunchKernelGGL(k_normalise, dim3(n_out), dim3(256), 0, s, n, n_out, dYraw.as<double>(),
                     dyn.as<double>(), g.ymean.as<double>(), g.ystd.as<double>());
  hipMemcpyAsync(dY.p, dyn.p, sizeof(double) * n * n_out, hipMemcpyDeviceToDevice, s);
  // W = L^-1 (identity right-hand side, lower-triangular result): the doubling inverse,
  // or the blocked TRSM (GPMPC_TRI_INV=0, n <= 128)
  hipLaunchKernelGGL(k_eye, dim3((n + 255) / 256, n), dim3(256), 0, s, n, g.W.as<double>());
  static const int tri_inv_env = [] {
    const char *e = getenv("GPMPC_TRI_INV");
    return e ? atoi(e) : 1;
  }();
  const bool inv = tri_inv_env && n > 128;
  {
    DevBuf tinv;
    hipError_t e = inv ? tinv.alloc(s, sizeof(double) * (size_t)n * n) : hipSuccess;
    if (e == hipSuccess)
      e = inv ? launch_tri_inverse(s, n, gp->L.as<double>(), n, g.W.as<double>(), n, tinv.as<double>())
              : launch_trsm_lower_ex(s, n, n, gp->L.as<double>(), n, g.W.as<double>(), n, 0, 1, nullptr);
    if (e != hipSuccess) {
      gpmpc_set_error("gp_fit_exact: W = L^-1 failed: %s", hipGetErrorString(e));
      return fail(-1);
    }
  }
  // alpha = L^-T L^-1 y for all outputs: through W with one refinement step
  // (GPMPC_ALPHA_INV=0: the per-column substitution kernel, or the blocked TRSMs)
  static const int alpha_inv_env = [] {
    const char *e = getenv("GPMPC_ALPHA_INV");
    return e ? atoi(e) : 1;
  }();
  hipError_t ea = hipSuccess;
  if (alpha_inv_env) {
    ea = cho_solve_inv(s, n, n_out, gp->L.as<double>(), g.W.as<double>(), dY.as<double>());
  } else if (potrs_cols_ok(n)) {
    hipLaunchKernelGGL(k_potrs_cols, dim3(n_out), dim3(256), sizeof(double) * n, s, n,
                       gp->L.as<double>(), (int64_t)n, dY.as<double>(), n_out);
  } else {
    ea = launch_trsm_lower_ex(s, n, n_out, gp->L.as<double>(), n, dY.as<double>(), n_out, 0, 0, nullptr);
    if (ea == hipSuccess)
      ea = launch_trsm_lower_ex(s, n, n_out, gp->L.as<double>(), n, dY.as<double>(), n_out, 1, 0, nullptr);
  }
  if (ea != hipSuccess) {
    gpmpc_set_error("gp_fit_exact: alpha solve failed: %s", hipGetErrorString(ea));
    return fail(-1);
  }
  // log marginal likelihood per output + alpha^T for the posterior GEMM (exact_gp.py:186-204)
  hipLaunchKernelGGL(k_lml_exact, dim3(n_out), dim3(256), 0, s, n, n_out, gp->L.as<double>(),
                     dyn.as<double>(), dY.as<double>(), g.alphaT.as<double>(), dlml.as<double>());
  // alpha^T below W: the variance GEMM produces the posterior mean in the same pass
  hipMemcpyAsync(g.W.as<double>() + (size_t)n * n, g.alphaT.p, sizeof(double) * n_out * n,
                 hipMemcpyDeviceToDevice, s);
  if (core_pack(s, g) != hipSuccess) {
    gpmpc_set_error("gp_fit_exact: posterior operand pack failed");
    return fail(-1);
  }
  g.h_ymean.resize(n_out);
  g.h_ystd.resize(n_out);
  hipMemcpyAsync(g.h_ymean.data(), g.ymean.p, sizeof(double) * n_out, hipMemcpyDeviceToHost, s);
  hipMemcpyAsync(g.h_ystd.data(), g.ystd.p, sizeof(double) * n_out, hipMemcpyDeviceToHost, s);
  std::vector<double> hl(n_out);
  hipMemcpyAsync(hl.data(), dlml.p, sizeof(double) * n_out, hipMemcpyDeviceToHost, s);
  if (hipStreamSynchronize(s) != hipSuccess) {
    gpmpc_set_error("gp_fit_exact: %s", hipGetErrorString(hipGetLastError()));
    return fail(-1);
  }
  for (int c = 0; c < n_out; ++c) {
    if (lml) lml[c] = hl[c];
    if (y_mean) y_mean[c] = g.h_ymean[c];
    if (y_std) y_std[c] = g.h_ystd[c];
  }
  *out = gp;
  return 0;
}

extern "C" int gpmpc_gp_fit_exact(gpmpc_ctx *ctx, int kind, const double *X, int n, int d,
                                  const double *Y, int n_out, const double *ls, double sigma2,
                                  double noise, gpmpc_gp **out, double *y_mean, double *y_std,
                                  double *lml, int *jitter_steps) {
  GPMPC_CHECK_ARG(ls);
  return exact_fit(ctx, kind, X, n, d, Y, n_out, ls, sigma2, noise, nullptr, out, y_mean, y_std, lml,
                   jitter_steps);
}

extern "C" int gpmpc_gp_fit_exact_prog(gpmpc_ctx *ctx, const int *ops, int nops, const double *par, int npar,
                                       const double *X, int n, int d, const double *Y, int n_out, double noise,
                                       gpmpc_gp **out, double *y_mean, double *y_std, double *lml,
                                       int *jitter_steps) {
  GPMPC_CHECK_ARG(ops && par && nops >= 1 && npar >= 1);
  const KProgArg prog{ops, nops, par, npar};
  return exact_fit(ctx, GPMPC_KPROG, X, n, d, Y, n_out, nullptr, 0.0, noise, &prog, out, y_mean, y_std, lml,
                   jitter_steps);
}

// device-side posterior for p queries given K* (p x n): mean/var (p x n_out) device
static int core_posterior(gpmpc_ctx *ctx, const GpCore &g, const double *Ks, int p, double *dmean,
                          double *dvar) {
  hipStream_t s = ctx->stream;
  const int nrt = gemm_row_tiles(g.n + g.n_out, p, g.n);
  DevBuf part, meanT;
  GPMPC_HIP(part.alloc(s, sizeof(double) * (size_t)nrt * p));
  GPMPC_HIP(meanT.alloc(s, sizeof(double) * (size_t)g.n_out * p));
  // one pass over K*: sum_i (W K*^T)_ij^2 per query j and alpha^T K*^T
  GPMPC_HIP(launch_gemm_sumsq_mean(s, g.n, g.n_out, p, g.W.as<double>(), Ks, part.as<double>(), p,
                                   meanT.as<double>(), p));
  hipLaunchKernelGGL(k_post_finish, dim3((p + 255) / 256), dim3(256), 0, s, p, g.n_out, nrt,
                     part.as<double>(), (int64_t)p, meanT.as<double>(), (int64_t)p,
                     g.ymean.as<double>(), g.ystd.as<double>(), g.sigma2, dmean, dvar);
  GPMPC_HIP(hipGetLastError());
  return 0;  // (stream-ordered: every caller reads the results after its own synchronisation)
}

// the posterior of p device-resident raw query rows (p x d): device mean / var (p x n_out)
int gp_posterior_dev(gpmpc_ctx *ctx, gpmpc_gp *gp, const double *dq, int p, double *dmean, double *dvar) {
  const GpCore &g = gp->core;
  DevBuf Ks;
  const int rc = core_cross(ctx, g, dq, p, Ks);
  if (rc) return rc;
  return core_posterior(ctx, g, Ks.as<double>(), p, dmean, dvar);
}

extern "C" int gpmpc_gp_predict(gpmpc_ctx *ctx, gpmpc_gp *gp, const double *Xq, int p,
                                double *mean, double *var) {
  GPMPC_CHECK_ARG(ctx && gp && Xq && mean && var && p >= 0);
  if (p == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const GpCore &g = gp->core;
  DevBuf Ks;
  // the queries in one pinned upload, mean and variance in one read-back
  const size_t P = p, bo = Stage::pad(8 * P * g.n_out);
  Stage sg(s, Stage::pad(8 * P * g.d) + 2 * bo);
  if (!sg.ok()) {
    gpmpc_set_error("gp_predict: staging buffers: out of memory");
    return -1;
  }
  double *dq = sg.in(Xq, P * g.d), *dmean = sg.out(mean, P * g.n_out), *dvar = sg.out(var, P * g.n_out);
  GPMPC_HIP(sg.upload());
  if (g.Wf.p && post_cs_env()) {
    // K* formed inside the column-stationary posterior (post.hip): no K* in HBM
    DevBuf qs, qn, part, meanT;
    GPMPC_HIP(qs.alloc(s, sizeof(double) * p * g.d));
    GPMPC_HIP(qn.alloc(s, sizeof(double) * p));
    GPMPC_HIP(part.alloc(s, sizeof(double) * POST_CS_PARTS * p));
    GPMPC_HIP(meanT.alloc(s, sizeof(double) * g.n_out * p));
    GPMPC_HIP(launch_scale_rows(s, dq, p, g.d, g.ls.as<double>(), g.kind == GPMPC_SE_ISO,
                                qs.as<double>(), qn.as<double>()));
    GPMPC_HIP(launch_post_cs(s, g.n, g.n_out, p, g.Wf.as<double>(), g.Xp.as<double>(), qs.as<double>(),
                             qn.as<double>(), g.d, g.kind, g.sigma2, g.iso_scale, part.as<double>(), p,
                             meanT.as<double>(), p));
    GPMPC_HIP(launch_post_finish(s, p, g.n_out, POST_CS_PARTS, part.as<double>(), p, meanT.as<double>(), p,
                                 g.ymean.as<double>(), g.ystd.as<double>(), g.sigma2, dmean,
                                 dvar));
  } else {
    int rc = core_cross(ctx, g, dq, p, Ks);
    if (rc) return rc;
    rc = core_posterior(ctx, g, Ks.as<double>(), p, dmean, dvar);
    if (rc) return rc;
  }
  GPMPC_HIP(sg.download());
  return 0;
}

extern "C" int gpmpc_gp_predict_cov(gpmpc_ctx *ctx, gpmpc_gp *gp, const double *Xq, int p,
                                    double *mean, double *cov) {
  GPMPC_CHECK_ARG(ctx && gp && Xq && mean && cov && p >= 0);
  if (p == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const GpCore &g = gp->core;
  DevBuf dq, Ks, qs, qn, V, C, dmean, dvar;
  GPMPC_HIP(dq.alloc(s, sizeof(double) * p * g.d));
  GPMPC_HIP(hipMemcpyAsync(dq.p, Xq, sizeof(double) * p * g.d, hipMemcpyHostToDevice, s));
  int rc = core_cross(ctx, g, dq.as<double>(), p, Ks, &qs, &qn);
  if (rc) return rc;
  // V^T = K* W^T  (p x n):  (V^T)_{jm} = sum_i K*_{ji} W_{mi}
  GPMPC_HIP(V.alloc(s, sizeof(double) * (size_t)p * g.n));
  GPMPC_HIP(launch_gemm_nt(s, EPI_STORE, p, g.n, g.n, Ks.as<double>(), g.n, g.W.as<double>(), g.n,
                           V.as<double>(), g.n, 1.0, 0.0, 0, 0, 1, 0, 0, 0));
  // C = K** - V^T V   (exact_gp.py:250-252), in normalised units
  GPMPC_HIP(C.alloc(s, sizeof(double) * (size_t)p * p));
  GPMPC_HIP(core_gram(s, g, qs.as<double>(), qn.as<double>(), p, qs.as<double>(), qn.as<double>(), p, 1,
                      C.as<double>(), p));
  GPMPC_HIP(launch_gemm_nt(s, EPI_STORE, p, p, g.n, V.as<double>(), g.n, V.as<double>(), g.n,
                           C.as<double>(), p, -1.0, 1.0, 0, 0, 1, 0, 0, 0));
  GPMPC_HIP(dmean.alloc(s, sizeof(double) * p * g.n_out));
  GPMPC_HIP(dvar.alloc(s, sizeof(double) * p * g.n_out));
  rc = core_posterior(ctx, g, Ks.as<double>(), p, dmean.as<double>(), dvar.as<double>());
  if (rc) return rc;
  GPMPC_HIP(hipMemcpyAsync(mean, dmean.p, sizeof(double) * p * g.n_out, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipMemcpyAsync(cov, C.p, sizeof(double) * p * p, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

extern "C" int gpmpc_gp_get_state(gpmpc_ctx *ctx, gpmpc_gp *gp, double *L, double *alpha) {
  GPMPC_CHECK_ARG(ctx && gp);
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const int n = gp->core.n, no = gp->core.n_out;
  if (L) {
    DevBuf t;
    GPMPC_HIP(t.alloc(s, sizeof(double) * (size_t)n * n));
    GPMPC_HIP(launch_copy_lower(s, n, gp->L.as<double>(), n, t.as<double>(), n));
    GPMPC_HIP(hipMemcpyAsync(L, t.p, sizeof(double) * (size_t)n * n, hipMemcpyDeviceToHost, s));
    GPMPC_HIP(hipStreamSynchronize(s));
  }
  if (alpha) {
    std::vector<double> aT((size_t)no * n);
    GPMPC_HIP(hipMemcpyAsync(aT.data(), gp->core.alphaT.p, sizeof(double) * no * n,
                             hipMemcpyDeviceToHost, s));
    GPMPC_HIP(hipStreamSynchronize(s));
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < no; ++c) alpha[(size_t)i * no + c] = aT[(size_t)c * n + i];
  }
  return 0;
}

// A handle's buffers come from its fitting context's stream pool, but fleets and
// rollouts read them from their own streams: drain the device before they go back.
extern "C" int gpmpc_gp_destroy(gpmpc_gp *gp) {
  if (gp) (void)hipDeviceSynchronize();
  delete gp;
  return 0;
}

// ---- internal accessor for the fleet ----------------------------------------
extern "C" int gpmpc_fitc_get_state(gpmpc_ctx *ctx, gpmpc_fitc *gp, double *alpha) {
  GPMPC_CHECK_ARG(ctx && gp && alpha);
  GPMPC_HIP(hipSetDevice(ctx->device));
  const int m = gp->core.n, no = gp->core.n_out;
  std::vector<double> aT((size_t)no * m);
  GPMPC_HIP(hipMemcpyAsync(aT.data(), gp->core.alphaT.p, sizeof(double) * no * m, hipMemcpyDeviceToHost,
                           ctx->stream));
  GPMPC_HIP(hipStreamSynchronize(ctx->stream));
  for (int i = 0; i < m; ++i)
    for (int c = 0; c < no; ++c) alpha[(size_t)i * no + c] = aT[(size_t)c * m + i];
  return 0;
}

GpView gp_view(const gpmpc_gp *gp) {
  const GpCore &g = gp->core;
  return GpView{g.kind, g.n, g.d, g.n_out, g.sigma2, g.iso_scale, g.ls.as<double>(),
                g.Xs.as<double>(), g.Xn.as<double>(), g.W.as<double>(), g.alphaT.as<double>(),
                g.ymean.as<double>(), g.ystd.as<double>(), g.Wf.as<double>(), g.Xp.as<double>()};
}

const double *fitc_W2(const gpmpc_fitc *gp) { return gp->W2.as<double>(); }

hipError_t launch_fitc_finish(hipStream_t s, int P, int n_out, int nrv, int nrw, const double *pv,
                              const double *pw, int64_t ldp, const double *meanT, int64_t ldm,
                              const double *ymean, const double *ystd, double sigma2, double *mean,
                              double *var) {
  hipLaunchKernelGGL(k_fitc_finish, dim3((P + 255) / 256), dim3(256), 0, s, P, n_out, nrv, nrw, pv, pw, ldp,
                     meanT, ldm, ymean, ystd, sigma2, mean, var);
  return hipGetLastError();
}

GpView fitc_view(const gpmpc_fitc *gp) {
  const GpCore &g = gp->core;
  return GpView{g.kind, g.n, g.d, g.n_out, g.sigma2, g.iso_scale, g.ls.as<double>(),
                g.Xs.as<double>(), g.Xn.as<double>(), g.W.as<double>(), g.alphaT.as<double>(),
                g.ymean.as<double>(), g.ystd.as<double>(), nullptr, nullptr};
}

// ---------------------------------------------------------------------------
// FITC (sparse_gp.py:150-219 fit, :255-305 predict)
// VFE per-column |A e_j|^2 (A = L_uu^-1 K_uf), the Q_ff diagonal of the trace term
__global__ void k_colsumsq(int m, int n, const double *A, double *q) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int i = 0; i < m; ++i) s += A[(int64_t)i * n + j] * A[(int64_t)i * n + j];
  q[j] = s;
}

__global__ void k_fill(int n, double v, double *x) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) x[j] = v;
}

// VFE lower bound (sparse_gp.py:232-249) and alpha^T, one workgroup per output:
//   -y.y/(2 s2n) + c.alpha - alpha^T K_uu alpha / 2 - (n sigma2 - sum q) / (2 s2n)
//   - sum log diag L_B + sum log diag L_uu - n/2 log s2n - n/2 log 2 pi
// with c = K_uf y / s2n, so y^T K_fu alpha / s2n = c.alpha
__global__ __launch_bounds__(256) void k_lml_vfe(int m, int n, int n_out, const double *LB,
                                                 const double *Luu, const double *Kuu,
                                                 const double *yn, const double *q,
                                                 const double *cvec, const double *alpha,
                                                 double sigma2, double noise, double *alphaT,
                                                 double *lml) {
  __shared__ double red[4];
  const int c = blockIdx.x;
  double ldb = 0.0, ldu = 0.0, ca = 0.0, aka = 0.0, yy = 0.0, qs = 0.0;
  for (int i = threadIdx.x; i < m; i += 256) {
    ldb += log(LB[(int64_t)i * m + i]);
    ldu += log(Luu[(int64_t)i * m + i]);
    const double a = alpha[(int64_t)i * n_out + c];
    ca += cvec[(int64_t)i * n_out + c] * a;
    alphaT[(int64_t)c * m + i] = a;
    double r = 0.0;
    for (int k = 0; k < m; ++k) r += Kuu[(int64_t)i * m + k] * alpha[(int64_t)k * n_out + c];
    aka += a * r;
  }
  for (int j = threadIdx.x; j < n; j += 256) {
    const double y = yn[(int64_t)j * n_out + c];
    yy += y * y;
    qs += q[j];
  }
  ldb = block_sum(ldb, red);
  ldu = block_sum(ldu, red);
  ca = block_sum(ca, red);
  aka = block_sum(aka, red);
  yy = block_sum(yy, red);
  qs = block_sum(qs, red);
  if (threadIdx.x == 0) {
    const double data_fit = -0.5 / noise * yy + ca - 0.5 * aka;
    const double trace_term = (n * sigma2 - qs) / noise;
    const double complexity = -ldb + ldu - 0.5 * n * log(noise);
    lml[c] = data_fit - 0.5 * trace_term + complexity - 0.5 * n * log(2.0 * M_PI);
  }
}

// VFE after L_uu, K_uf and W = L_uu^-1 are formed (sparse_gp.py:221-249): B = K_uu +
// K_uf K_fu / s2n + jitter I -> L_B, c = K_uf y / s2n, alpha = B^-1 c, the bound
static int vfe_tail(gpmpc_ctx *ctx, gpmpc_fitc *gp, DevBuf &Luu, DevBuf &Kuf, DevBuf &B,
                    DevBuf &dinfo, const double *Y, int n, int n_out, double sigma2, double noise,
                    double jitter, gpmpc_fitc **out, double *y_mean, double *y_std, double *lml) {
  hipStream_t s = ctx->stream;
  GpCore &g = gp->core;
  const int m = gp->m;
  auto fail = [&](int code) { delete gp; return code; };
  DevBuf Kuu, q, dYraw, dyn, yl, sig, cvec, alpha, dlml;
  if (Kuu.alloc(s, sizeof(double) * (size_t)m * m) || q.alloc(s, sizeof(double) * n) ||
      dYraw.alloc(s, sizeof(double) * n * n_out) || dyn.alloc(s, sizeof(double) * n * n_out) ||
      yl.alloc(s, sizeof(double) * n * n_out) || sig.alloc(s, sizeof(double) * n) ||
      cvec.alloc(s, sizeof(double) * m * n_out) || alpha.alloc(s, sizeof(double) * m * n_out) ||
      dlml.alloc(s, sizeof(double) * n_out) || g.ymean.alloc(s, sizeof(double) * n_out) ||
      g.ystd.alloc(s, sizeof(double) * n_out) || g.alphaT.alloc(s, sizeof(double) * n_out * m)) {
    gpmpc_set_error("vfe_fit: out of device memory");
    return fail(-1);
  }
  g.n_out = n_out;
  // K_uu into B (kept for alpha^T K_uu alpha), then B += K_uf K_fu / s2n (SYRK on
  // MFMA, lower triangle), then + jitter I in the reference's order
  core_gram(s, g, g.Xs.as<double>(), g.Xn.as<double>(), m, g.Xs.as<double>(), g.Xn.as<double>(), m, 1,
            B.as<double>(), m);
  hipMemcpyAsync(Kuu.p, B.p, sizeof(double) * (size_t)m * m, hipMemcpyDeviceToDevice, s);
  launch_gemm_nt(s, EPI_STORE, m, m, n, Kuf.as<double>(), n, Kuf.as<double>(), n, B.as<double>(), m,
                 1.0 / noise, 1.0, 0, 1, 1, 0, 0, 0);
  launch_add_diag(s, m, B.as<double>(), m, jitter, 1, 0);
  // normalised targets; c = K_uf (y / s2n)  (sparse_gp.py:160-166, 231)
  hipMemcpyAsync(dYraw.p, Y, sizeof(double) * n * n_out, hipMemcpyHostToDevice, s);
  hipLaunchKernelGGL(k_normalise, dim3(n_out), dim3(256), 0, s, n, n_out, dYraw.as<double>(),
                     dyn.as<double>(), g.ymean.as<double>(), g.ystd.as<double>());
  hipLaunchKernelGGL(k_fill, dim3((n + 255) / 256), dim3(256), 0, s, n, noise, sig.as<double>());
  hipLaunchKernelGGL(k_fitc_yl, dim3((n + 255) / 256, n_out), dim3(256), 0, s, n, n_out,
                     dyn.as<double>(), sig.as<double>(), yl.as<double>());
  launch_gemm_nt(s, EPI_STORE, m, n_out, n, Kuf.as<double>(), n, yl.as<double>(), n,
                 cvec.as<double>(), n_out, 1.0, 0.0, 0, 0, 1, 0, 0, 0);
  // Q_ff diagonal for the trace term: colsum((L_uu^-1 K_uf)^2)  (sparse_gp.py:240-242)
  launch_trsm_lower_ex(s, m, n, Luu.as<double>(), m, Kuf.as<double>(), n, 0, 0, nullptr);
  hipLaunchKernelGGL(k_colsumsq, dim3((n + 255) / 256), dim3(256), 0, s, m, n, Kuf.as<double>(),
                     q.as<double>());
  int info = 0;
  launch_potrf_batched(s, m, 1, B.as<double>(), m, 0, dinfo.as<int>());
  hipMemcpyAsync(&info, dinfo.p, sizeof(int), hipMemcpyDeviceToHost, s);
  GPMPC_HIP(hipStreamSynchronize(s));
  if (info) return fail(gpmpc_potrf_info_error(info, "B"));
  // W2 = L_B^-1 L_uu^-1: the predict's w = L_B^-1 v as the reference writes it for both
  // methods (sparse_gp.py:292-296)
  hipMemcpyAsync(gp->W2.p, g.W.p, sizeof(double) * (size_t)m * m, hipMemcpyDeviceToDevice, s);
  launch_trsm_lower_ex(s, m, m, B.as<double>(), m, gp->W2.as<double>(), m, 0, 1, nullptr);
  hipMemcpyAsync(alpha.p, cvec.p, sizeof(double) * m * n_out, hipMemcpyDeviceToDevice, s);
  if (potrs_cols_ok(m)) {
    hipLaunchKernelGGL(k_potrs_cols, dim3(n_out), dim3(256), sizeof(double) * m, s, m,
                       B.as<double>(), (int64_t)m, alpha.as<double>(), n_out);
  } else {
    launch_trsm_lower_ex(s, m, n_out, B.as<double>(), m, alpha.as<double>(), n_out, 0, 0, nullptr);
    launch_trsm_lower_ex(s, m, n_out, B.as<double>(), m, alpha.as<double>(), n_out, 1, 0, nullptr);
  }
  hipLaunchKernelGGL(k_lml_vfe, dim3(n_out), dim3(256), 0, s, m, n, n_out, B.as<double>(),
                     Luu.as<double>(), Kuu.as<double>(), dyn.as<double>(), q.as<double>(),
                     cvec.as<double>(), alpha.as<double>(), sigma2, noise, g.alphaT.as<double>(),
                     dlml.as<double>());
  hipMemcpyAsync(g.W.as<double>() + (size_t)m * m, g.alphaT.p, sizeof(double) * n_out * m,
                 hipMemcpyDeviceToDevice, s);
  g.h_ymean.resize(n_out);
  g.h_ystd.resize(n_out);
  std::vector<double> hl(n_out);
  hipMemcpyAsync(g.h_ymean.data(), g.ymean.p, sizeof(double) * n_out, hipMemcpyDeviceToHost, s);
  hipMemcpyAsync(g.h_ystd.data(), g.ystd.p, sizeof(double) * n_out, hipMemcpyDeviceToHost, s);
  hipMemcpyAsync(hl.data(), dlml.p, sizeof(double) * n_out, hipMemcpyDeviceToHost, s);
  if (hipStreamSynchronize(s) != hipSuccess) {
    gpmpc_set_error("vfe_fit: %s", hipGetErrorString(hipGetLastError()));
    return fail(-1);
  }
  for (int c = 0; c < n_out; ++c) {
    if (lml) lml[c] = hl[c];
    if (y_mean) y_mean[c] = g.h_ymean[c];
    if (y_std) y_std[c] = g.h_ystd[c];
  }
  *out = gp;
  return 0;
}

// SparseGP.fit, FITC (vfe = 0, sparse_gp.py:181-219) or VFE (vfe = 1, :181-188 then
// :221-249).  Both leave the same handle: W = [L_uu^-1; alpha^T], W2 = L_B^-1 L_uu^-1,
// so gpmpc_fitc_predict serves both (the reference's predict has one body for the two).
static int sparse_fit(gpmpc_ctx *ctx, const double *Z, int m, const double *X, int n, int d,
                      const double *Y, int n_out, const double *ls, double sigma2, double noise,
                      double jitter, gpmpc_fitc **out, double *y_mean, double *y_std, double *lml,
                      double *lambda_diag, int vfe, const KProgArg *prog = nullptr) {
  GPMPC_CHECK_ARG(ctx && Z && X && Y && (ls || prog) && out && m >= 1 && n >= 1 && d >= 1 && d <= 32);
  GPMPC_CHECK_ARG(n_out >= 1 && n_out <= 16);
  GPMPC_CHECK_ARG(!vfe || noise > 0.0);
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  auto *gp = new gpmpc_fitc();
  GpCore &g = gp->core;
  gp->m = m;
  int rc = core_setup(ctx, g, GPMPC_SE_ARD, Z, m, d, ls, sigma2, prog);
  if (rc) { delete gp; return rc; }
  sigma2 = g.sigma2;  // a program's diagonal: kernel.diagonal(X) in Lambda and the VFE trace
  auto fail = [&](int code) { delete gp; return code; };
  DevBuf dX, Kuf, Luu, B, dinfo, lam, Xs, Xn, part;
  if (dX.alloc(s, sizeof(double) * n * d) || Kuf.alloc(s, sizeof(double) * (size_t)m * n) ||
      Luu.alloc(s, sizeof(double) * (size_t)m * m) || B.alloc(s, sizeof(double) * (size_t)m * m) ||
      dinfo.alloc(s, sizeof(int)) || lam.alloc(s, sizeof(double) * n) ||
      Xs.alloc(s, sizeof(double) * n * d) || Xn.alloc(s, sizeof(double) * n) ||
      g.W.alloc(s, sizeof(double) * (size_t)(m + n_out) * m) ||  // [L_uu^-1; alpha^T]
      gp->W2.alloc(s, sizeof(double) * (size_t)m * m)) {
    gpmpc_set_error("fitc_fit: out of device memory");
    return fail(-1);
  }
  hipMemcpyAsync(dX.p, X, sizeof(double) * n * d, hipMemcpyHostToDevice, s);
  core_rows(s, g, dX.as<double>(), n, Xs.as<double>(), Xn.as<double>());
  // K_uu + jitter I -> L_uu   (sparse_gp.py:181-187; no jitter ladder in the reference)
  core_gram(s, g, g.Xs.as<double>(), g.Xn.as<double>(), m, g.Xs.as<double>(), g.Xn.as<double>(), m, 1,
            Luu.as<double>(), m);
  launch_add_diag(s, m, Luu.as<double>(), m, jitter, 1, 0);
  int info = 0;
  launch_potrf_batched(s, m, 1, Luu.as<double>(), m, 0, dinfo.as<int>());
  hipMemcpyAsync(&info, dinfo.p, sizeof(int), hipMemcpyDeviceToHost, s);
  GPMPC_HIP(hipStreamSynchronize(s));
  if (info) return fail(gpmpc_potrf_info_error(info, "K_uu"));
  // A = L_uu^-1 K_uf  (m x n); VFE forms B and c from K_uf itself first
  core_gram(s, g, g.Xs.as<double>(), g.Xn.as<double>(), m, Xs.as<double>(), Xn.as<double>(), n, 0,
            Kuf.as<double>(), n);
  hipLaunchKernelGGL(k_eye, dim3((m + 255) / 256, m), dim3(256), 0, s, m, g.W.as<double>());
  {
    DevBuf tinv;  // W = L_uu^-1 by the doubling inverse (exact fit's W, §10)
    const bool inv = m > 128;
    hipError_t e = inv ? tinv.alloc(s, sizeof(double) * (size_t)m * m) : hipSuccess;
    if (e == hipSuccess)
      e = inv ? launch_tri_inverse(s, m, Luu.as<double>(), m, g.W.as<double>(), m, tinv.as<double>())
              : launch_trsm_lower_ex(s, m, m, Luu.as<double>(), m, g.W.as<double>(), m, 0, 1, nullptr);
    if (e != hipSuccess) {
      gpmpc_set_error("sparse fit: W = L_uu^-1 failed: %s", hipGetErrorString(e));
      return fail(-1);
    }
  }
  if (vfe) return vfe_tail(ctx, gp, Luu, Kuf, B, dinfo, Y, n, n_out, sigma2, noise, jitter, out,
                           y_mean, y_std, lml);
  launch_trsm_lower_ex(s, m, n, Luu.as<double>(), m, Kuf.as<double>(), n, 0, 0, nullptr);
  // normalised targets; c = A (y / Lambda) before A is rescaled  (sparse_gp.py:160-166, 204)
  DevBuf isq, dYraw, dyn, yl, cvec, alpha, dlml;
  if (isq.alloc(s, sizeof(double) * n) || dYraw.alloc(s, sizeof(double) * n * n_out) ||
      dyn.alloc(s, sizeof(double) * n * n_out) || yl.alloc(s, sizeof(double) * n * n_out) ||
      cvec.alloc(s, sizeof(double) * m * n_out) || alpha.alloc(s, sizeof(double) * m * n_out) ||
      dlml.alloc(s, sizeof(double) * n_out) || g.ymean.alloc(s, sizeof(double) * n_out) ||
      g.ystd.alloc(s, sizeof(double) * n_out) || g.alphaT.alloc(s, sizeof(double) * n_out * m))
    return fail(-1);
  g.n_out = n_out;
  // Lambda = max(sigma2 - colsum(A^2) + noise, 1e-10)   (sparse_gp.py:193-199)
  hipLaunchKernelGGL(k_fitc_lambda, dim3((n + 255) / 256), dim3(256), 0, s, m, n, Kuf.as<double>(),
                     sigma2, noise, lam.as<double>(), isq.as<double>());
  hipMemcpyAsync(dYraw.p, Y, sizeof(double) * n * n_out, hipMemcpyHostToDevice, s);
  hipLaunchKernelGGL(k_normalise, dim3(n_out), dim3(256), 0, s, n, n_out, dYraw.as<double>(),
                     dyn.as<double>(), g.ymean.as<double>(), g.ystd.as<double>());
  hipLaunchKernelGGL(k_fitc_yl, dim3((n + 255) / 256, n_out), dim3(256), 0, s, n, n_out,
                     dyn.as<double>(), lam.as<double>(), yl.as<double>());
  launch_gemm_nt(s, EPI_STORE, m, n_out, n, Kuf.as<double>(), n, yl.as<double>(), n,
                 cvec.as<double>(), n_out, 1.0, 0.0, 0, 0, 1, 0, 0, 0);
  // B = I + A_s A_s^T, A_s = A Lambda^-1/2  (SYRK on MFMA, K = n)
  hipLaunchKernelGGL(k_scale_cols, dim3((n + 255) / 256, m), dim3(256), 0, s, m, n,
                     Kuf.as<double>(), (int64_t)n, isq.as<double>());
  hipLaunchKernelGGL(k_eye, dim3((m + 255) / 256, m), dim3(256), 0, s, m, B.as<double>());
  // lower triangle only (potrf, the TRSMs and the lml read nothing above the diagonal)
  launch_gemm_nt(s, EPI_STORE, m, m, n, Kuf.as<double>(), n, Kuf.as<double>(), n, B.as<double>(), m,
                 1.0, 1.0, 0, 1, 1, 0, 0, 0);
  launch_potrf_batched(s, m, 1, B.as<double>(), m, 0, dinfo.as<int>());
  hipMemcpyAsync(&info, dinfo.p, sizeof(int), hipMemcpyDeviceToHost, s);
  GPMPC_HIP(hipStreamSynchronize(s));
  if (info) return fail(gpmpc_potrf_info_error(info, "B"));
  // W2 = L_B^-1 L_uu^-1 (a lower right-hand side): the predict gets |w|^2 from one
  // triangular pass over K*u instead of storing v = L_uu^-1 K*u^T and solving again
  hipMemcpyAsync(gp->W2.p, g.W.p, sizeof(double) * (size_t)m * m, hipMemcpyDeviceToDevice, s);
  launch_trsm_lower_ex(s, m, m, B.as<double>(), m, gp->W2.as<double>(), m, 0, 1, nullptr);
  // alpha = B^-1 c  and the FITC lml  (sparse_gp.py:207-218)
  hipMemcpyAsync(alpha.p, cvec.p, sizeof(double) * m * n_out, hipMemcpyDeviceToDevice, s);
  if (potrs_cols_ok(m)) {
    hipLaunchKernelGGL(k_potrs_cols, dim3(n_out), dim3(256), sizeof(double) * m, s, m,
                       B.as<double>(), (int64_t)m, alpha.as<double>(), n_out);
  } else {
    launch_trsm_lower_ex(s, m, n_out, B.as<double>(), m, alpha.as<double>(), n_out, 0, 0, nullptr);
    launch_trsm_lower_ex(s, m, n_out, B.as<double>(), m, alpha.as<double>(), n_out, 1, 0, nullptr);
  }
  hipLaunchKernelGGL(k_lml_fitc, dim3(n_out), dim3(256), 0, s, m, n, n_out, B.as<double>(),
                     dyn.as<double>(), lam.as<double>(), cvec.as<double>(), alpha.as<double>(),
                     g.alphaT.as<double>(), dlml.as<double>());
  // alpha^T below L_uu^-1: the predict's first pass yields the mean as well
  hipMemcpyAsync(g.W.as<double>() + (size_t)m * m, g.alphaT.p, sizeof(double) * n_out * m,
                 hipMemcpyDeviceToDevice, s);
  g.h_ymean.resize(n_out);
  g.h_ystd.resize(n_out);
  std::vector<double> hl(n_out);
  hipMemcpyAsync(g.h_ymean.data(), g.ymean.p, sizeof(double) * n_out, hipMemcpyDeviceToHost, s);
  hipMemcpyAsync(g.h_ystd.data(), g.ystd.p, sizeof(double) * n_out, hipMemcpyDeviceToHost, s);
  hipMemcpyAsync(hl.data(), dlml.p, sizeof(double) * n_out, hipMemcpyDeviceToHost, s);
  if (lambda_diag)
    hipMemcpyAsync(lambda_diag, lam.p, sizeof(double) * n, hipMemcpyDeviceToHost, s);
  if (hipStreamSynchronize(s) != hipSuccess) {
    gpmpc_set_error("fitc_fit: %s", hipGetErrorString(hipGetLastError()));
    return fail(-1);
  }
  for (int c = 0; c < n_out; ++c) {
    if (lml) lml[c] = hl[c];
    if (y_mean) y_mean[c] = g.h_ymean[c];
    if (y_std) y_std[c] = g.h_ystd[c];
  }
  *out = gp;
  return 0;
}

extern "C" int gpmpc_fitc_fit(gpmpc_ctx *ctx, const double *Z, int m, const double *X, int n,
                              int d, const double *Y, int n_out, const double *ls, double sigma2,
                              double noise, double jitter, gpmpc_fitc **out, double *y_mean,
                              double *y_std, double *lml, double *lambda_diag) {
  return sparse_fit(ctx, Z, m, X, n, d, Y, n_out, ls, sigma2, noise, jitter, out, y_mean, y_std,
                    lml, lambda_diag, 0);
}

extern "C" int gpmpc_vfe_fit(gpmpc_ctx *ctx, const double *Z, int m, const double *X, int n,
                             int d, const double *Y, int n_out, const double *ls, double sigma2,
                             double noise, double jitter, gpmpc_fitc **out, double *y_mean,
                             double *y_std, double *lml) {
  return sparse_fit(ctx, Z, m, X, n, d, Y, n_out, ls, sigma2, noise, jitter, out, y_mean, y_std,
                    lml, nullptr, 1);
}

extern "C" int gpmpc_sparse_fit_prog(gpmpc_ctx *ctx, int method, const int *ops, int nops, const double *par,
                                     int npar, const double *Z, int m, const double *X, int n, int d,
                                     const double *Y, int n_out, double noise, double jitter, gpmpc_fitc **out,
                                     double *y_mean, double *y_std, double *lml, double *lambda_diag) {
  GPMPC_CHECK_ARG(ops && par && nops >= 1 && npar >= 1 && (method == 0 || method == 1));
  const KProgArg prog{ops, nops, par, npar};
  return sparse_fit(ctx, Z, m, X, n, d, Y, n_out, nullptr, 0.0, noise, jitter, out, y_mean, y_std, lml,
                    method == 0 ? lambda_diag : nullptr, method, &prog);
}

// FITC posterior for small inducing sets (m <= 256): one workgroup per query forms k*
// (the k_scale_rows / k_gram arithmetic: same bits), v = L_uu^-1 k* over the lower triangle,
// w = W2 k*, the mean alpha^T k* and the k_fitc_finish epilogue in one launch instead of five.
// The sums |v|^2, |w|^2 and alpha^T k* run as a block reduction (another order than the
// row-tile partials of the GEMM form: equal to ~1e-16 relative).
#define FITC_SMALL_M 256
#define FITC_SMALL_D 64
#define FITC_SMALL_NO 8
__global__ __launch_bounds__(256) void k_fitc_post_small(GpView g, int m, const double *__restrict__ W2,
                                                         const double *__restrict__ Xq, double *__restrict__ mean,
                                                         double *__restrict__ var) {
  const int j = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6, d = g.d, no = g.n_out;
  __shared__ double sz[FITC_SMALL_D], sk[FITC_SMALL_M], red[4][FITC_SMALL_NO + 2];
  __shared__ double szn;
  if (t < d) sz[t] = g.kind == GPMPC_SE_ISO ? Xq[(int64_t)j * d + t] : Xq[(int64_t)j * d + t] / g.ls[t];
  __syncthreads();
  if (t == 0) {
    double q = 0.0;
    for (int f = 0; f < d; ++f) q += sz[f] * sz[f];
    szn = q;
  }
  __syncthreads();
  if (t < m) {
    double dot = 0.0;
    for (int f = 0; f < d; ++f) dot = fma(sz[f], g.Xs[(int64_t)t * d + f], dot);
    sk[t] = kernel_epilogue(g.kind, (szn + g.Xn[t]) - 2.0 * dot, g.sigma2, g.iso_scale);
  }
  __syncthreads();
  double acc[FITC_SMALL_NO + 2];
#pragma unroll
  for (int c = 0; c < FITC_SMALL_NO + 2; ++c) acc[c] = 0.0;
  if (t < m) {
    const double *wr = g.W + (int64_t)t * m, *w2 = W2 + (int64_t)t * m;
    double v = 0.0, w = 0.0;
    for (int i = 0; i <= t; ++i) v = fma(wr[i], sk[i], v);
    for (int i = 0; i < m; ++i) w = fma(w2[i], sk[i], w);
    acc[0] = v * v;
    acc[1] = w * w;
    for (int c = 0; c < no; ++c) acc[2 + c] = g.alphaT[(int64_t)c * m + t] * sk[t];
  }
#pragma unroll
  for (int c = 0; c < FITC_SMALL_NO + 2; ++c)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc[c] += __shfl_xor(acc[c], o);
  if (lane == 0)
    for (int c = 0; c < FITC_SMALL_NO + 2; ++c) red[wave][c] = acc[c];
  __syncthreads();
  if (t < no) {
    double r[2 + 1];
    const int cs[3] = {0, 1, 2 + t};
    for (int q = 0; q < 3; ++q) r[q] = ((red[0][cs[q]] + red[1][cs[q]]) + red[2][cs[q]]) + red[3][cs[q]];
    double lat = g.sigma2 - r[0] + r[1];
    lat = lat > 1e-10 ? lat : 1e-10;
    mean[(int64_t)j * no + t] = r[2] * g.ystd[t] + g.ymean[t];
    var[(int64_t)j * no + t] = lat * g.ystd[t] * g.ystd[t];
  }
}

// the FITC posterior of p device-resident raw query rows (sparse_gp.py:255-305): mean / var (p x n_out)
int fitc_posterior_dev(gpmpc_ctx *ctx, gpmpc_fitc *gp, const double *dq, int p, double *dmean, double *dvar) {
  hipStream_t s = ctx->stream;
  const GpCore &g = gp->core;
  const int m = gp->m;
  // small inducing sets: one launch (GPMPC_FITC_SMALL=0: the GEMM form at every size)
  const char *fs = getenv("GPMPC_FITC_SMALL");
  if ((!fs || atoi(fs)) && m <= FITC_SMALL_M && g.d <= FITC_SMALL_D && g.n_out <= FITC_SMALL_NO &&
      g.kind != GPMPC_KPROG) {
    hipLaunchKernelGGL(k_fitc_post_small, dim3(p), dim3(256), 0, s, fitc_view(gp), m, gp->W2.as<double>(), dq,
                       dmean, dvar);
    GPMPC_HIP(hipGetLastError());
    return 0;
  }
  DevBuf Ks, pv, pw, meanT;
  int rc = core_cross(ctx, g, dq, p, Ks);  // K*u (p x m)
  if (rc) return rc;
  const int nrv = gemm_row_tiles(m + g.n_out, p, m), nrw = gemm_row_tiles(m, p, m);
  GPMPC_HIP(pv.alloc(s, sizeof(double) * (size_t)nrv * p));
  GPMPC_HIP(pw.alloc(s, sizeof(double) * (size_t)nrw * p));
  GPMPC_HIP(meanT.alloc(s, sizeof(double) * (size_t)g.n_out * p));
  // |v|^2 = |L_uu^-1 k*|^2 and the mean alpha^T k* in one pass; |w|^2 = |W2 k*|^2
  GPMPC_HIP(launch_gemm_sumsq_mean(s, m, g.n_out, p, g.W.as<double>(), Ks.as<double>(),
                                   pv.as<double>(), p, meanT.as<double>(), p));
  GPMPC_HIP(launch_gemm_nt(s, EPI_SUMSQ, m, p, m, gp->W2.as<double>(), m, Ks.as<double>(), m,
                           pw.as<double>(), p, 1.0, 0.0, 1, 0, 1, 0, 0, 0));
  hipLaunchKernelGGL(k_fitc_finish, dim3((p + 255) / 256), dim3(256), 0, s, p, g.n_out, nrv, nrw,
                     pv.as<double>(), pw.as<double>(), (int64_t)p, meanT.as<double>(), (int64_t)p,
                     g.ymean.as<double>(), g.ystd.as<double>(), g.sigma2, dmean, dvar);
  GPMPC_HIP(hipGetLastError());
  return 0;
}

extern "C" int gpmpc_fitc_predict(gpmpc_ctx *ctx, gpmpc_fitc *gp, const double *Xq, int p,
                                  double *mean, double *var) {
  GPMPC_CHECK_ARG(ctx && gp && Xq && mean && var && p >= 0);
  if (p == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  const GpCore &g = gp->core;
  // the queries in one pinned upload, mean and variance in one read-back
  const size_t P = p, bo = Stage::pad(8 * P * g.n_out);
  Stage sg(ctx->stream, Stage::pad(8 * P * g.d) + 2 * bo);
  if (!sg.ok()) {
    gpmpc_set_error("fitc_predict: staging buffers: out of memory");
    return -1;
  }
  double *dq = sg.in(Xq, P * g.d), *dmean = sg.out(mean, P * g.n_out), *dvar = sg.out(var, P * g.n_out);
  GPMPC_HIP(sg.upload());
  const int rc = fitc_posterior_dev(ctx, gp, dq, p, dmean, dvar);
  if (rc) return rc;
  GPMPC_HIP(sg.download());
  return 0;
}

extern "C" int gpmpc_fitc_destroy(gpmpc_fitc *gp) {
  if (gp) (void)hipDeviceSynchronize();  // as gpmpc_gp_destroy
  delete gp;
  return 0;
}

// ---------------------------------------------------------------------------
// batched log marginal likelihood for hyperparameter search
// (ExactGP.optimize_hyperparameters, exact_gp.py:357-421: every objective call
// is a full ExactGP.fit, :118-204).  Per parameter set b: K_b + noise_b I,
// Cholesky (all B in one batched potrf, the jitter ladder of :163-175 for the
// ones that fail), then lml_b = -1/2 |L_b^-1 y|^2 - sum log L_ii - n/2 log 2 pi
// (|L^-1 y|^2 = y^T alpha).
//
// k_lml_trsv: one workgroup per matrix, x = L^-1 y right-looking by 32-row
// blocks: wave 0 solves the block's triangle in registers (readlane
// broadcasts), then all 256 threads subtract L[r, blk] x_blk from the
// remaining right-hand side (one row per thread, its 32 block entries are
// contiguous), so L's lower triangle is read once.
__global__ __launch_bounds__(256) void k_lml_trsv(int n, const double *__restrict__ L,
                                                  int64_t stride, const double *__restrict__ yn,
                                                  const int *__restrict__ info,
                                                  double *__restrict__ lml) {
  const int b = blockIdx.x;
  if (info[b]) return;
  const double *M = L + (int64_t)b * stride;
  extern __shared__ double s_[];  // rhs / solution (n), then 4 reduction slots
  double *x = s_, *red = s_ + n;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int i = tid; i < n; i += 256) x[i] = yn[i];
  __syncthreads();
  double logdet = 0.0;
  for (int r0 = 0; r0 < n; r0 += 32) {
    const int nb = min(32, n - r0);
    if (wave == 0) {
      double a[32];
#pragma unroll
      for (int j = 0; j < 32; ++j)
        a[j] = (lane < nb && j <= lane) ? M[(int64_t)(r0 + lane) * n + r0 + j] : 1.0;
      double s = lane < nb ? x[r0 + lane] : 0.0, dg = 1.0;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        if (j < nb) {
          if (lane == j) {
            dg = a[j];
            s = s / a[j];
          }
          const double xj = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(s), j),
                                             __builtin_amdgcn_readlane(__double2loint(s), j));
          if (lane > j) s = fma(-a[j], xj, s);
        }
      }
      if (lane < nb) {
        x[r0 + lane] = s;
        logdet += log(dg);
      }
    }
    __syncthreads();
    const int r1 = r0 + nb;
    if (r1 < n) {
      double xb[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) xb[j] = x[r0 + j];  // LDS broadcast
      for (int r = r1 + tid; r < n; r += 256) {
        const double *row = M + (int64_t)r * n + r0;
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < 32; ++j) acc = fma(row[j], xb[j], acc);
        x[r] -= acc;
      }
    }
    __syncthreads();
  }
  double fit = 0.0;
  for (int i = tid; i < n; i += 256) fit = fma(x[i], x[i], fit);
  fit = block_sum(fit, red);
  const double ld = block_sum(logdet, red);
  if (tid == 0) lml[b] = -0.5 * fit - ld - 0.5 * n * log(2.0 * M_PI);
}

extern "C" int gpmpc_gp_lml_batched(gpmpc_ctx *ctx, int kind, const double *X, int n, int d,
                                    const double *y, int B, const double *ls,
                                    const double *sigma2, const double *noise, double *lml,
                                    int *jitter_steps) {
  GPMPC_CHECK_ARG(ctx && X && y && ls && sigma2 && noise && lml && jitter_steps);
  GPMPC_CHECK_ARG(n >= 1 && d >= 1 && d <= 32 && B >= 1 && kind >= 0 && kind <= 3);
  GPMPC_CHECK_ARG((size_t)n * sizeof(double) + 64 <= 160 * 1024);
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const int iso = (kind == GPMPC_SE_ISO);
  const size_t nn = (size_t)n * n;
  DevBuf dX, dY, dyn, dm, dsd, dls, Xs, Xn, dinfo, dlml;
  GPMPC_HIP(dX.alloc(s, sizeof(double) * n * d));
  GPMPC_HIP(dY.alloc(s, sizeof(double) * n));
  GPMPC_HIP(dyn.alloc(s, sizeof(double) * n));
  GPMPC_HIP(dm.alloc(s, sizeof(double)));
  GPMPC_HIP(dsd.alloc(s, sizeof(double)));
  GPMPC_HIP(dls.alloc(s, sizeof(double) * B * d));
  GPMPC_HIP(Xs.alloc(s, sizeof(double) * (size_t)B * n * d));
  GPMPC_HIP(Xn.alloc(s, sizeof(double) * (size_t)B * n));
  // the B Gram / factor matrices live in persistent scratch (slot 3): one
  // optimiser gradient per call, so a per-call hipMalloc of B n^2 doubles
  // (112 MB at n = 1000) would cost more than the factorisations
  double *Kbuf = (double *)gpmpc_scratch(ctx->stream, 3, sizeof(double) * nn * B);
  if (!Kbuf) {
    gpmpc_set_error("gp_lml_batched: out of device memory for %d x %d^2 doubles", B, n);
    return -1;
  }
  GPMPC_HIP(dinfo.alloc(s, sizeof(int) * B));
  GPMPC_HIP(dlml.alloc(s, sizeof(double) * B));
  GPMPC_HIP(hipMemcpyAsync(dX.p, X, sizeof(double) * n * d, hipMemcpyHostToDevice, s));
  GPMPC_HIP(hipMemcpyAsync(dY.p, y, sizeof(double) * n, hipMemcpyHostToDevice, s));
  GPMPC_HIP(hipMemcpyAsync(dls.p, ls, sizeof(double) * B * d, hipMemcpyHostToDevice, s));
  // exact_gp.py:141-150 (the same normalisation for every parameter set)
  hipLaunchKernelGGL(k_normalise, dim3(1), dim3(256), 0, s, n, 1, dY.as<double>(), dyn.as<double>(),
                     dm.as<double>(), dsd.as<double>());
  auto build = [&](int b, double jit) -> hipError_t {  // K_b + noise_b I (+ jit I)
    double *Kb = Kbuf + nn * b;
    hipError_t e = launch_gram(s, kind, Xs.as<double>() + (size_t)b * n * d,
                               Xn.as<double>() + (size_t)b * n, n,
                               Xs.as<double>() + (size_t)b * n * d, Xn.as<double>() + (size_t)b * n,
                               n, d, sigma2[b], iso ? 1.0 / (2.0 * ls[(size_t)b * d] * ls[(size_t)b * d]) : 0.0,
                               Kb, n, 0);
    if (e == hipSuccess) e = launch_add_diag(s, n, Kb, n, noise[b], 1, 0);
    if (e == hipSuccess && jit > 0.0) e = launch_add_diag(s, n, Kb, n, jit, 1, 0);
    return e;
  };
  for (int b = 0; b < B; ++b) {
    GPMPC_HIP(launch_scale_rows(s, dX.as<double>(), n, d, dls.as<double>() + (size_t)b * d, iso,
                                Xs.as<double>() + (size_t)b * n * d, Xn.as<double>() + (size_t)b * n));
    GPMPC_HIP(build(b, 0.0));
  }
  GPMPC_HIP(launch_potrf_batched(s, n, B, Kbuf, n, (int64_t)nn, dinfo.as<int>()));
  std::vector<int> info(B);
  GPMPC_HIP(hipMemcpyAsync(info.data(), dinfo.p, sizeof(int) * B, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  // jitter ladder (exact_gp.py:163-175) for the sets whose first factorisation failed
  for (int b = 0; b < B; ++b) {
    jitter_steps[b] = 0;
    if (info[b] < 0) return gpmpc_potrf_info_error(info[b], "gp_lml_batched");
    if (!info[b]) continue;
    double jit = 1e-6;
    int steps = 1, ok = 0;
    while (jit < 1.0) {
      GPMPC_HIP(build(b, jit));
      GPMPC_HIP(launch_potrf_batched(s, n, 1, Kbuf + nn * b, n, 0,
                                     dinfo.as<int>() + b));
      int ib = 0;
      GPMPC_HIP(hipMemcpyAsync(&ib, dinfo.as<int>() + b, sizeof(int), hipMemcpyDeviceToHost, s));
      GPMPC_HIP(hipStreamSynchronize(s));
      if (ib < 0) return gpmpc_potrf_info_error(ib, "gp_lml_batched");
      if (!ib) { ok = 1; break; }
      jit *= 10;
      ++steps;
    }
    jitter_steps[b] = ok ? steps : -1;
  }
  static const bool attr = hipFuncSetAttribute((const void *)k_lml_trsv,
                                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                                160 * 1024) == hipSuccess;
  if (!attr) {
    gpmpc_set_error("gp_lml_batched: LDS attribute");
    return -1;
  }
  hipLaunchKernelGGL(k_lml_trsv, dim3(B), dim3(256), sizeof(double) * (n + 4), s, n,
                     Kbuf, (int64_t)nn, dyn.as<double>(), dinfo.as<int>(),
                     dlml.as<double>());
  GPMPC_HIP(hipGetLastError());
  GPMPC_HIP(hipMemcpyAsync(lml, dlml.p, sizeof(double) * B, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  for (int b = 0; b < B; ++b)
    if (jitter_steps[b] < 0) lml[b] = -INFINITY;
  return 0;
}

// ---------------------------------------------------------------------------
// incremental exact GP -- append k training rows to a fitted GP in
// O(n^2 k) instead of the O(n^3) refit on the concatenated data
// (SparseGP.update semantics, sparse_gp.py:328-353; the online refit cadence of
// online_update.py:361-408).  With K = [[K11, K12], [K21, K22]]:
//   B^T = K21 W^T              (W = L11^-1, the stored inverse)
//   S   = K22 + noise I - B^T B,  Ls = chol(S)
//   L   = [[L11, 0], [B^T, Ls]],  W = [[W, 0], [-Ls^-1 B^T W, Ls^-1]]
// then the targets of all n + k rows are renormalised (exact_gp.py:141-150) and
// alpha = W^T W y, lml as in the fit.  The refit's plain Cholesky of K succeeds
// exactly when L11's did and S is positive definite; a GP fitted with jitter, or
// an indefinite S, returns GPMPC_ERR_NOT_PD with the handle unchanged, and the
// caller refits (the refit reruns the jitter ladder on the whole matrix).
extern "C" int gpmpc_gp_append(gpmpc_ctx *ctx, gpmpc_gp *gp, const double *Xnew, int k,
                               const double *Yall, double *y_mean, double *y_std, double *lml) {
  GPMPC_CHECK_ARG(ctx && gp && Xnew && Yall && k >= 1);
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  GpCore &g = gp->core;
  if (gp->jitter_steps != 0) {
    gpmpc_set_error("gp_append: the GP was fitted with jitter; refit the concatenated data");
    return GPMPC_ERR_NOT_PD;
  }
  if (g.kind == GPMPC_KPROG) {
    gpmpc_set_error("gp_append: composite-kernel GP; refit the concatenated data");
    return GPMPC_ERR_NOT_PD;
  }
  const int n = g.n, m = n + k, d = g.d, no = g.n_out;
  // temporaries carved from persistent scratch (slot 4): a per-call hipMalloc /
  // hipFree of each cost more than the O(n^2 k) arithmetic
  const size_t need = 64 + 32 * 16 + (size_t)k * d * 2 + k + (size_t)k * n * 3 + (size_t)k * k * 2 +
                      (size_t)m * no * 4 + no * 3;
  double *scr = (double *)gpmpc_scratch(ctx->stream, 4, sizeof(double) * need);
  if (!scr) {
    gpmpc_set_error("gp_append: out of device memory");
    return -1;
  }
  ScratchCarve cv{scr};
  ScratchPtr xr{cv.take((size_t)k * d)}, xs{cv.take((size_t)k * d)}, xn{cv.take(k)},
      Kt{cv.take((size_t)k * n)}, Bt{cv.take((size_t)k * n)}, Sm{cv.take((size_t)k * k)},
      Li{cv.take((size_t)k * k)}, C{cv.take((size_t)k * n)}, dinfo{cv.take(1)};
  GPMPC_HIP(hipMemcpyAsync(xr.p, Xnew, sizeof(double) * k * d, hipMemcpyHostToDevice, s));
  GPMPC_HIP(launch_scale_rows(s, xr.as<double>(), k, d, g.ls.as<double>(), g.kind == GPMPC_SE_ISO,
                              xs.as<double>(), xn.as<double>()));
  // K21 (k x n), B^T = K21 W^T, S = K22 + noise I - B^T B
  GPMPC_HIP(launch_gram(s, g.kind, xs.as<double>(), xn.as<double>(), k, g.Xs.as<double>(),
                        g.Xn.as<double>(), n, d, g.sigma2, g.iso_scale, Kt.as<double>(), n, 0));
  GPMPC_HIP(launch_gemm_nt(s, EPI_STORE, k, n, n, Kt.as<double>(), n, g.W.as<double>(), n,
                           Bt.as<double>(), n, 1.0, 0.0, 0, 0, 1, 0, 0, 0));
  GPMPC_HIP(launch_gram(s, g.kind, xs.as<double>(), xn.as<double>(), k, xs.as<double>(),
                        xn.as<double>(), k, d, g.sigma2, g.iso_scale, Sm.as<double>(), k, 0));
  GPMPC_HIP(launch_add_diag(s, k, Sm.as<double>(), k, gp->noise, 1, 0));
  GPMPC_HIP(launch_gemm_nt(s, EPI_STORE, k, k, n, Bt.as<double>(), n, Bt.as<double>(), n,
                           Sm.as<double>(), k, -1.0, 1.0, 0, 0, 1, 0, 0, 0));
  GPMPC_HIP(launch_potrf_batched(s, k, 1, Sm.as<double>(), k, 0, dinfo.as<int>()));
  // the pivot check comes with the one read-back below: nothing before the commit
  // touches the handle, so a failed factor only discards the new buffers
  // Ls^-1 (lower) and the new rows of W: [-(Ls^-1 (B^T W)) | Ls^-1]
  hipLaunchKernelGGL(k_eye, dim3((k + 255) / 256, k), dim3(256), 0, s, k, Li.as<double>());
  GPMPC_HIP(launch_trsm_lower_ex(s, k, k, Sm.as<double>(), k, Li.as<double>(), k, 0, 1, nullptr));
  GPMPC_HIP(launch_gemm_nn(s, k, n, n, Bt.as<double>(), n, g.W.as<double>(), n, C.as<double>(), n,
                           1.0, 0.0));
  DevBuf L2, W2, Xs2, Xn2, alphaT;  // kept by the handle
  ScratchPtr yraw{cv.take((size_t)m * no)}, yn{cv.take((size_t)m * no)}, t{cv.take((size_t)m * no)},
      alpha{cv.take((size_t)m * no)}, dlml{cv.take(no)}, ym{cv.take(no)}, ys{cv.take(no)};
  GPMPC_HIP(L2.alloc(s, sizeof(double) * (size_t)m * m));
  GPMPC_HIP(W2.alloc(s, sizeof(double) * (size_t)(m + no) * m));
  GPMPC_HIP(Xs2.alloc(s, sizeof(double) * (size_t)m * d));
  GPMPC_HIP(Xn2.alloc(s, sizeof(double) * m));
  GPMPC_HIP(alphaT.alloc(s, sizeof(double) * (size_t)no * m));
  GPMPC_HIP(hipMemsetAsync(L2.p, 0, sizeof(double) * (size_t)m * m, s));
  GPMPC_HIP(hipMemsetAsync(W2.p, 0, sizeof(double) * (size_t)(m + no) * m, s));
  const size_t rowb = sizeof(double) * n;
  GPMPC_HIP(hipMemcpy2DAsync(L2.p, sizeof(double) * m, gp->L.p, rowb, rowb, n,
                             hipMemcpyDeviceToDevice, s));
  GPMPC_HIP(hipMemcpy2DAsync(L2.as<double>() + (size_t)n * m, sizeof(double) * m, Bt.p, rowb, rowb,
                             k, hipMemcpyDeviceToDevice, s));
  GPMPC_HIP(hipMemcpy2DAsync(L2.as<double>() + (size_t)n * m + n, sizeof(double) * m, Sm.p,
                             sizeof(double) * k, sizeof(double) * k, k, hipMemcpyDeviceToDevice, s));
  GPMPC_HIP(hipMemcpy2DAsync(W2.p, sizeof(double) * m, g.W.p, rowb, rowb, n,
                             hipMemcpyDeviceToDevice, s));
  GPMPC_HIP(launch_gemm_nn(s, k, n, k, Li.as<double>(), k, C.as<double>(), n,
                           W2.as<double>() + (size_t)n * m, m, -1.0, 0.0));
  GPMPC_HIP(hipMemcpy2DAsync(W2.as<double>() + (size_t)n * m + n, sizeof(double) * m, Li.p,
                             sizeof(double) * k, sizeof(double) * k, k, hipMemcpyDeviceToDevice, s));
  // training rows
  GPMPC_HIP(hipMemcpyAsync(Xs2.p, g.Xs.p, sizeof(double) * (size_t)n * d, hipMemcpyDeviceToDevice, s));
  GPMPC_HIP(hipMemcpyAsync(Xs2.as<double>() + (size_t)n * d, xs.p, sizeof(double) * (size_t)k * d,
                           hipMemcpyDeviceToDevice, s));
  GPMPC_HIP(hipMemcpyAsync(Xn2.p, g.Xn.p, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
  GPMPC_HIP(hipMemcpyAsync(Xn2.as<double>() + n, xn.p, sizeof(double) * k, hipMemcpyDeviceToDevice, s));
  // all targets renormalised (into scratch: the handle's mean / std change only
  // at the commit below); alpha = W^T (W y); lml
  GPMPC_HIP(hipMemcpyAsync(yraw.p, Yall, sizeof(double) * (size_t)m * no, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_normalise, dim3(no), dim3(256), 0, s, m, no, yraw.as<double>(),
                     yn.as<double>(), ym.as<double>(), ys.as<double>());
  GPMPC_HIP(launch_gemm_nn(s, m, no, m, W2.as<double>(), m, yn.as<double>(), no, t.as<double>(), no,
                           1.0, 0.0));
  GPMPC_HIP(launch_gemm_tn(s, m, no, m, W2.as<double>(), m, t.as<double>(), no, alpha.as<double>(),
                           no, 1.0, 0.0));
  hipLaunchKernelGGL(k_lml_exact, dim3(no), dim3(256), 0, s, m, no, L2.as<double>(), yn.as<double>(),
                     alpha.as<double>(), alphaT.as<double>(), dlml.as<double>());
  GPMPC_HIP(hipMemcpyAsync(W2.as<double>() + (size_t)m * m, alphaT.p, sizeof(double) * (size_t)no * m,
                           hipMemcpyDeviceToDevice, s));
  std::vector<double> hl(no), hm(no), hs(no);
  int info = 0;
  GPMPC_HIP(hipMemcpyAsync(&info, dinfo.p, sizeof(int), hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipMemcpyAsync(hm.data(), ym.p, sizeof(double) * no, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipMemcpyAsync(hs.data(), ys.p, sizeof(double) * no, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipMemcpyAsync(hl.data(), dlml.p, sizeof(double) * no, hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  if (info < 0) return gpmpc_potrf_info_error(info, "gp_append");
  if (info) {
    gpmpc_set_error("gp_append: Schur complement not positive definite (pivot %d); refit", info);
    return GPMPC_ERR_NOT_PD;
  }
  // commit: the new normalisation, then swap the grown buffers into the handle
  // (nothing below can fail half-way: the copies are of buffers already sized; the
  // device synchronisation at the end covers them)
  GPMPC_HIP(hipMemcpyAsync(g.ymean.p, ym.p, sizeof(double) * no, hipMemcpyDeviceToDevice, s));
  GPMPC_HIP(hipMemcpyAsync(g.ystd.p, ys.p, sizeof(double) * no, hipMemcpyDeviceToDevice, s));
  g.h_ymean = hm;
  g.h_ystd = hs;
  gp->L.swap(L2);
  g.W.swap(W2);
  g.alphaT.swap(alphaT);
  g.Xs.swap(Xs2);
  g.Xn.swap(Xn2);
  g.n = m;
  if (core_pack(s, g) != hipSuccess) {  // the handle is committed: predicts take the K* path
    (void)hipGetLastError();
    g.Wf.release();
    g.Xp.release();
  }
  // the replaced buffers go back to the pool when this returns; another context's
  // stream may still be reading them (as gpmpc_gp_destroy)
  (void)hipDeviceSynchronize();
  for (int c = 0; c < no; ++c) {
    if (lml) lml[c] = hl[c];
    if (y_mean) y_mean[c] = g.h_ymean[c];
    if (y_std) y_std[c] = g.h_ystd[c];
  }
  return 0;
}
