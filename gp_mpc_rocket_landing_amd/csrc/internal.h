// internal.h -- shared helpers for libgpmpc_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include "../../include/gpmpc.h"

struct gpmpc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
};

void gpmpc_set_error(const char *fmt, ...);
// persistent scratch per stream (= per context; slots: 0 trsm block inverses,
// 1 potrf 32x32 inverses, 2 potrf 128x128 inverses, 3 batched-LML Gram/factor
// matrices, 4 gp_append temporaries, 5 split-K partials, 7 the Stage device arena; slots 0..7).  Valid until the next call
// on the same stream that asks the slot for more bytes.
#define GPMPC_SCRATCH_SLOTS 8
void *gpmpc_scratch(hipStream_t s, int slot, size_t bytes);

#define GPMPC_HIP(call)                                                               \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess) {                                                           \
      gpmpc_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      return -1;                                                                      \
    }                                                                                 \
  } while (0)

#define GPMPC_CHECK_ARG(cond)                                    \
  do {                                                           \
    if (!(cond)) {                                               \
      gpmpc_set_error("%s:%d bad argument: %s", __FILE__, __LINE__, #cond); \
      return -2;                                                 \
    }                                                            \
  } while (0)

// Per-stream caching pool for the temporaries of host-boundary calls (fits, predicts,
// solves): a released block goes back to its stream's free list instead of hipFree
// (an implicit device-wide synchronisation, ~41 us a call: ~15 per exact fit, DESIGN
// §11).  A block is handed out again only on the stream it was last used on, so that
// stream's order keeps its earlier readers ahead of the next writer.  Blocks are sized
// in classes (<= 12.5% rounding), cached up to a per-stream cap (GPMPC_POOL_CAP_MB, 8 GB),
// and released with the context (gpmpc_ctx_destroy); a failed hipMalloc first gives the
// stream's cached blocks back and retries.  gen: the pool generation the block came from
// (a block returned after its context's destruction is freed, not cached).
void *gpmpc_pool_get(hipStream_t s, size_t bytes, size_t *cls, uint64_t *gen);
void gpmpc_pool_put(hipStream_t s, void *p, size_t cls, uint64_t gen);

// RAII device buffer (host-side bookkeeping only).  alloc(bytes): its own hipMalloc
// (handle-owned state that outlives the call); alloc(stream, bytes): a pooled
// temporary of that stream.
struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  hipStream_t pool = nullptr;  // non-null: pooled on this stream
  size_t cls = 0;
  uint64_t gen = 0;            // the pool generation it came from
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) {
      if (pool) gpmpc_pool_put(pool, p, cls, gen);
      else (void)hipFree(p);
    }
    p = nullptr;
    pool = nullptr;
  }
  hipError_t alloc(size_t b) {
    release();
    bytes = b;
    return b ? hipMalloc(&p, b) : hipSuccess;
  }
  hipError_t alloc(hipStream_t s, size_t b) {
    release();
    bytes = b;
    if (!b) return hipSuccess;
    p = gpmpc_pool_get(s, b, &cls, &gen);
    if (!p) return hipErrorOutOfMemory;
    pool = s;
    return hipSuccess;
  }
  void swap(DevBuf &o) {
    std::swap(p, o.p); std::swap(bytes, o.bytes); std::swap(pool, o.pool); std::swap(cls, o.cls);
    std::swap(gen, o.gen);
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

// Staging for the host-buffer entry points: a call packs its inputs into one pinned
// arena and uploads them with ONE copy, and places its outputs in one device range
// read back with ONE copy (a pageable hipMemcpyAsync costs 10-30 us of host time; a
// single-landing QP solve made 14 of them).  The arenas are per stream (= per
// context; device side = gpmpc_scratch slot 7), grown after the stream drains, and
// valid until the next Stage on the stream.  Order of use: in() for pure inputs,
// inout() for buffers both read and written back, then out(); upload() after the
// last in/inout, download() after the last kernel (it synchronises the stream).
char *gpmpc_stage_host(hipStream_t s, size_t bytes);
void gpmpc_qp_cache_release(hipStream_t s);  // qp.hip: the stream's kept QP pattern
struct Stage {
  struct Back { void *dst; size_t off, bytes; };
  hipStream_t s;
  char *h = nullptr, *d = nullptr;
  size_t off = 0, in_end = 0, back_lo = (size_t)-1, cap = 0;
  bool bad = false;  // a buffer past the arena (the caller's byte count was short): upload() refuses
  Back backs[24];
  int nback = 0;
  static size_t pad(size_t b) { return (b + 255) & ~(size_t)255; }
  // bytes: the sum of pad(size) over every buffer the call stages
  Stage(hipStream_t st, size_t bytes) : s(st), cap(bytes) {
    h = gpmpc_stage_host(s, bytes);
    d = (char *)gpmpc_scratch(s, 7, bytes);
  }
  bool fits(size_t b) {
    if (off + pad(b) <= cap) return true;
    bad = true;
    return false;
  }
  bool ok() const { return h && d; }
  template <class T> T *in(const T *src, size_t n) {
    const size_t b = sizeof(T) * n;
    if (!fits(b)) return (T *)d;
    if (b) memcpy(h + off, src, b);
    T *r = (T *)(d + off);
    off += pad(b);
    return r;
  }
  template <class T> T *inout(T *src, size_t n) {
    const size_t o = off;
    T *r = in(src, n);
    if (!bad) back(src, o, sizeof(T) * n);
    return r;
  }
  template <class T> T *out(T *dst, size_t n) {
    const size_t o = off;
    if (!fits(sizeof(T) * n)) return (T *)d;
    off += pad(sizeof(T) * n);
    back(dst, o, sizeof(T) * n);
    return (T *)(d + o);
  }
  void back(void *dst, size_t o, size_t b) {
    if (o < back_lo) back_lo = o;
    if (nback < (int)(sizeof(backs) / sizeof(backs[0]))) backs[nback] = Back{dst, o, b};
    ++nback;  // (past the table: download() refuses)
  }
  hipError_t upload() {
    if (bad) return hipErrorInvalidValue;
    in_end = off;
    return off ? hipMemcpyAsync(d, h, off, hipMemcpyHostToDevice, s) : hipSuccess;
  }
  hipError_t download() {
    if (bad || nback > (int)(sizeof(backs) / sizeof(backs[0]))) return hipErrorInvalidValue;
    if (nback) {
      hipError_t e = hipMemcpyAsync(h + back_lo, d + back_lo, off - back_lo, hipMemcpyDeviceToHost, s);
      if (e != hipSuccess) return e;
    }
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    for (int i = 0; i < nback; ++i)
      if (backs[i].bytes) memcpy(backs[i].dst, h + backs[i].off, backs[i].bytes);
    return hipSuccess;
  }
};

// kernel value from r^2 of the length-scaled rows (the k_gram epilogue; shared
// so that every kernel that forms K*(x, x') produces the same bits)
__device__ __forceinline__ double kernel_epilogue(int kind, double d2, double sigma2,
                                                  double iso_scale) {
  d2 = d2 > 0.0 ? d2 : 0.0;  // np.maximum(dist_sq, 0.0)
  switch (kind) {
    case GPMPC_SE_ARD: return sigma2 * exp(-0.5 * d2);
    case GPMPC_SE_ISO: return sigma2 * exp(-d2 * iso_scale);
    case GPMPC_MATERN32: {
      double r = sqrt(d2);
      double s3 = 1.7320508075688772 * r;
      return sigma2 * (1.0 + s3) * exp(-s3);
    }
    default: {
      double r = sqrt(d2);
      double s5 = 2.23606797749979 * r;
      return sigma2 * (1.0 + s5 + 5.0 * (r * r) / 3.0) * exp(-s5);
    }
  }
}

// ---- internal device entry points shared across translation units ----------
// Gram: K (n1 x n2, ldk) from pre-scaled rows (a = X1/ls, b = X2/ls) and their
// squared norms; kind selects the epilogue.
hipError_t launch_gram(hipStream_t s, int kind, const double *a, const double *na, int n1,
                       const double *b, const double *nb, int n2, int d, double sigma2,
                       double iso_scale, double *K, int64_t ldk, int transpose_out);
#define GPMPC_KPROG 16  // GpCore kind of a composite-kernel program
// composite kernel programs (gram.hip; codes GPMPC_KP_* in gpmpc.h): Gram of raw rows,
// same = 1: one row set (X2 ignored; WhiteNoise on the diagonal)
hipError_t launch_gram_prog(hipStream_t s, const int *ops, int nops, const double *par, const double *X1, int n1,
                            const double *X2, int n2, int d, int same, double *K, int64_t ldk);
int kprog_check(const int *ops, int nops, int npar, int d, const double *par, double *diag);
// rows / lengthscales -> scaled rows + squared norms
hipError_t launch_scale_rows(hipStream_t s, const double *X, int n, int d, const double *ls,
                             int iso, double *out, double *norms);
// blocked Cholesky of batch matrices; info (device int[batch]), 1-based pivot
hipError_t launch_potrf_batched(hipStream_t s, int n, int batch, double *A, int64_t lda,
                                int64_t stride, int *info);
// info < 0 from the blocked Cholesky: the 128-column diagonal kernel's bounded wait
// for an LDS step flag expired (a broken invariant, not a non-PD matrix); the factor of
// that matrix is unreliable and is never reported as success or as a pivot column
#define GPMPC_POTRF_SWEEP_TIMEOUT (-1)
int gpmpc_potrf_info_error(int info, const char *what);  // sets the message, returns the code
// X <- L^-1 X (L lower n x n, X n x nrhs row-major ld ldx), batch via strides
hipError_t launch_trsm_lower(hipStream_t s, int n, int nrhs, const double *L, int64_t ldl,
                             double *X, int64_t ldx, int transpose_L);
// add value to the diagonal of A
hipError_t launch_add_diag(hipStream_t s, int n, double *A, int64_t lda, double v, int batch,
                           int64_t stride);
// copy lower triangle of src into dst and zero the strict upper part of dst
hipError_t launch_copy_lower(hipStream_t s, int n, const double *src, int64_t lds, double *dst,
                             int64_t ldd);

// read-only view of a fitted exact GP (gp.hip) for the fleet
struct GpView {
  int kind, n, d, n_out;
  double sigma2, iso_scale;
  const double *ls, *Xs, *Xn, *W, *alphaT, *ymean, *ystd;
  const double *Wf, *Xp;  // column-stationary posterior operands (post.hip), or null
};
GpView gp_view(const gpmpc_gp *gp);
// the exact GP's posterior of p device-resident raw query rows (gp.hip): mean / var (p x n_out)
int gp_posterior_dev(gpmpc_ctx *ctx, gpmpc_gp *gp, const double *dq, int p, double *dmean, double *dvar);
// the same for a FITC GP (gp.hip, the gpmpc_fitc_predict arithmetic)
int fitc_posterior_dev(gpmpc_ctx *ctx, gpmpc_fitc *gp, const double *dq, int p, double *dmean, double *dvar);
// the same view of a FITC GP: n = inducing points, Xs / Xn their scaled rows, alphaT
GpView fitc_view(const gpmpc_fitc *gp);
// its W2 = L_B^-1 L_uu^-1 (n x n lower): the predict's w = W2 k* (sparse_gp.py:293-296)
const double *fitc_W2(const gpmpc_fitc *gp);
// the sparse posterior finish (k_fitc_finish): var = sigma2 - sum pv + sum pw, mean
hipError_t launch_fitc_finish(hipStream_t s, int P, int n_out, int nrv, int nrw, const double *pv,
                              const double *pw, int64_t ldp, const double *meanT, int64_t ldm,
                              const double *ymean, const double *ystd, double sigma2, double *mean,
                              double *var);
// posterior finish: var/mean (P x n_out) from SUMSQ partials and K* alpha (gp.hip)
hipError_t launch_post_finish(hipStream_t s, int P, int n_out, int nrt, const double *part,
                              int64_t ldp, const double *meanT, int64_t ldm, const double *ymean,
                              const double *ystd, double sigma2, double *mean, double *var);
