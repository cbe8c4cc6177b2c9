// ctx.hip -- context, error reporting, small utility kernels.
#include "internal.h"
#include <cstdarg>
#include <mutex>
#include <cstdlib>

static thread_local char g_err[1024] = "";

void gpmpc_set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Persistent device scratch per (stream, slot), grown with hipMalloc after the
// stream has drained.  Every context owns one stream, so two contexts (e.g. on
// two threads) never share a buffer; gpmpc_ctx_destroy releases its stream's
// slots.  (Stream-ordered hipMallocAsync scratch returned buffers the next
// kernel on the same stream did not see written on ROCm 7.2 -- see DESIGN.md.)
#include <map>
#include <array>
struct ScratchSlot { void *p = nullptr; size_t bytes = 0; };
static std::mutex g_scratch_mu;
static std::map<hipStream_t, std::array<ScratchSlot, GPMPC_SCRATCH_SLOTS>> g_scratch;

void *gpmpc_scratch(hipStream_t s, int slot, size_t bytes) {
  if (slot < 0 || slot >= GPMPC_SCRATCH_SLOTS) return nullptr;
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  ScratchSlot &e = g_scratch[s][slot];
  if (e.bytes < bytes) {
    (void)hipStreamSynchronize(s);  // earlier work on this stream may still read it
    if (e.p) (void)hipFree(e.p);
    e.p = nullptr;
    e.bytes = 0;
    if (hipMalloc(&e.p, bytes) != hipSuccess) return nullptr;
    e.bytes = bytes;
  }
  return e.p;
}

// Pinned host arena of a stream's Stage (internal.h), grown like the scratch slots.
struct StageHost { char *p = nullptr; size_t bytes = 0; };
static std::map<hipStream_t, StageHost> g_stage;

char *gpmpc_stage_host(hipStream_t s, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  StageHost &e = g_stage[s];
  if (e.bytes < bytes) {
    (void)hipStreamSynchronize(s);  // a copy on this stream may still read or fill it
    if (e.p) (void)hipHostFree(e.p);
    e.p = nullptr;
    e.bytes = 0;
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    e.p = (char *)p;
    e.bytes = bytes;
  }
  return e.p;
}

// ---- per-stream caching pool (internal.h) ------------------------------------
// Each stream's pool carries a generation: a context's destruction ends its pool,
// and a later context whose stream handle happens to have the same value starts a
// new generation, so a block allocated under the old one (a handle that outlived
// its context) is freed on return instead of joining a stranger's free list.
#include <vector>
struct StreamPool {
  std::map<size_t, std::vector<void *>> free;  // size class -> cached blocks
  size_t cached = 0;
  uint64_t gen = 0;
};
static std::mutex g_pool_mu;
static std::map<hipStream_t, StreamPool> g_pool;
static uint64_t g_pool_gen = 0;

static size_t pool_cap() {  // per stream; GPMPC_POOL_CAP_MB overrides the 8 GB default
  static const size_t cap = [] {
    const char *e = getenv("GPMPC_POOL_CAP_MB");
    return e ? (size_t)strtoull(e, nullptr, 10) << 20 : (size_t)8 << 30;
  }();
  return cap;
}

static size_t pool_class(size_t b) {
  if (b <= 256) return 256;
  size_t p2 = 256;
  while (p2 < b) p2 <<= 1;
  const size_t g = p2 >= 2048 ? p2 / 8 : 256;  // eighths of the power of two above
  return (b + g - 1) / g * g;
}

static StreamPool &pool_of(hipStream_t s) {  // g_pool_mu held
  auto it = g_pool.find(s);
  if (it == g_pool.end()) {
    it = g_pool.emplace(s, StreamPool{}).first;
    it->second.gen = ++g_pool_gen;
  }
  return it->second;
}

// drop every cached block of stream s (after s has drained: its kernels may still read them)
static void pool_trim(hipStream_t s) {
  std::vector<void *> blocks;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto it = g_pool.find(s);
    if (it == g_pool.end()) return;
    for (auto &kv : it->second.free)
      for (void *p : kv.second) blocks.push_back(p);
    it->second.free.clear();
    it->second.cached = 0;
  }
  for (void *p : blocks) (void)hipFree(p);
}

void *gpmpc_pool_get(hipStream_t s, size_t bytes, size_t *cls, uint64_t *gen) {
  const size_t c = pool_class(bytes);
  *cls = c;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    StreamPool &sp = pool_of(s);
    *gen = sp.gen;
    auto it = sp.free.find(c);
    if (it != sp.free.end() && !it->second.empty()) {
      void *p = it->second.back();
      it->second.pop_back();
      sp.cached -= c;
      return p;
    }
  }
  void *p = nullptr;
  if (hipMalloc(&p, c) == hipSuccess) return p;
  // out of memory: the stream's cached blocks are the first thing to give back
  // (ADVICE r4), then one retry
  (void)hipGetLastError();
  (void)hipStreamSynchronize(s);
  pool_trim(s);
  p = nullptr;
  if (hipMalloc(&p, c) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void gpmpc_pool_put(hipStream_t s, void *p, size_t cls, uint64_t gen) {
  if (!p) return;
  bool live = false;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto it = g_pool.find(s);
    live = it != g_pool.end() && it->second.gen == gen;
    if (live && it->second.cached + cls <= pool_cap()) {
      it->second.free[cls].push_back(p);
      it->second.cached += cls;
      return;
    }
  }
  // over the cap: let the stream's earlier readers finish first; a block whose pool
  // generation is gone belongs to a destroyed context (hipFree synchronises the device)
  if (live) (void)hipStreamSynchronize(s);
  (void)hipFree(p);
}

static void pool_release(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  auto it = g_pool.find(s);
  if (it == g_pool.end()) return;
  for (auto &kv : it->second.free)
    for (void *p : kv.second) (void)hipFree(p);
  g_pool.erase(it);
}

static void scratch_release(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  auto st = g_stage.find(s);
  if (st != g_stage.end()) {
    if (st->second.p) (void)hipHostFree(st->second.p);
    g_stage.erase(st);
  }
  auto it = g_scratch.find(s);
  if (it == g_scratch.end()) return;
  for (ScratchSlot &e : it->second)
    if (e.p) (void)hipFree(e.p);
  g_scratch.erase(it);
}

extern "C" int gpmpc_abi_version(void) { return GPMPC_ABI_VERSION; }
extern "C" const char *gpmpc_last_error(void) { return g_err; }

extern "C" int gpmpc_ctx_create(int device, gpmpc_ctx **out) {
  GPMPC_CHECK_ARG(out != nullptr);
  int ndev = 0;
  GPMPC_HIP(hipGetDeviceCount(&ndev));
  GPMPC_CHECK_ARG(device >= 0 && device < ndev);
  GPMPC_HIP(hipSetDevice(device));
  auto *c = new gpmpc_ctx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    gpmpc_set_error("hipStreamCreate: %s", hipGetErrorString(e));
    return -1;
  }
  *out = c;
  return 0;
}

extern "C" int gpmpc_ctx_destroy(gpmpc_ctx *ctx) {
  if (!ctx) return 0;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->stream) scratch_release(ctx->stream);
  if (ctx->stream) gpmpc_qp_cache_release(ctx->stream);
  if (ctx->stream) pool_release(ctx->stream);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return 0;
}

extern "C" int gpmpc_ctx_sync(gpmpc_ctx *ctx) {
  GPMPC_CHECK_ARG(ctx != nullptr);
  GPMPC_HIP(hipStreamSynchronize(ctx->stream));
  return 0;
}

extern "C" void *gpmpc_ctx_stream(gpmpc_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

// ---------------------------------------------------------------------------
__global__ void k_add_diag(int n, double *A, int64_t lda, double v, int64_t stride) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  double *M = A + (int64_t)blockIdx.y * stride;
  if (i < n) M[(int64_t)i * lda + i] += v;
}

hipError_t launch_add_diag(hipStream_t s, int n, double *A, int64_t lda, double v, int batch,
                           int64_t stride) {
  dim3 g((n + 255) / 256, batch);
  hipLaunchKernelGGL(k_add_diag, g, dim3(256), 0, s, n, A, lda, v, stride);
  return hipGetLastError();
}

__global__ void k_copy_lower(int n, const double *src, int64_t lds, double *dst, int64_t ldd) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  int i = blockIdx.y;
  if (j < n) dst[(int64_t)i * ldd + j] = (j <= i) ? src[(int64_t)i * lds + j] : 0.0;
}

hipError_t launch_copy_lower(hipStream_t s, int n, const double *src, int64_t lds, double *dst,
                             int64_t ldd) {
  dim3 g((n + 255) / 256, n);
  hipLaunchKernelGGL(k_copy_lower, g, dim3(256), 0, s, n, src, lds, dst, ldd);
  return hipGetLastError();
}
