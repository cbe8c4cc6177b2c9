// ctx.hip -- context, error reporting, small utility kernels.
#include "internal.h"
#include <cstdarg>
#include <mutex>

static thread_local char g_err[1024] = "";

void gpmpc_set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Persistent device scratch per (device, slot), grown with hipMalloc after a full
// device sync.  (Stream-ordered hipMallocAsync scratch returned buffers the next
// kernel on the same stream did not see written on ROCm 7.2 -- see DESIGN.md.)
static std::mutex g_scratch_mu;
#define GPMPC_SCRATCH_SLOTS 8
static void *g_scratch[64][GPMPC_SCRATCH_SLOTS];
static size_t g_scratch_bytes[64][GPMPC_SCRATCH_SLOTS];

void *gpmpc_scratch(int slot, size_t bytes) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  if (dev < 0 || dev >= 64 || slot < 0 || slot >= GPMPC_SCRATCH_SLOTS) return nullptr;
  if (g_scratch_bytes[dev][slot] < bytes) {
    (void)hipDeviceSynchronize();
    if (g_scratch[dev][slot]) (void)hipFree(g_scratch[dev][slot]);
    g_scratch[dev][slot] = nullptr;
    g_scratch_bytes[dev][slot] = 0;
    if (hipMalloc(&g_scratch[dev][slot], bytes) != hipSuccess) return nullptr;
    g_scratch_bytes[dev][slot] = bytes;
  }
  return g_scratch[dev][slot];
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
  if (ctx->scratch) (void)hipFree(ctx->scratch);
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
