// comm.hip -- the one collective of SURVEY 8e: every rank's per-landing records
// to the root with one RCCL ncclGather over xGMI.
//
// Landings (monte_carlo.py:401-583) are independent, so the batch is sharded
// in contiguous blocks, one process per GPU, with no data-path collective; at
// the end each rank's record block (count x GPMPC_REC_LEN doubles, device
// resident: gpmpc_fleet_records_dev / gpmpc_rollout6_records_dev) goes to the
// root.  ncclGather takes one send count, so ragged shards are padded on the
// device to the largest shard (rows of NaN) and compacted on the root.
//
// RCCL is resolved at run time (dlopen of librccl.so.1): a process that has
// torch's RCCL loaded (same SONAME) shares that one instance, and a process
// that never gathers never loads RCCL.
#include "internal.h"
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <cmath>
#include <algorithm>
#include <cstring>
#include <vector>

namespace {
struct RcclApi {
  ncclResult_t (*getUniqueId)(ncclUniqueId *) = nullptr;
  ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*commCount)(const ncclComm_t, int *) = nullptr;
  ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char *(*errorString)(ncclResult_t) = nullptr;
  bool ok = false;
};

const RcclApi &rccl() {
  static RcclApi api = [] {
    RcclApi a;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return a;
    a.getUniqueId = (decltype(a.getUniqueId))dlsym(h, "ncclGetUniqueId");
    a.commInitRank = (decltype(a.commInitRank))dlsym(h, "ncclCommInitRank");
    a.commDestroy = (decltype(a.commDestroy))dlsym(h, "ncclCommDestroy");
    a.commCount = (decltype(a.commCount))dlsym(h, "ncclCommCount");
    a.gather = (decltype(a.gather))dlsym(h, "ncclGather");
    a.errorString = (decltype(a.errorString))dlsym(h, "ncclGetErrorString");
    a.ok = a.getUniqueId && a.commInitRank && a.commDestroy && a.commCount && a.gather && a.errorString;
    return a;
  }();
  return api;
}
}  // namespace

#define GPMPC_RCCL(call)                                                                         \
  do {                                                                                           \
    ncclResult_t r_ = (call);                                                                    \
    if (r_ != ncclSuccess) {                                                                     \
      gpmpc_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, rccl().errorString(r_));       \
      return -1;                                                                                 \
    }                                                                                            \
  } while (0)

#define GPMPC_RCCL_LOADED()                                                     \
  do {                                                                          \
    if (!rccl().ok) {                                                           \
      gpmpc_set_error("RCCL (librccl.so.1) could not be loaded: %s", dlerror()); \
      return -1;                                                                \
    }                                                                           \
  } while (0)

struct gpmpc_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  DevBuf send, recv;  // padded blocks (grown on demand)
  bool prepared = false;  // gpmpc_gather_prepare succeeded since the last collective
  // what that prepare was for: the collective must be called with the same counts and
  // root, since the send / receive buffers were sized and padded for them
  int prep_root = -1;
  std::vector<int> prep_counts;
};

extern "C" int gpmpc_comm_unique_id(unsigned char *id) {
  GPMPC_CHECK_ARG(id);
  GPMPC_RCCL_LOADED();
  ncclUniqueId u;
  GPMPC_RCCL(rccl().getUniqueId(&u));
  static_assert(sizeof(u) == GPMPC_COMM_ID_BYTES, "ncclUniqueId size");
  memcpy(id, &u, sizeof(u));
  return 0;
}

extern "C" int gpmpc_comm_init(gpmpc_ctx *ctx, const unsigned char *id, int nranks, int rank, gpmpc_comm **out) {
  GPMPC_CHECK_ARG(ctx && id && out && nranks >= 1 && rank >= 0 && rank < nranks);
  GPMPC_RCCL_LOADED();
  GPMPC_HIP(hipSetDevice(ctx->device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  auto *c = new gpmpc_comm();
  c->nranks = nranks; c->rank = rank; c->device = ctx->device;
  const ncclResult_t r = rccl().commInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    gpmpc_set_error("ncclCommInitRank(%d ranks, rank %d) -> %s", nranks, rank, rccl().errorString(r));
    delete c;
    return -1;
  }
  *out = c;
  return 0;
}

extern "C" int gpmpc_comm_destroy(gpmpc_comm *c) {
  if (!c) return 0;
  if (c->comm && rccl().ok) (void)rccl().commDestroy(c->comm);
  delete c;
  return 0;
}

// the number of ranks RCCL's communicator spans (ncclCommCount), so a caller can
// record what the collective actually saw rather than what it asked for
extern "C" int gpmpc_comm_count(gpmpc_comm *c, int *nranks) {
  GPMPC_CHECK_ARG(c && c->comm && nranks);
  GPMPC_RCCL_LOADED();
  GPMPC_RCCL(rccl().commCount(c->comm, nranks));
  return 0;
}

// padded block: rows [0, count) copied, [count, cmax) NaN
__global__ void k_pad_records(int count, int cmax, const double *__restrict__ src, double *__restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cmax * GPMPC_REC_LEN) return;
  dst[i] = i < count * GPMPC_REC_LEN ? src[i] : __builtin_nan("");
}

// The gather in two steps, so that ranks can agree between them: every
// failure a rank can meet on its own (argument checks, the send / receive buffers'
// allocation, the pad kernel) happens in gpmpc_gather_prepare, which ends with the
// stream drained; gpmpc_gather_collective then only issues the ncclGather and the
// root's compaction.  A caller agrees on every rank's prepare status (one all-reduce)
// before any rank enters the collective.
struct GatherPlan {
  int cmax = 0, total = 0;
};

static int gather_plan(gpmpc_comm *c, const int *counts, int root, GatherPlan &p) {
  GPMPC_CHECK_ARG(counts && root >= 0 && root < c->nranks);
  p = GatherPlan{};
  for (int r = 0; r < c->nranks; ++r) {
    GPMPC_CHECK_ARG(counts[r] >= 0);
    p.cmax = counts[r] > p.cmax ? counts[r] : p.cmax;
    p.total += counts[r];
  }
  return 0;
}

extern "C" int gpmpc_gather_prepare(gpmpc_ctx *ctx, gpmpc_comm *c, const double *d_records, const int *counts,
                                    int root) {
  GPMPC_CHECK_ARG(ctx && c);
  GPMPC_CHECK_ARG(c->device == ctx->device);
  GatherPlan p;
  if (int rc = gather_plan(c, counts, root, p)) return rc;
  const int count = counts[c->rank];
  GPMPC_CHECK_ARG(count == 0 || d_records);
  c->prepared = false;
  if (p.cmax == 0) {
    c->prep_root = root;
    c->prep_counts.assign(counts, counts + c->nranks);
    c->prepared = true;
    return 0;
  }
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const size_t blk = (size_t)p.cmax * GPMPC_REC_LEN;
  if (c->send.bytes < blk * sizeof(double)) GPMPC_HIP(c->send.alloc(blk * sizeof(double)));
  if (c->rank == root && c->recv.bytes < blk * c->nranks * sizeof(double))
    GPMPC_HIP(c->recv.alloc(blk * c->nranks * sizeof(double)));
  hipLaunchKernelGGL(k_pad_records, dim3((unsigned)((blk + 255) / 256)), dim3(256), 0, s, count, p.cmax, d_records,
                     c->send.as<double>());
  GPMPC_HIP(hipGetLastError());
  GPMPC_HIP(hipStreamSynchronize(s));
  c->prep_root = root;
  c->prep_counts.assign(counts, counts + c->nranks);
  c->prepared = true;
  return 0;
}

extern "C" int gpmpc_gather_collective(gpmpc_ctx *ctx, gpmpc_comm *c, const int *counts, int root, double *out) {
  GPMPC_CHECK_ARG(ctx && c);
  GatherPlan p;
  if (int rc = gather_plan(c, counts, root, p)) return rc;
  GPMPC_CHECK_ARG(c->rank != root || out || p.total == 0);
  if (!c->prepared) {
    gpmpc_set_error("gather: gpmpc_gather_prepare did not succeed on this rank");
    return -2;
  }
  if (root != c->prep_root || !std::equal(c->prep_counts.begin(), c->prep_counts.end(), counts)) {
    gpmpc_set_error("gather: counts / root differ from those gpmpc_gather_prepare was called with");
    return -2;  // (the prepared block stays valid for a call with the right arguments)
  }
  c->prepared = false;
  if (p.cmax == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const size_t blk = (size_t)p.cmax * GPMPC_REC_LEN;
  GPMPC_RCCL(rccl().gather(c->send.p, c->rank == root ? c->recv.p : c->send.p, blk, ncclFloat64, root, c->comm, s));
  if (c->rank == root) {
    // compact: rank r's rows [0, counts[r]) in rank order
    size_t off = 0;
    for (int r = 0; r < c->nranks; ++r) {
      if (counts[r])
        GPMPC_HIP(hipMemcpyAsync(out + off, c->recv.as<double>() + (size_t)r * blk,
                                 sizeof(double) * (size_t)counts[r] * GPMPC_REC_LEN, hipMemcpyDeviceToHost, s));
      off += (size_t)counts[r] * GPMPC_REC_LEN;
    }
  }
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}

// both steps in one call, for a caller that does not need the agreement in between
extern "C" int gpmpc_gather_results(gpmpc_ctx *ctx, gpmpc_comm *c, const double *d_records, const int *counts,
                                    int root, double *out) {
  if (int rc = gpmpc_gather_prepare(ctx, c, d_records, counts, root)) return rc;
  return gpmpc_gather_collective(ctx, c, counts, root, out);
}
