// qp.hip -- batched OSQP-style ADMM: one workgroup (256 threads) per QP.
//
// Replaces the osqp.OSQP() setup / update(q) / update(l, u, Ax) / warm_start(x)
// / solve() sequence of OSQPRTIMPC (osqp_rti.py:454-567) for a whole batch of
// QPs that share one sparsity pattern.  The pattern is pre-processed once on
// the host (CSR -> CSC map, banded-KKT product terms) and shared by every
// workgroup; the numeric data of each problem is staged into LDS.
#include "internal.h"
#include "qp.h"
#include <algorithm>
#include <cstdlib>
#include <vector>

extern "C" void gpmpc_qp_default_settings(gpmpc_qp_settings *s) {
  // osqp_rti.py:54-60 (max_iter 50, eps 1e-4, polish off, warm start, scaling 3)
  // + OSQP 0.6 defaults pinned, adaptive-rho interval fixed at 25.
  s->rho = 0.1;
  s->sigma = 1e-6;
  s->alpha = 1.6;
  s->eps_abs = 1e-4;
  s->eps_rel = 1e-4;
  s->eps_prim_inf = 1e-4;
  s->eps_dual_inf = 1e-4;
  s->max_iter = 50;
  s->check_termination = 25;
  s->adaptive_rho = 1;
  s->adaptive_rho_interval = 25;
  s->adaptive_rho_tolerance = 5.0;
  s->scaling = 3;
  s->warm_start = 1;
}

QPSettingsDev to_dev(const gpmpc_qp_settings &s) {
  QPSettingsDev d;
  d.rho = s.rho; d.sigma = s.sigma; d.alpha = s.alpha; d.eps_abs = s.eps_abs;
  d.eps_rel = s.eps_rel; d.eps_prim_inf = s.eps_prim_inf; d.eps_dual_inf = s.eps_dual_inf;
  d.max_iter = s.max_iter; d.check_termination = s.check_termination;
  d.adaptive_rho = s.adaptive_rho; d.adaptive_rho_interval = s.adaptive_rho_interval;
  d.adaptive_rho_tolerance = s.adaptive_rho_tolerance; d.scaling = s.scaling;
  d.warm_start = s.warm_start;
  return d;
}

int QPPatternHost::build(int n_, int m_, const int *rowptr, const int *colidx, hipStream_t s) {
  n = n_;
  m = m_;
  nnz = rowptr[m];
  w = 0;
  for (int r = 0; r < m; ++r)
    for (int a = rowptr[r]; a < rowptr[r + 1]; ++a)
      for (int b = rowptr[r]; b < rowptr[r + 1]; ++b) w = std::max(w, colidx[a] - colidx[b]);
  const int nb = w + 1;
  maxrow = 0;
  for (int r = 0; r < m; ++r) maxrow = std::max(maxrow, rowptr[r + 1] - rowptr[r]);
  // CSC map
  std::vector<int> colptr(n + 1, 0), csc2csr(nnz), cscrow(nnz);
  for (int k = 0; k < nnz; ++k) colptr[colidx[k] + 1]++;
  for (int j = 0; j < n; ++j) colptr[j + 1] += colptr[j];
  maxcol = 0;
  for (int j = 0; j < n; ++j) maxcol = std::max(maxcol, colptr[j + 1] - colptr[j]);
  std::vector<int> fill(colptr.begin(), colptr.end() - 1);
  for (int r = 0; r < m; ++r)
    for (int k = rowptr[r]; k < rowptr[r + 1]; ++k) {
      const int p = fill[colidx[k]]++;
      csc2csr[p] = k;
      cscrow[p] = r;
    }
  // Factor layout.  Mode 1 (block tridiagonal, qp_block.h) when every coupled
  // pair (i >= j) of M = P + A'RA lies in one block of QP_BLK_SZ variables or
  // in neighbouring blocks with i among the first QP_BLK_CM rows of its block
  // (the MPC stage structure); otherwise mode 0, the banded LDL^T with column
  // stride QP_W+1.  Either way every LDS slot gets its list of rho_r A[a] A[b]
  // terms, generated in (row, a, b) order like the C oracle's factor().
  constexpr int NB = QP_W + 1, SZ = QP_BLK_SZ, CM = QP_BLK_CM, BS = SZ * SZ + SZ * CM;
  nblk = (n + SZ - 1) / SZ;
  bool blk = true;
  for (int r = 0; r < m && blk; ++r)
    for (int a = rowptr[r]; a < rowptr[r + 1]; ++a)
      for (int b = rowptr[r]; b < rowptr[r + 1]; ++b) {
        const int i = colidx[a], j = colidx[b];
        if (j > i) continue;
        const int bi = i / SZ, bj = j / SZ;
        if (!(bi == bj || (bi == bj + 1 && i - bi * SZ < CM))) blk = false;
      }
  if (blk && nblk * BS - SZ * CM > QP_FAC_CAP) blk = false;
  mode = blk ? 1 : 0;
  fac_len = blk ? nblk * BS - SZ * CM : n * NB;
  struct T { int e, r, a, b; };
  std::vector<T> terms;
  std::vector<int> facdiag(fac_len, -1);
  for (int r = 0; r < m; ++r)
    for (int a = rowptr[r]; a < rowptr[r + 1]; ++a)
      for (int b = rowptr[r]; b < rowptr[r + 1]; ++b) {
        const int i = colidx[a], j = colidx[b];
        if (j > i) continue;
        if (!blk) {
          terms.push_back(T{j * NB + (i - j), r, a, b});
          continue;
        }
        const int bi = i / SZ, bj = j / SZ, ri = i - bi * SZ, rj = j - bj * SZ;
        if (bi == bj) {
          terms.push_back(T{bi * BS + rj * SZ + ri, r, a, b});
          if (i != j) terms.push_back(T{bi * BS + ri * SZ + rj, r, a, b});
        } else {
          terms.push_back(T{bj * BS + SZ * SZ + rj * CM + ri, r, a, b});
        }
      }
  if (blk) {
    for (int v = 0; v < nblk * SZ; ++v) {
      const int k = v / SZ, rv = v - k * SZ;
      facdiag[k * BS + rv * SZ + rv] = (v < n) ? v : -2;  // identity rows pad the last block
    }
  } else {
    for (int j = 0; j < n; ++j) facdiag[j * NB] = j;
  }
  std::stable_sort(terms.begin(), terms.end(), [](const T &x, const T &y) { return x.e < y.e; });
  std::vector<int> facptr(fac_len + 1, 0), tv(3 * terms.size());
  for (size_t k = 0; k < terms.size(); ++k) {
    facptr[terms[k].e + 1]++;
    tv[3 * k] = terms[k].r;
    tv[3 * k + 1] = terms[k].a;
    tv[3 * k + 2] = terms[k].b;
  }
  for (int e = 0; e < fac_len; ++e) facptr[e + 1] += facptr[e];
  // mode 1: the non-diagonal slots that are not plain zeros, one int4 each
  // (QPPattern::offd), so the fleet's assembly reads one coalesced item per
  // slot instead of walking facdiag / facptr / terms for every slot
  std::vector<int> offd;
  int n_offd = -1;
  if (blk && fac_len < (1 << 15) && nnz < (1 << 16)) {
    n_offd = 0;
    for (int e = 0; e < fac_len && n_offd >= 0; ++e) {
      if (facdiag[e] >= 0) continue;
      const int k0 = facptr[e], k1 = facptr[e + 1], one = facdiag[e] == -2;
      if (k1 == k0 && !one) continue;
      if (k1 - k0 > 3) { n_offd = -1; break; }
      int it[4] = {e | (one << 15) | ((k1 - k0) << 16), 0, 0, 0};
      for (int k = k0; k < k1; ++k) it[1 + k - k0] = tv[3 * k + 1] | (tv[3 * k + 2] << 16);
      offd.insert(offd.end(), it, it + 4);
      ++n_offd;
    }
  }
  if (n_offd < 0) offd.clear();
  // one device block: rowptr | colidx | colptr | csc2csr | cscrow | facptr | facdiag | terms | offd
  std::vector<int> all;
  auto app = [&](const int *p, size_t k) { all.insert(all.end(), p, p + k); };
  const size_t o_rp = 0;
  app(rowptr, m + 1);
  const size_t o_ci = all.size();
  app(colidx, nnz);
  const size_t o_cp = all.size();
  app(colptr.data(), n + 1);
  const size_t o_cm = all.size();
  app(csc2csr.data(), nnz);
  const size_t o_cr = all.size();
  app(cscrow.data(), nnz);
  const size_t o_bp = all.size();
  app(facptr.data(), facptr.size());
  const size_t o_fd = all.size();
  app(facdiag.data(), facdiag.size());
  const size_t o_tv = all.size();
  app(tv.data(), tv.size());
  while (all.size() % 4) all.push_back(0);  // int4 alignment (the buffer itself is 256-B aligned)
  const size_t o_od = all.size();
  app(offd.data(), offd.size());
  if (buf.alloc(sizeof(int) * all.size()) != hipSuccess) return -1;
  if (hipMemcpyAsync(buf.p, all.data(), sizeof(int) * all.size(), hipMemcpyHostToDevice, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return -1;
  const int *d = buf.as<int>();
  dev.n = n; dev.m = m; dev.nnz = nnz; dev.w = w;
  dev.rowptr = d + o_rp; dev.colidx = d + o_ci; dev.colptr = d + o_cp; dev.csc2csr = d + o_cm;
  dev.cscrow = d + o_cr; dev.facptr = d + o_bp; dev.facdiag = d + o_fd; dev.terms = d + o_tv;
  dev.mode = mode; dev.fac_len = fac_len; dev.nblk = nblk; dev.bsz = SZ; dev.bcm = CM;
  dev.offd = reinterpret_cast<const int4 *>(d + o_od);
  dev.n_offd = n_offd;
  return 0;
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_qp_batched(QPPattern pt, QPSettingsDev st,
                                                    const double *__restrict__ Aval,
                                                    const double *__restrict__ Pd,
                                                    const double *__restrict__ q,
                                                    const double *__restrict__ l,
                                                    const double *__restrict__ u,
                                                    const double *__restrict__ xws, double *rho,
                                                    double *yst, double *xo, double *yo,
                                                    int *iters, int *status, double *obj,
                                                    unsigned long long *stamps) {
  __shared__ QPSmemStd s;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int n = pt.n, m = pt.m, nnz = pt.nnz;
  for (int k = tid; k < nnz; k += nt) s.A[k] = Aval[(int64_t)b * nnz + k];
  for (int j = tid; j < n; j += nt) {
    s.P[j] = Pd[(int64_t)b * n + j];
    s.q[j] = q[(int64_t)b * n + j];
    s.x[j] = xws ? xws[(int64_t)b * n + j] : 0.0;
  }
  for (int r = tid; r < m; r += nt) {
    s.l[r] = l[(int64_t)b * m + r];
    s.u[r] = u[(int64_t)b * m + r];
    s.y[r] = yst[(int64_t)b * m + r];
  }
  if (tid == 0) s.rho_s = rho[b];
  __syncthreads();
  QPStamps T;
  if (b == 0) T.out = stamps;  // (GPMPC_QP_STAMPS: problem 0's phase cycles)
  T.start();
  QPResult res = qp_solve(pt, s, st, &T);
  T.mark(7);
  T.flush();
  if (res.factor_fail) {
    if (tid == 0) { status[b] = -100; iters[b] = 0; obj[b] = nan(""); }
    return;
  }
  const bool has = (res.status == 1 || res.status == 2 || res.status == -2);
  for (int j = tid; j < n; j += nt) xo[(int64_t)b * n + j] = has ? s.D[j] * s.x[j] : nan("");
  for (int r = tid; r < m; r += nt) {
    yo[(int64_t)b * m + r] = has ? s.E[r] * s.y[r] / s.c : nan("");
    yst[(int64_t)b * m + r] = s.y[r];
  }
  if (tid == 0) {
    rho[b] = s.rho_s;
    iters[b] = res.iter;
    status[b] = res.status;
    obj[b] = has ? res.obj : nan("");
  }
}

hipError_t launch_qp_batched(hipStream_t s, const QPPattern &pt, const QPSettingsDev &st,
                             int batch, const double *Aval, const double *Pd, const double *q,
                             const double *l, const double *u, const double *xws, double *rho,
                             double *yst, double *xo, double *yo, int *iters, int *status,
                             double *obj, unsigned long long *stamps = nullptr) {
  hipLaunchKernelGGL(k_qp_batched, dim3(batch), dim3(256), 0, s, pt, st, Aval, Pd, q, l, u, xws,
                     rho, yst, xo, yo, iters, status, obj, stamps);
  return hipGetLastError();
}

// The last pattern of each stream, kept: a caller that re-solves one pattern (the OSQP
// workspace, QPWorkspace.solve, once per control step) pays its host pre-processing,
// upload and the upload's synchronisation once instead of per solve.
#include <map>
#include <memory>
#include <mutex>
struct QPPatCache {
  std::vector<int> rowptr, colidx;
  int n = 0;
  std::unique_ptr<QPPatternHost> pat;
};
static std::mutex g_qpcache_mu;
static std::map<hipStream_t, QPPatCache> g_qpcache;

void gpmpc_qp_cache_release(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_qpcache_mu);
  g_qpcache.erase(s);
}

static QPPatternHost *qp_pattern(hipStream_t s, int n, int m, const int *rowptr, const int *colidx) {
  std::lock_guard<std::mutex> lk(g_qpcache_mu);
  QPPatCache &c = g_qpcache[s];
  const int nnz = rowptr[m];
  if (c.pat && c.n == n && (int)c.rowptr.size() == m + 1 && (int)c.colidx.size() == nnz &&
      !memcmp(c.rowptr.data(), rowptr, sizeof(int) * (m + 1)) &&
      !memcmp(c.colidx.data(), colidx, sizeof(int) * nnz))
    return c.pat.get();
  c.pat.reset();
  auto pat = std::make_unique<QPPatternHost>();
  if (pat->build(n, m, rowptr, colidx, s)) return nullptr;
  c.rowptr.assign(rowptr, rowptr + m + 1);
  c.colidx.assign(colidx, colidx + nnz);
  c.n = n;
  c.pat = std::move(pat);
  return c.pat.get();
}

static int qp_cu_count(int dev) {
  static int cus[64] = {0};
  if (dev < 0 || dev >= 64) return 0;
  if (!cus[dev]) (void)hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev);
  return cus[dev];
}

extern "C" int gpmpc_qp_solve_batched(gpmpc_ctx *ctx, int batch, int n, int m, int nnz,
                                      const int *rowptr, const int *colidx, const double *Aval,
                                      const double *Pdiag, const double *q, const double *l,
                                      const double *u, const gpmpc_qp_settings *st,
                                      const double *x_ws, double *rho, double *y_scaled,
                                      double *x, double *y, int *iters, int *status,
                                      double *obj) {
  GPMPC_CHECK_ARG(ctx && rowptr && colidx && Aval && Pdiag && q && l && u && st && rho &&
                  y_scaled && x && y && iters && status && obj);
  GPMPC_CHECK_ARG(batch >= 0 && n > 0 && m > 0 && nnz == rowptr[m]);
  GPMPC_CHECK_ARG(n <= QP_NMAX && m <= QP_MMAX && nnz <= QP_NNZMAX);
  if (batch == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const QPPatternHost *pat = qp_pattern(s, n, m, rowptr, colidx);
  if (!pat) {
    gpmpc_set_error("qp: pattern upload failed");
    return -1;
  }
  if (!pat->fits()) {
    gpmpc_set_error("qp: pattern outside the compiled caps (n %d<=256, m %d<=512, half-bandwidth "
                    "%d<=%d, row nnz %d<=%d, col nnz %d<=%d)", pat->n, pat->m, pat->w, QP_W,
                    pat->maxrow, QP_RMAX, pat->maxcol, QP_CMAX);
    return -2;
  }
  // The fleet's solver (fleet_qp.h, registers + twisted KKT solve) for its own pattern -- the
  // 3-DoF MPC at N = 20 -- when the dynamics rows are equalities, as that solver assumes
  // (GPMPC_QP_FLEET=0: always the generic kernel).  The same OSQP iteration; the block-wide
  // sums and the KKT solve round differently from the generic kernel's.
  const char *fe = getenv("GPMPC_QP_FLEET");  // (read per call: tests switch it)
  const bool fleet_env = !fe || atoi(fe);
  bool fleet = fleet_env && qp_is_fleet_pattern(n, m, rowptr, colidx);
  for (int64_t r = 0; fleet && r < (int64_t)batch * m; ++r)
    if (r % m < QP_FLEET_MD && l[r] != u[r]) fleet = false;
  // every input in one pinned upload, every output in one read-back
  const size_t B = batch, dn = 8 * B * n, dm = 8 * B * m;
  const size_t bytes = Stage::pad(8 * B * nnz) + 2 * Stage::pad(dn) + 2 * Stage::pad(dm) +
                       (x_ws ? Stage::pad(dn) : 0) + Stage::pad(8 * B) + Stage::pad(dm) + Stage::pad(dn) +
                       Stage::pad(dm) + 2 * Stage::pad(4 * B) + Stage::pad(8 * B);
  Stage sg(s, bytes);
  if (!sg.ok()) {
    gpmpc_set_error("qp: staging buffers: out of memory");
    return -1;
  }
  const double *dA = sg.in(Aval, B * nnz), *dP = sg.in(Pdiag, B * n), *dq = sg.in(q, B * n);
  const double *dl = sg.in(l, B * m), *du = sg.in(u, B * m);
  const double *dx0 = x_ws ? sg.in(x_ws, B * n) : nullptr;
  double *drho = sg.inout(rho, B), *dy0 = sg.inout(y_scaled, B * m);
  double *dxo = sg.out(x, B * n), *dyo = sg.out(y, B * m);
  int *dit = sg.out(iters, B), *dst = sg.out(status, B);
  double *dob = sg.out(obj, B);
  GPMPC_HIP(sg.upload());
  // GPMPC_QP_STAMPS=1: problem 0's phase cycles (s_memtime) to stderr, a diagnostic
  static const bool stamp = getenv("GPMPC_QP_STAMPS") && atoi(getenv("GPMPC_QP_STAMPS"));
  DevBuf dts;
  if (stamp) {
    GPMPC_HIP(dts.alloc(s, 16 * sizeof(unsigned long long)));
    GPMPC_HIP(hipMemsetAsync(dts.p, 0, 16 * sizeof(unsigned long long), s));
  }
  if (fleet) {
    GPMPC_HIP((batch <= qp_cu_count(ctx->device) ? launch_qp_fleet_wide : launch_qp_fleet_narrow)(
        s, batch, pat->dev, to_dev(*st), dA, dP, dq, dl, du, dx0, drho, dy0, dxo, dyo, dit, dst, dob));
  } else {
    GPMPC_HIP(launch_qp_batched(s, pat->dev, to_dev(*st), batch, dA, dP, dq, dl, du, dx0, drho, dy0, dxo, dyo,
                                dit, dst, dob, dts.as<unsigned long long>()));
  }
  GPMPC_HIP(sg.download());
  if (stamp) {
    unsigned long long h[16];
    GPMPC_HIP(hipMemcpy(h, dts.p, sizeof(h), hipMemcpyDeviceToHost));
    fprintf(stderr, "qp_stamps iter %d:", iters[0]);
    for (int k = 0; k < 16; ++k) fprintf(stderr, " %llu", h[k]);
    fprintf(stderr, "\n");
  }
  return 0;
}
