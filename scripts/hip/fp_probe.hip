// fp_probe.hip -- standalone timing / correctness probe of the wide control build's KKT
// solvers (csrc/fleet_part.h partitioned, csrc/fleet_twist.h twisted) on a random SPD
// block-tridiagonal matrix of the fleet's shape (21 blocks of 10, coupling through the
// first 7 rows, the last block padded to identity).  One workgroup of 256 threads, each
// wave's lane 0 stamps s_memtime around every phase.  Prints per-phase cycles per solve
// and the solution's error against a host Gaussian elimination.
//   hipcc -O3 --offload-arch=gfx950 -I gp_mpc_rocket_landing_amd/csrc scripts/hip/fp_probe.hip -o /tmp/fp_probe
#define FQ_T 256
#define FQ_WPE 1
#define FQ_PART 1
#include <hip/hip_runtime.h>
__device__ unsigned long long g_fpm[8];
#define FP_MARK(k) { if ((threadIdx.x & 63) == 0) g_fpm[k] = __builtin_amdgcn_s_memtime(); }
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "internal.h"
#include "qp.h"
#include "fleet_qp.h"

#define NSTAMP 16
#define REPS 64

template <bool PART>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_probe(
    const double *band, const double *rhs, double *x, unsigned long long *st, int *fail) {
  __shared__ FleetSmem s;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  for (int e = tid; e < FQ_FAC; e += 256) s.band_store[e] = band[e];
  for (int e = tid; e < FQ_NMAX; e += 256) s.rhs[e] = 0.0;
  __syncthreads();
  unsigned long long t[NSTAMP] = {};
  auto mark = [&](int k, unsigned long long &last) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    t[k] += now - last;
    last = now;
  };
  unsigned long long last = __builtin_amdgcn_s_memtime();
  int f;
  if (PART) f = fp_factor(s, 0);
  else f = ft_factor(s, 0);
  if (wv == 0 && lane == 0) *fail = f;
  __syncthreads();
  double vsp[17], xc = 0.0;
  if (PART) fp_load_spikes(s, tid, vsp);
  mark(0, last);
  for (int r = 0; r < REPS; ++r) {
    for (int e = tid; e < 210; e += 256) {
      s.rhs[e] = rhs[e];
#if FQ_PART
      s.brhs[e] = rhs[e];
#endif
    }
    __syncthreads();
    mark(1, last);
    if (PART) {
      fp_solve<1>(s, s.rhs, 0); mark(2, last); lds_sync(); mark(3, last);
      fp_solve<2>(s, s.rhs, 0); mark(4, last); lds_sync(); mark(5, last);
      fp_solve<4>(s, s.rhs, 0); mark(6, last); lds_sync(); mark(7, last);
      xc = s.rhs[tid < 210 ? tid : 0] - fp_corr(s, fp_seg(tid / 10), vsp); mark(8, last);
    } else {
      ft_solve<1>(s, s.rhs, 0); mark(2, last); lds_sync(); mark(3, last);
      ft_solve<2>(s, s.rhs, 0); mark(4, last); lds_sync(); mark(5, last);
      ft_solve<4>(s, s.rhs, 0); mark(6, last);
    }
    __syncthreads();
    mark(9, last);
  }
  if (PART) { if (tid < 210) x[tid] = xc; }
  else for (int e = tid; e < 210; e += 256) x[e] = s.rhs[e];
  if (lane == 0)
    for (int k = 0; k < NSTAMP; ++k) st[wv * NSTAMP + k] = t[k];
}

int main() {
  const int SZ = 10, CM = 7, NB = 21, BS = SZ * SZ + SZ * CM, n = NB * SZ;
  srand(7);
  auto rnd = [] { return 2.0 * rand() / RAND_MAX - 1.0; };
  std::vector<double> M(n * n, 0.0), band(FQ_FAC, 0.0), b(n);
  for (int k = 0; k < NB; ++k) {
    double A[SZ][SZ];
    for (int i = 0; i < SZ; ++i)
      for (int j = 0; j < SZ; ++j) A[i][j] = rnd();
    for (int i = 0; i < SZ; ++i)
      for (int j = 0; j < SZ; ++j) {
        double v = (i == j) ? 12.0 : 0.0;
        for (int l = 0; l < SZ; ++l) v += A[i][l] * A[j][l];
        M[(k * SZ + i) * n + k * SZ + j] = v;
      }
    if (k + 1 < NB)
      for (int i = 0; i < CM; ++i)
        for (int j = 0; j < SZ; ++j) {
          const double v = rnd();
          M[((k + 1) * SZ + i) * n + k * SZ + j] = v;
          M[(k * SZ + j) * n + (k + 1) * SZ + i] = v;
        }
  }
  for (int j = 207; j < 210; ++j) {
    for (int i = 0; i < n; ++i) M[j * n + i] = M[i * n + j] = 0.0;
    M[j * n + j] = 1.0;
  }
  for (int k = 0; k < NB; ++k) {
    for (int i = 0; i < SZ; ++i)
      for (int j = 0; j < SZ; ++j) band[k * BS + j * SZ + i] = M[(k * SZ + i) * n + k * SZ + j];
    if (k + 1 < NB)
      for (int i = 0; i < CM; ++i)
        for (int j = 0; j < SZ; ++j) band[k * BS + SZ * SZ + j * CM + i] = M[((k + 1) * SZ + i) * n + k * SZ + j];
  }
  for (int i = 0; i < n; ++i) b[i] = i < 207 ? rnd() : 0.0;
  // host reference: Gaussian elimination
  std::vector<double> A2(M), x2(b);
  for (int p = 0; p < n; ++p)
    for (int i = p + 1; i < n; ++i) {
      const double f = A2[i * n + p] / A2[p * n + p];
      if (f == 0.0) continue;
      for (int j = p; j < n; ++j) A2[i * n + j] -= f * A2[p * n + j];
      x2[i] -= f * x2[p];
    }
  for (int i = n - 1; i >= 0; --i) {
    double v = x2[i];
    for (int j = i + 1; j < n; ++j) v -= A2[i * n + j] * x2[j];
    x2[i] = v / A2[i * n + i];
  }
  double *dband, *db, *dx;
  unsigned long long *dst;
  int *dfail;
  hipMalloc(&dband, sizeof(double) * FQ_FAC);
  hipMalloc(&db, sizeof(double) * n);
  hipMalloc(&dx, sizeof(double) * n);
  hipMalloc(&dst, sizeof(unsigned long long) * 4 * NSTAMP);
  hipMalloc(&dfail, sizeof(int));
  hipMemcpy(dband, band.data(), sizeof(double) * FQ_FAC, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), sizeof(double) * n, hipMemcpyHostToDevice);
  const char *names[] = {"factor", "rhs+sync", "ph1", "sync1", "ph2", "sync2", "ph4", "sync4", "ph8", "sync8",
                         "fwd", "bwd", "bhat", "xs"};
  for (int part = 0; part < 2; ++part) {
    for (int rep = 0; rep < 3; ++rep) {
      if (part) hipLaunchKernelGGL(k_probe<true>, dim3(1), dim3(256), 0, 0, dband, db, dx, dst, dfail);
      else hipLaunchKernelGGL(k_probe<false>, dim3(1), dim3(256), 0, 0, dband, db, dx, dst, dfail);
    }
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    std::vector<unsigned long long> st(4 * NSTAMP);
    std::vector<double> x(n);
    int fail = 0;
    hipMemcpy(st.data(), dst, sizeof(unsigned long long) * 4 * NSTAMP, hipMemcpyDeviceToHost);
    hipMemcpy(x.data(), dx, sizeof(double) * n, hipMemcpyDeviceToHost);
    hipMemcpy(&fail, dfail, sizeof(int), hipMemcpyDeviceToHost);
    if (part) {
      unsigned long long fpm[8];
      hipMemcpyFromSymbol(fpm, HIP_SYMBOL(g_fpm), sizeof(fpm));
      const char *fn[] = {"segfactor", "startspike", "endspike", "shat", "gj"};
      printf("  factor sections:");
      for (int k = 0; k < 5; ++k) printf(" %s %llu", fn[k], fpm[k + 1] - fpm[k]);
      printf("\n");
    }
    double err = 0.0, nx = 0.0;
    for (int i = 0; i < 207; ++i) { err = fmax(err, fabs(x[i] - x2[i])); nx = fmax(nx, fabs(x2[i])); }
    printf("%s: factor code %d, max |x - x_ref| %.3e (max |x_ref| %.3e)\n", part ? "partitioned" : "twisted", fail,
           err, nx);
    for (int w = 0; w < 4; ++w) {
      printf("  wave %d:", w);
      for (int k = 0; k < 14; ++k)
        printf(" %s %.0f", names[k], k == 0 ? (double)st[w * NSTAMP] : (double)st[w * NSTAMP + k] / REPS);
      printf("\n");
    }
  }
  return 0;
}
