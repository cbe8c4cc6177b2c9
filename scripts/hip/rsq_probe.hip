// Accuracy of v_rsq_f64 and of 0 / 1 / 2 Newton steps on it (the Cholesky
// pivot's 1/sqrt), in ulps of the correctly rounded host value.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/hip/rsq_probe.hip -o /tmp/rsq_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__global__ void k_rsq(const double *x, double *o0, double *o1, double *o2, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double p = x[i];
  double id = __builtin_amdgcn_rsq(p);
  o0[i] = id;
  id = id * fma(-0.5 * p * id, id, 1.5);
  o1[i] = id;
  id = id * fma(-0.5 * p * id, id, 1.5);
  o2[i] = id;
}

int main() {
  const int n = 1 << 20;
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(-6.0, 6.0);
  std::vector<double> x(n), r0(n), r1(n), r2(n);
  for (auto &v : x) v = std::pow(10.0, u(g));
  double *dx, *d0, *d1, *d2;
  hipMalloc(&dx, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d2, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_rsq, dim3(n / 256), dim3(256), 0, 0, dx, d0, d1, d2, n);
  hipMemcpy(r0.data(), d0, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r1.data(), d1, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r2.data(), d2, n * 8, hipMemcpyDeviceToHost);
  double m[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const long double ref = 1.0L / std::sqrt((long double)x[i]);
    const double refd = (double)ref;
    const double ulp = std::nextafter(refd, INFINITY) - refd;
    const double e[3] = {std::fabs((double)(r0[i] - ref)) / ulp, std::fabs((double)(r1[i] - ref)) / ulp,
                         std::fabs((double)(r2[i] - ref)) / ulp};
    for (int k = 0; k < 3; ++k) m[k] = std::max(m[k], e[k]);
  }
  printf("rsq max ulp: raw %.3g  newton1 %.3g  newton2 %.3g\n", m[0], m[1], m[2]);
  return 0;
}
