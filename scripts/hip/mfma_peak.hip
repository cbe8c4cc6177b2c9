// FP64 MFMA issue-rate probe: v_mfma_f64_16x16x4f64 from registers only (no memory in the
// loop), NACC independent accumulators per wave, W waves per workgroup, G workgroups.
//   hipcc --offload-arch=gfx950 -O3 scripts/hip/mfma_peak.hip -o /tmp/mfma_peak && /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4_t __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k_peak(int iters, double *out) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + lane * 1e-3, b = 1.0 - lane * 1e-3;
  d4_t acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (d4_t){0.0, 0.0, 0.0, 0.0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
void run(int wgs, int threads, int iters) {
  double *out;
  hipMalloc(&out, sizeof(double) * wgs * threads);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_peak<NACC>, dim3(wgs), dim3(threads), 0, 0, iters, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_peak<NACC>, dim3(wgs), dim3(threads), 0, 0, iters, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double fl = 2048.0 * NACC * (double)iters * (wgs * threads / 64);
  printf("nacc %2d wgs %4d threads %3d: %.3f ms  %.2f TF  %.3f of 78.6\n", NACC, wgs, threads, ms, fl / ms / 1e9,
         fl / ms / 1e9 / 78.6);
  hipFree(out);
}
int main() {
  run<16>(256, 256, 4000);   // 1 wave / SIMD
  run<16>(512, 256, 4000);   // 2 waves / SIMD
  run<16>(1024, 256, 4000);  // 4 waves / SIMD
  run<4>(512, 256, 16000);
  run<8>(512, 256, 8000);
  return 0;
}
