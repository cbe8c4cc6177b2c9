// micro-benchmark: cycles per FP64 chain step on one wave (DPP row_newbcast FMAs
// against plain FMAs, 2 and 4 accumulators) -- sizes the 6-DoF chain design
#include <hip/hip_runtime.h>
#include <cstdio>

template <int J>
__device__ __forceinline__ void fbc(double &acc, double src, double mul) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc) : "v"(src), "v"(mul), "i"(J));
}
__device__ __forceinline__ void fpl(double &acc, double src, double mul) {
  asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(acc) : "v"(src), "v"(mul));
}

template <int MODE>
__global__ void k(double *out, long long *cyc, int n) {
  double g[16];
  for (int j = 0; j < 16; ++j) g[j] = 1e-3 * (threadIdx.x + j);
  double y = threadIdx.x * 1e-2;
  asm volatile("s_nop 1");
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < n; ++it) {
    double a0 = y, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (MODE == 0) {  // DPP, 2 accumulators
      asm volatile("s_nop 1");
      fbc<0>(a0, y, g[0]); fbc<1>(a1, y, g[1]); fbc<2>(a0, y, g[2]); fbc<3>(a1, y, g[3]);
      fbc<4>(a0, y, g[4]); fbc<5>(a1, y, g[5]); fbc<6>(a0, y, g[6]); fbc<7>(a1, y, g[7]);
      fbc<8>(a0, y, g[8]); fbc<9>(a1, y, g[9]); fbc<10>(a0, y, g[10]); fbc<11>(a1, y, g[11]);
      fbc<12>(a0, y, g[12]); fbc<13>(a1, y, g[13]); fbc<14>(a0, y, g[14]); fbc<15>(a1, y, g[15]);
    } else if (MODE == 1) {  // plain, 2 accumulators
      fpl(a0, y, g[0]); fpl(a1, y, g[1]); fpl(a0, y, g[2]); fpl(a1, y, g[3]);
      fpl(a0, y, g[4]); fpl(a1, y, g[5]); fpl(a0, y, g[6]); fpl(a1, y, g[7]);
      fpl(a0, y, g[8]); fpl(a1, y, g[9]); fpl(a0, y, g[10]); fpl(a1, y, g[11]);
      fpl(a0, y, g[12]); fpl(a1, y, g[13]); fpl(a0, y, g[14]); fpl(a1, y, g[15]);
    } else if (MODE == 2) {  // DPP, 4 accumulators
      asm volatile("s_nop 1");
      fbc<0>(a0, y, g[0]); fbc<1>(a1, y, g[1]); fbc<2>(a2, y, g[2]); fbc<3>(a3, y, g[3]);
      fbc<4>(a0, y, g[4]); fbc<5>(a1, y, g[5]); fbc<6>(a2, y, g[6]); fbc<7>(a3, y, g[7]);
      fbc<8>(a0, y, g[8]); fbc<9>(a1, y, g[9]); fbc<10>(a2, y, g[10]); fbc<11>(a3, y, g[11]);
      fbc<12>(a0, y, g[12]); fbc<13>(a1, y, g[13]); fbc<14>(a2, y, g[14]); fbc<15>(a3, y, g[15]);
    } else if (MODE == 3) {  // DPP, 1 accumulator
      asm volatile("s_nop 1");
      fbc<0>(a0, y, g[0]); fbc<1>(a0, y, g[1]); fbc<2>(a0, y, g[2]); fbc<3>(a0, y, g[3]);
      fbc<4>(a0, y, g[4]); fbc<5>(a0, y, g[5]); fbc<6>(a0, y, g[6]); fbc<7>(a0, y, g[7]);
      fbc<8>(a0, y, g[8]); fbc<9>(a0, y, g[9]); fbc<10>(a0, y, g[10]); fbc<11>(a0, y, g[11]);
      fbc<12>(a0, y, g[12]); fbc<13>(a0, y, g[13]); fbc<14>(a0, y, g[14]); fbc<15>(a0, y, g[15]);
    } else {  // plain, 1 accumulator
      fpl(a0, y, g[0]); fpl(a0, y, g[1]); fpl(a0, y, g[2]); fpl(a0, y, g[3]);
      fpl(a0, y, g[4]); fpl(a0, y, g[5]); fpl(a0, y, g[6]); fpl(a0, y, g[7]);
      fpl(a0, y, g[8]); fpl(a0, y, g[9]); fpl(a0, y, g[10]); fpl(a0, y, g[11]);
      fpl(a0, y, g[12]); fpl(a0, y, g[13]); fpl(a0, y, g[14]); fpl(a0, y, g[15]);
    }
    y = (a0 + a1) + (a2 + a3);
    y *= 1e-3;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = y;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int n = 4096;
  double *out; long long *cyc;
  hipMalloc(&out, sizeof(double) * 64 * 8);
  hipMalloc(&cyc, sizeof(long long) * 8);
  const char *nm[5] = {"dpp 2acc", "plain 2acc", "dpp 4acc", "dpp 1acc", "plain 1acc"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 5; ++m) {
      switch (m) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
        default: hipLaunchKernelGGL(k<4>, dim3(1), dim3(64), 0, 0, out, cyc, n); break;
      }
      long long h = 0;
      hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      // s_memtime counts at the 100 MHz reference clock on CDNA: report both
      printf("%-11s %8.2f memtime ticks per step\n", nm[m], (double)h / n);
    }
  return 0;
}
