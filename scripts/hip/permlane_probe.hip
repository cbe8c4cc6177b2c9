// semantics of __builtin_amdgcn_permlane16_swap on gfx950 (prints lane -> source lane)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o) {
  const unsigned a = threadIdx.x, b = 100 + threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  o[threadIdx.x] = r[0];
  o[64 + threadIdx.x] = r[1];
}
int main() {
  unsigned *d, h[128];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int r = 0; r < 2; ++r) {
    printf("r[%d]:", r);
    for (int i = 0; i < 64; ++i) printf(" %u", h[r * 64 + i]);
    printf("\n");
  }
  return 0;
}
