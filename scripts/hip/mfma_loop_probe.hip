// What the 128-tile loop's non-MFMA parts cost: 64 v_mfma_f64_16x16x4f64 per step and wave
// (16 accumulators x 4 substeps), 256-thread workgroups, two per CU, with
//   BAR: one __syncthreads per step;  LDS: the step's 16 ds_read_b128 operand reads;
//   DMA: 8 global_load_lds_dwordx4 per wave and step, vmcnt(0) before the barrier.
//   hipcc --offload-arch=gfx950 -O3 scripts/hip/mfma_loop_probe.hip -o scripts/mfma_loop_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef double d4_t __attribute__((ext_vector_type(4)));
#define MF(acc, a, b) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
template <bool BAR, bool LDS, bool DMA, int AHEAD = 1>
__global__ __launch_bounds__(256, 2) void k_loop(int steps, const double *src, double *out) {
  __shared__ __attribute__((aligned(16))) double S[4 * 2048];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 4 * 2048; i += 256) S[i] = 1.0 + 1e-3 * (i & 63);
  __syncthreads();
  d4_t acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = (d4_t){0.0, 0.0, 0.0, 0.0};
  double2 fa[8], fb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[i] = fb[i] = make_double2(1.0 + lane * 1e-3, 1.0 - lane * 1e-3);
  int cur = 0;
  for (int s = 0; s < steps; ++s) {
    if (DMA) {
      const double *g = src + ((int64_t)(blockIdx.x * 4 + wave) * 8 * 128 + s % 64 * 8192) % (1 << 22) + 2 * lane;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t l = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)(S + (cur ^ 1) * 4096 + (4 * wave + (j & 3)) * 128 + (j >> 2) * 2048);
        int keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g + j * 128), "s"(__builtin_amdgcn_readfirstlane(l)) : "memory");
      }
    }
    if (LDS) {
      const double *L = S + cur * 4096 + (lane & 15) * 16 + 2 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        fa[i] = *(const double2 *)(L + (i & 3) * 256 + (i >> 2) * 4);
        fb[i] = *(const double2 *)(L + 2048 + (i & 3) * 256 + (i >> 2) * 4);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const double a = (q & 1) ? fa[4 * (q >> 1) + x].y : fa[4 * (q >> 1) + x].x;
          const double b = (q & 1) ? fb[4 * (q >> 1) + y].y : fb[4 * (q >> 1) + y].x;
          MF(acc[4 * x + y], a, b);
        }
    __builtin_amdgcn_sched_barrier(0);
    if (DMA && AHEAD == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (DMA && AHEAD == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    if (BAR) __syncthreads();
    cur ^= 1;
  }
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < 16; ++i) t += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + tid] = t;
}
template <bool BAR, bool LDS, bool DMA, int AHEAD = 1>
void run(const char *name, const double *src, double *out) {
  const int wgs = 512, steps = 2000;
  hipLaunchKernelGGL((k_loop<BAR, LDS, DMA, AHEAD>), dim3(wgs), dim3(256), 0, 0, steps, src, out);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_loop<BAR, LDS, DMA, AHEAD>), dim3(wgs), dim3(256), 0, 0, steps, src, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double fl = 2048.0 * 64 * steps * wgs * 4;
  printf("%-18s %.3f ms  %.2f TF  %.3f of 78.6\n", name, ms, fl / ms / 1e9, fl / ms / 1e9 / 78.6);
}
int main() {
  double *src, *out;
  hipMalloc(&src, sizeof(double) * ((1 << 22) + 8192));
  hipMemset(src, 0, sizeof(double) * ((1 << 22) + 8192));
  hipMalloc(&out, sizeof(double) * 512 * 256);
  run<false, false, false>("mfma", src, out);
  run<true, false, false>("mfma+bar", src, out);
  run<false, true, false>("mfma+lds", src, out);
  run<true, true, false>("mfma+lds+bar", src, out);
  run<true, true, true>("mfma+lds+bar+dma", src, out);
  run<true, false, true>("mfma+bar+dma", src, out);
  run<true, true, true, 2>("...+dma 2 ahead", src, out);
  run<true, false, true, 2>("bar+dma 2 ahead", src, out);
  return 0;
}
