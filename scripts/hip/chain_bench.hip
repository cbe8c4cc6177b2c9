// micro-benchmark: one KKT chain step of the 6-DoF control kernel in isolation
// (16 DPP FMAs with their operand rows reloaded from LDS a step ahead, one
// store), to split its ~400 cycles into FMA issue and LDS cost.
//   mode 0: operands in registers only (no LDS)
//   mode 1: one ds_read_b64 per operand, each right after its FMA (the kernel's form)
//   mode 2: operand pairs as one 16-byte read after every second FMA
#include <hip/hip_runtime.h>
#include <cstdio>

template <int J>
__device__ __forceinline__ void fbc(double &acc, double src, double mul) {
  if (J == 0)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "i"(J));
  else
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "i"(J));
}

// the sum of this lane's value and its partner's in the other row of the row pair
// (rows 0/1, 2/3): v_permlane16_swap on both halves, then one add; both rows get
// the same bits (the add is commutative)
__device__ __forceinline__ double pair_sum(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}
// odd rows rotated by 8 lanes (DPP row_ror:8 on both halves, rows 1 and 3 only)
__device__ __forceinline__ double ror8_odd(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int l = __builtin_amdgcn_update_dpp(lo, lo, 0x128, 0xa, 0xf, false);
  const int h = __builtin_amdgcn_update_dpp(hi, hi, 0x128, 0xa, 0xf, false);
  return __hiloint2double(h, l);
}

#define STEPS 15
template <int MODE>
__global__ __launch_bounds__(512) void k(double *out, long long *cyc, int reps, int nw) {
  __shared__ double F[STEPS + 2][16][18];
  __shared__ double Y[STEPS + 2][16];
  __shared__ double dump[64];
  const int tid = threadIdx.x, lane = tid & 63, rr = lane & 15, wv = tid >> 6;
  for (int i = tid; i < (STEPS + 2) * 16 * 18; i += blockDim.x) (&F[0][0][0])[i] = 1e-3 * (i % 97);
  for (int i = tid; i < (STEPS + 2) * 16; i += blockDim.x) (&Y[0][0])[i] = 1e-2 * i;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  double y = 0.0;
  for (int r = 0; r < reps; ++r) {
    if (wv < nw) {
      double g[16];
      const double *f = &F[0][rr][0];
#pragma unroll
      for (int j = 0; j < 16; ++j) g[j] = f[j];
      y = Y[0][rr];
#pragma unroll 3
      for (int t = 0; t < STEPS; ++t) {
        const double *fn = &F[t + 1][rr][0];
        double a0 = Y[t + 1][rr], a1 = 0.0;
        if (MODE == 0) {
          fbc<0>(a0, y, g[0]); fbc<1>(a1, y, g[1]); fbc<2>(a0, y, g[2]); fbc<3>(a1, y, g[3]);
          fbc<4>(a0, y, g[4]); fbc<5>(a1, y, g[5]); fbc<6>(a0, y, g[6]); fbc<7>(a1, y, g[7]);
          fbc<8>(a0, y, g[8]); fbc<9>(a1, y, g[9]); fbc<10>(a0, y, g[10]); fbc<11>(a1, y, g[11]);
          fbc<12>(a0, y, g[12]); fbc<13>(a1, y, g[13]); fbc<14>(a0, y, g[14]); fbc<15>(a1, y, g[15]);
        } else if (MODE == 1) {
          fbc<0>(a0, y, g[0]); g[0] = fn[0]; fbc<1>(a1, y, g[1]); g[1] = fn[1];
          fbc<2>(a0, y, g[2]); g[2] = fn[2]; fbc<3>(a1, y, g[3]); g[3] = fn[3];
          fbc<4>(a0, y, g[4]); g[4] = fn[4]; fbc<5>(a1, y, g[5]); g[5] = fn[5];
          fbc<6>(a0, y, g[6]); g[6] = fn[6]; fbc<7>(a1, y, g[7]); g[7] = fn[7];
          fbc<8>(a0, y, g[8]); g[8] = fn[8]; fbc<9>(a1, y, g[9]); g[9] = fn[9];
          fbc<10>(a0, y, g[10]); g[10] = fn[10]; fbc<11>(a1, y, g[11]); g[11] = fn[11];
          fbc<12>(a0, y, g[12]); g[12] = fn[12]; fbc<13>(a1, y, g[13]); g[13] = fn[13];
          fbc<14>(a0, y, g[14]); g[14] = fn[14]; fbc<15>(a1, y, g[15]); g[15] = fn[15];
        } else if (MODE == 3) {
          // two rows: row 0 terms 0..7, row 1 terms 8..15 (its vector rotated by 8),
          // operands in 16-byte pairs, then the pair sum and the odd rows' rotation
          const double2 *f2 = reinterpret_cast<const double2 *>(fn + ((lane & 16) ? 8 : 0));
          double2 p;
          if (lane & 16) a0 = 0.0;
          fbc<0>(a0, y, g[0]); fbc<1>(a1, y, g[1]); p = f2[0]; g[0] = p.x; g[1] = p.y;
          fbc<2>(a0, y, g[2]); fbc<3>(a1, y, g[3]); p = f2[1]; g[2] = p.x; g[3] = p.y;
          fbc<4>(a0, y, g[4]); fbc<5>(a1, y, g[5]); p = f2[2]; g[4] = p.x; g[5] = p.y;
          fbc<6>(a0, y, g[6]); fbc<7>(a1, y, g[7]); p = f2[3]; g[6] = p.x; g[7] = p.y;
          y = ror8_odd(pair_sum(a0 + a1));
          *(lane < 14 ? &Y[t + 1][rr] : &dump[lane]) = y;
          continue;
        } else {
          const double2 *f2 = reinterpret_cast<const double2 *>(fn);
          double2 p;
          fbc<0>(a0, y, g[0]); fbc<1>(a1, y, g[1]); p = f2[0]; g[0] = p.x; g[1] = p.y;
          fbc<2>(a0, y, g[2]); fbc<3>(a1, y, g[3]); p = f2[1]; g[2] = p.x; g[3] = p.y;
          fbc<4>(a0, y, g[4]); fbc<5>(a1, y, g[5]); p = f2[2]; g[4] = p.x; g[5] = p.y;
          fbc<6>(a0, y, g[6]); fbc<7>(a1, y, g[7]); p = f2[3]; g[6] = p.x; g[7] = p.y;
          fbc<8>(a0, y, g[8]); fbc<9>(a1, y, g[9]); p = f2[4]; g[8] = p.x; g[9] = p.y;
          fbc<10>(a0, y, g[10]); fbc<11>(a1, y, g[11]); p = f2[5]; g[10] = p.x; g[11] = p.y;
          fbc<12>(a0, y, g[12]); fbc<13>(a1, y, g[13]); p = f2[6]; g[12] = p.x; g[13] = p.y;
          fbc<14>(a0, y, g[14]); fbc<15>(a1, y, g[15]); p = f2[7]; g[14] = p.x; g[15] = p.y;
        }
        y = a0 + a1;
        *(lane < 14 ? &Y[t + 1][rr] : &dump[lane]) = y;
      }
    }
    __syncthreads();
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + tid] = y;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double *out; long long *cyc;
  hipMalloc(&out, sizeof(double) * 512);
  hipMalloc(&cyc, sizeof(long long));
  const int reps = 200;
  const char *nm[4] = {"registers", "b64 each", "b128 pairs", "two rows"};
  for (int nw = 1; nw <= 2; ++nw)
    for (int m = 0; m < 4; ++m) {
      if (m == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(512), 0, 0, out, cyc, reps, nw);
      if (m == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(512), 0, 0, out, cyc, reps, nw);
      if (m == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(512), 0, 0, out, cyc, reps, nw);
      if (m == 3) hipLaunchKernelGGL(k<3>, dim3(1), dim3(512), 0, 0, out, cyc, reps, nw);
      long long h = 0;
      hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      printf("%d chain wave(s), %-11s %8.1f ticks per step (incl. the per-pass barrier)\n", nw, nm[m],
             (double)h / (reps * STEPS));
    }
  return 0;
}
