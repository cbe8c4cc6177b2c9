// uprop.hip -- batched linear covariance propagation along MPC horizons
// (reference src/mpc/uncertainty_prop.py:117-177, UncertaintyPropagator._propagate_linear):
//
//   Sigma_{k+1} = (A_k Sigma_k) A_k^T + diag(q_k),   k = 0 .. N-1
//
// q_k is the GP variance as process noise (var * dt^2 on the velocity block,
// and on the angular-rate block for 6-DoF), A_k the discrete Jacobian of the
// nominal step.  The mean recursion does not depend on Sigma, so the host
// (or the fleet) produces every A_k and q_k first and one launch runs all
// trajectories.  One workgroup per trajectory with one thread per entry of Sigma (n_x <=
// 16: 64 threads at n_x = 7, 256 at 14), so a step is two n_x-term dot products per
// thread and two barriers; the A_k and q_k of UP_CHUNK steps are staged into LDS in one
// cooperative load, off the step chain (one global round trip per chunk, not per step).
// HBM traffic per trajectory-step: read A_k (8 n_x^2 B) and q_k (8 n_x B), write
// Sigma_{k+1} (8 n_x^2 B).
#include "internal.h"

#define UP_NXMAX 16

#define UP_CHUNK 16

// NXC > 0: n_x known at compile time (7, 14): the dot products unrolled, their LDS reads in
// flight together (same terms, same order: the same bits as the runtime-n_x form)
template <int NXC>
__global__ __launch_bounds__(256) void k_cov_propagate(int N, int nx_rt, const double *__restrict__ A,
                                                       const double *__restrict__ q,
                                                       const double *__restrict__ S0, double s0_diag,
                                                       double *__restrict__ out) {
  __shared__ double sA[UP_CHUNK][UP_NXMAX][UP_NXMAX + 1];
  __shared__ double sq[UP_CHUNK][UP_NXMAX];
  __shared__ double sS[UP_NXMAX][UP_NXMAX + 1];
  __shared__ double sT[UP_NXMAX][UP_NXMAX + 1];
  const int nx = NXC > 0 ? NXC : nx_rt;
  const int b = blockIdx.x, e = threadIdx.x, nt = blockDim.x, nn = nx * nx;
  const int64_t mat = (int64_t)nn;
  const bool act = e < nn;
  const int i = act ? e / nx : 0, j = act ? e - (e / nx) * nx : 0;
  double *ob = out + (int64_t)b * (N + 1) * mat;
  if (act) {
    const double v = S0 ? S0[(int64_t)b * mat + e] : (i == j ? s0_diag : 0.0);
    sS[i][j] = v;
    ob[e] = v;
  }
  for (int k0 = 0; k0 < N; k0 += UP_CHUNK) {
    const int kc = min(UP_CHUNK, N - k0);
    const double *Ac = A + ((int64_t)b * N + k0) * mat;
    const double *qc = q + ((int64_t)b * N + k0) * nx;
    for (int t = e; t < kc * nn; t += nt) {
      const int kk = t / nn, r = t - kk * nn, ri = r / nx;
      sA[kk][ri][r - ri * nx] = Ac[t];
    }
    for (int t = e; t < kc * nx; t += nt) {
      const int kk = t / nx;
      sq[kk][t - kk * nx] = qc[t];
    }
    __syncthreads();
    for (int kk = 0; kk < kc; ++kk) {
      if (act) {  // T = A Sigma
        double t = 0.0;
#pragma unroll
        for (int c = 0; c < (NXC > 0 ? NXC : UP_NXMAX); ++c)
          if (NXC > 0 || c < nx) t = fma(sA[kk][i][c], sS[c][j], t);
        sT[i][j] = t;
      }
      __syncthreads();
      if (act) {  // Sigma' = T A^T + diag(q)
        double t = 0.0;
#pragma unroll
        for (int c = 0; c < (NXC > 0 ? NXC : UP_NXMAX); ++c)
          if (NXC > 0 || c < nx) t = fma(sT[i][c], sA[kk][j][c], t);
        if (i == j) t += sq[kk][i];
        ob[(int64_t)(k0 + kk + 1) * mat + e] = t;
        sS[i][j] = t;
      }
      __syncthreads();
    }
  }
}

static hipError_t launch_cov_propagate(hipStream_t s, int batch, int N, int nx, const double *A,
                                       const double *q, const double *S0, double s0_diag,
                                       double *out) {
  const dim3 g(batch), t((nx * nx + 63) / 64 * 64);
  if (nx == 7) hipLaunchKernelGGL(k_cov_propagate<7>, g, t, 0, s, N, nx, A, q, S0, s0_diag, out);
  else if (nx == 14) hipLaunchKernelGGL(k_cov_propagate<14>, g, t, 0, s, N, nx, A, q, S0, s0_diag, out);
  else hipLaunchKernelGGL(k_cov_propagate<0>, g, t, 0, s, N, nx, A, q, S0, s0_diag, out);
  return hipGetLastError();
}

extern "C" int gpmpc_cov_propagate_dev(gpmpc_ctx *ctx, int batch, int N, int nx, const double *dA,
                                       const double *dq, const double *dS0, double s0_diag,
                                       double *dout) {
  GPMPC_CHECK_ARG(ctx && dA && dq && dout && batch >= 0 && N >= 0 && nx >= 1 && nx <= UP_NXMAX);
  if (batch == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  GPMPC_HIP(launch_cov_propagate(ctx->stream, batch, N, nx, dA, dq, dS0, s0_diag, dout));
  return 0;
}

extern "C" int gpmpc_cov_propagate(gpmpc_ctx *ctx, int batch, int N, int nx, const double *A,
                                   const double *q, const double *S0, double s0_diag,
                                   double *out) {
  GPMPC_CHECK_ARG(ctx && A && q && out && batch >= 0 && N >= 0 && nx >= 1 && nx <= UP_NXMAX);
  if (batch == 0) return 0;
  GPMPC_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const size_t mat = (size_t)nx * nx;
  DevBuf dA, dq, dS, dout;
  GPMPC_HIP(dA.alloc(s, sizeof(double) * (size_t)batch * N * mat + 8));
  GPMPC_HIP(dq.alloc(s, sizeof(double) * (size_t)batch * N * nx + 8));
  GPMPC_HIP(dout.alloc(s, sizeof(double) * (size_t)batch * (N + 1) * mat));
  if (N > 0) {
    GPMPC_HIP(hipMemcpyAsync(dA.p, A, sizeof(double) * (size_t)batch * N * mat,
                             hipMemcpyHostToDevice, s));
    GPMPC_HIP(hipMemcpyAsync(dq.p, q, sizeof(double) * (size_t)batch * N * nx,
                             hipMemcpyHostToDevice, s));
  }
  if (S0) {
    GPMPC_HIP(dS.alloc(s, sizeof(double) * (size_t)batch * mat));
    GPMPC_HIP(hipMemcpyAsync(dS.p, S0, sizeof(double) * (size_t)batch * mat,
                             hipMemcpyHostToDevice, s));
  }
  GPMPC_HIP(launch_cov_propagate(s, batch, N, nx, dA.as<double>(), dq.as<double>(),
                                 S0 ? dS.as<double>() : nullptr, s0_diag, dout.as<double>()));
  GPMPC_HIP(hipMemcpyAsync(out, dout.p, sizeof(double) * (size_t)batch * (N + 1) * mat,
                           hipMemcpyDeviceToHost, s));
  GPMPC_HIP(hipStreamSynchronize(s));
  return 0;
}
