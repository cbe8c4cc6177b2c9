// uprop.hip -- batched linear covariance propagation along MPC horizons
// (reference src/mpc/uncertainty_prop.py:117-177, UncertaintyPropagator._propagate_linear):
//
//   Sigma_{k+1} = (A_k Sigma_k) A_k^T + diag(q_k),   k = 0 .. N-1
//
// q_k is the GP variance as process noise (var * dt^2 on the velocity block,
// and on the angular-rate block for 6-DoF), A_k the discrete Jacobian of the
// nominal step.  The mean recursion does not depend on Sigma, so the host
// (or the fleet) produces every A_k and q_k first and one launch runs all
// trajectories.  One 64-lane wave per trajectory; n_x <= 16, so Sigma, A_k and
// the product A_k Sigma_k live in LDS and each lane owns up to 4 of the n_x^2
// entries.  HBM traffic per trajectory-step: read A_k (8 n_x^2 B) and q_k
// (8 n_x B), write Sigma_{k+1} (8 n_x^2 B).
#include "internal.h"

#define UP_NXMAX 16

__global__ __launch_bounds__(64) void k_cov_propagate(int N, int nx, const double *__restrict__ A,
                                                      const double *__restrict__ q,
                                                      const double *__restrict__ S0, double s0_diag,
                                                      double *__restrict__ out) {
  __shared__ double sA[UP_NXMAX][UP_NXMAX + 1];
  __shared__ double sS[UP_NXMAX][UP_NXMAX + 1];
  __shared__ double sT[UP_NXMAX][UP_NXMAX + 1];
  const int b = blockIdx.x, lane = threadIdx.x, nn = nx * nx;
  const int64_t mat = (int64_t)nn;
  double *ob = out + (int64_t)b * (N + 1) * mat;
  for (int e = lane; e < nn; e += 64) {
    const int i = e / nx, j = e % nx;
    const double v = S0 ? S0[(int64_t)b * mat + e] : (i == j ? s0_diag : 0.0);
    sS[i][j] = v;
    ob[e] = v;
  }
  for (int k = 0; k < N; ++k) {
    const double *Ak = A + ((int64_t)b * N + k) * mat;
    const double *qk = q + ((int64_t)b * N + k) * nx;
    for (int e = lane; e < nn; e += 64) sA[e / nx][e % nx] = Ak[e];
    __syncthreads();
    for (int e = lane; e < nn; e += 64) {  // T = A Sigma
      const int i = e / nx, j = e % nx;
      double t = 0.0;
      for (int c = 0; c < nx; ++c) t = fma(sA[i][c], sS[c][j], t);
      sT[i][j] = t;
    }
    __syncthreads();
    double *ok = ob + (int64_t)(k + 1) * mat;
    for (int e = lane; e < nn; e += 64) {  // Sigma' = T A^T + diag(q)
      const int i = e / nx, j = e % nx;
      double t = 0.0;
      for (int c = 0; c < nx; ++c) t = fma(sT[i][c], sA[j][c], t);
      if (i == j) t += qk[i];
      ok[e] = t;
      sS[i][j] = t;
    }
    __syncthreads();
  }
}

static hipError_t launch_cov_propagate(hipStream_t s, int batch, int N, int nx, const double *A,
                                       const double *q, const double *S0, double s0_diag,
                                       double *out) {
  hipLaunchKernelGGL(k_cov_propagate, dim3(batch), dim3(64), 0, s, N, nx, A, q, S0, s0_diag, out);
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
