// gemm.h -- internal launchers shared across translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>

enum { EPI_STORE = 0, EPI_SUMSQ = 1 };

// acc = A(M x K) B(N x K)^T; see gemm.hip.  For EPI_SUMSQ, C is the partial
// buffer (ceil(M/64) x ldc) and row tile t writes row t.
hipError_t launch_gemm_nt(hipStream_t s, int epi, int M, int N, int K, const double *A,
                          int64_t lda, const double *B, int64_t ldb, double *C, int64_t ldc,
                          double alpha, double beta, int tri_a, int lower_c, int batch,
                          int64_t sA, int64_t sB, int64_t sC);

// C = alpha A B^T + beta C, N <= 128, one workgroup per 128-row block (C may alias
// A); lower_c: only C[i][j] with j <= i (relative to C) is written
hipError_t launch_gemm_nt_rowblock(hipStream_t s, int M, int N, int K, const double *A,
                                   int64_t lda, const double *B, int64_t ldb, double *C,
                                   int64_t ldc, double alpha, double beta, int batch, int64_t sA,
                                   int64_t sB, int64_t sC, int lower_c = 0, int ksplit = 1);

// the potrf's diagonal-block update C -= A A^T (lower w x w, w <= 128; A: the block's rows'
// K left columns, ld lda; C ld lda; batch matrices stride apart; K split in ks, atomics)
hipError_t launch_syrk128_diag(hipStream_t s, int w, int K, const double *A, int64_t lda, double *C, int batch,
                               int64_t stride, int ks);

// the potrf's fused left-looking step for the rows below a diagonal block (gemm.hip):
// C (M x 128) <- (C - A B^T) Linv^T, A (M x K) and B (128 x K) with leading dimension lda,
// Linv (128 x 128, lower, ld 128); batch a multiple of 8.  wn > 0 (<= 128, <= M): also
// D -= A[0:wn, 0:K+128] A[0:wn, 0:K+128]^T (lower) for the next diagonal block D = C + 128
hipError_t launch_gemm_updsolve(hipStream_t s, int M, int K, const double *A, int64_t lda, const double *B,
                                double *C, const double *Linv, int batch, int64_t sA, int64_t sC, int64_t sL,
                                int wn = 0);

// latency form for K <= 128 (see gemm.hip): mode 0 = rows in place (N <= 128,
// C may alias A; tri_b: B lower-triangular), mode 1 = lower C += A A^T (M == N)
hipError_t launch_gemm_lat(hipStream_t s, int mode, int M, int N, int K, const double *A,
                           int64_t lda, const double *B, int64_t ldb, double *C, int64_t ldc,
                           double alpha, double beta, int tri_b, int batch, int64_t sA, int64_t sB,
                           int64_t sC);

// C = alpha A B + beta C with B (K x N) row-major ("NN")
hipError_t launch_gemm_nn(hipStream_t s, int M, int N, int K, const double *A, int64_t lda,
                          const double *B, int64_t ldb, double *C, int64_t ldc, double alpha,
                          double beta);

hipError_t launch_gemm_nn_batched(hipStream_t s, int M, int N, int K, const double *A, int64_t lda, int64_t sA,
                                  const double *B, int64_t ldb, int64_t sB, double *C, int64_t ldc, int64_t sC,
                                  double alpha, double beta, int batch);

// C = alpha A^T B + beta C with A (K x M) and B (K x N) row-major ("TN")
hipError_t launch_gemm_tn(hipStream_t s, int M, int N, int K, const double *A, int64_t lda,
                          const double *B, int64_t ldb, double *C, int64_t ldc, double alpha,
                          double beta);

// W = L^-1 with W preset to the identity; tmp: >= (n/2 rounded up to TB) squared doubles
hipError_t launch_tri_inverse(hipStream_t s, int n, const double *L, int64_t ldl, double *W,
                              int64_t ldw, double *tmp);

hipError_t launch_trsm_lower_ex(hipStream_t s, int n, int nrhs, const double *L, int64_t ldl,
                                double *X, int64_t ldx, int trans, int rhs_lower,
                                double *Linv_blocks);

// posterior in one pass: Wext = [W (n x n, lower); alpha^T (n_out x n)]:
// part[t][j] = sum over W rows of tile t of (W K*^T)^2, meanT = alpha^T K*^T
// (n_out x P).  part has gemm_row_tiles(n + n_out) rows -- gemm_sumsq_rows(kind) with a
// forced kind.  The kernels sum in different k orders (not the same bits), so a caller
// whose P shrinks over time passes the kind of its planned size (gemm_sumsq_kind).
enum { GEMM_SUMSQ_64 = 0, GEMM_SUMSQ_128 = 1, GEMM_SUMSQ_SPLITK = 2 };
int gemm_sumsq_kind(int M, int N, int K);
inline int gemm_sumsq_rows(int kind, int M) { return kind == GEMM_SUMSQ_128 ? (M + 127) / 128 : (M + 63) / 64; }
hipError_t launch_gemm_sumsq_mean(hipStream_t s, int n, int n_out, int P, const double *Wext,
                                  const double *Ks, double *part, int64_t ldp, double *meanT,
                                  int64_t ldm, int kind = -1);
// part[t][j] = sum over the rows of tile t of (A K*^T)^2, A (n x n lower, ld n), K* (P x n)
hipError_t launch_gemm_sumsq(hipStream_t s, int n, int P, const double *A, const double *Ks, double *part,
                             int64_t ldp, int kind = -1);

// the same pass with K* formed in the operand load from the scaled query rows
// Qs (P x d) / norms Qn and training rows Xs (n x d) / norms Xn (d = 11..13;
// hipErrorInvalidValue otherwise): no K* buffer.  128-row tiles: part has
// ceil((n + n_out) / 128) rows.
hipError_t launch_gemm_post_fused(hipStream_t s, int n, int n_out, int P, const double *Wext,
                                  const double *Qs, const double *Qn, const double *Xs,
                                  const double *Xn, int d, int kind, double sigma2,
                                  double iso_scale, double *part, int64_t ldp, double *meanT,
                                  int64_t ldm);

// the column-stationary posterior (post.hip): exact GPs with n <= 1008 (63 row blocks of
// 16 + the alpha block), n_out <= 16, d in 11..13.  launch_post_pack forms its operands
// (Wf: post_cs_frag_doubles(n) doubles; Xp: n x post_cs_row_pitch(d)) from [W; alpha^T]
// (ld ldw), Xs, Xn; launch_post_cs forms K* from the scaled queries Qs (P x d) / Qn on the
// fly and writes part (2 rows, ld ldp: the two row halves' sums of squares) and meanT.
bool post_cs_ok(int n, int n_out, int d);
int post_cs_blocks(int n);
size_t post_cs_frag_doubles(int n);
int post_cs_row_pitch(int d);
hipError_t launch_post_pack(hipStream_t s, int n, int n_out, const double *Wext, int64_t ldw,
                            const double *Xs, const double *Xn, int d, double *Wf, double *Xp);
hipError_t launch_post_cs(hipStream_t s, int n, int n_out, int P, const double *Wf, const double *Xp,
                          const double *Qs, const double *Qn, int d, int kind, double sigma2, double iso_scale,
                          double *part, int64_t ldp, double *meanT, int64_t ldm);
#define POST_CS_PARTS 2
bool post_cs_env();  // GPMPC_POST_CS (default 0)

// rows of the SUMSQ partial buffer for an M x N x K product (tile height of
// the kernel launch_gemm_* picks: 128 when M, N and K >= 256, else 64)
inline int gemm_row_tiles(int M, int N = 0, int K = 0) {
  const char *e = getenv("GPMPC_GEMM128");
  const bool big = (!e || atoi(e)) && M >= 256 && N >= 256 && K >= 256;
  return big ? (M + 127) / 128 : (M + 63) / 64;
}
