/*
 * gpmpc.h -- C-ABI of libgpmpc_hip.so, the MI355X (gfx950) GP + QP hot path.
 *
 * The reference (shiivashaakeri/gp-mpc-rocket-landing) is pure Python: its
 * "boundary" for this path is a set of duck-typed classes whose heavy lifting
 * is numpy/LAPACK and the third-party OSQP C solver.  Each entry point below
 * replaces one of those native calls; the Python mirror in
 * gp_mpc_rocket_landing_amd/ binds them with ctypes.
 *
 * Conventions
 *   - every function returns int: 0 = ok, >0 = LAPACK-style info (e.g. the
 *     1-based column of the first non-positive pivot), <0 = argument / HIP
 *     error (gpmpc_last_error() has the message).  Nothing throws.
 *   - all arithmetic is fp64; host buffers are caller-owned, row-major, with
 *     explicit leading dimensions.  Functions suffixed _dev take device
 *     pointers that must stay resident for the call.
 *   - one gpmpc_ctx per process/rank owns one HIP stream; a ctx is not
 *     thread-safe.
 */
#ifndef GPMPC_H
#define GPMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: gpmpc_fleet_config gained sqp_iters / sqp_tol (round 2) and
 * gpmpc_rollout6_config the GPMPC problem data (round 3);
 * 3: gpmpc_rollout6_config gained the rocket parameters and horizon 20 or 30,
 * gpmpc_rollout6_solve_ref (X_ref / U_ref), gpmpc_comm_count (round 4); round 4 also
 * gave gpmpc_fleet_config.sqp_qp the max_iter = 0 "same as qp" meaning.  Round 5 adds
 * entry points only (gpmpc_fleet_get_posterior, gpmpc_gather_prepare / _collective) and
 * refuses a fleet config whose sqp_qp was edited with max_iter left 0.
 * 4 (round 6): gpmpc_rollout6_config gained rocket_J (the full inertia tensor); new
 * entry points gpmpc_fleet_create_shard, gpmpc_fleet_create_fitc. */
#define GPMPC_ABI_VERSION 4

typedef struct gpmpc_ctx gpmpc_ctx;
typedef struct gpmpc_gp gpmpc_gp;
typedef struct gpmpc_fitc gpmpc_fitc;
typedef struct gpmpc_fleet gpmpc_fleet;

/* kernel kinds: kernels.py:130 (SE-ARD), :392 (isotropic SE), :482 (Matern32), :579 (Matern52) */
enum { GPMPC_SE_ARD = 0, GPMPC_SE_ISO = 1, GPMPC_MATERN32 = 2, GPMPC_MATERN52 = 3 };

/* Composite kernels (kernels.py:676-844: SumKernel, ProductKernel, WhiteNoise) as a
 * postfix program: nops pairs (code, offset into par).  Leaves: the four kinds above
 * (par[off] = sigma2, then the d lengthscales; SE_ISO: sigma2, l) and GPMPC_KP_WHITE
 * (par[off] = its noise variance: on the diagonal of a Gram of one row set, zero
 * between two sets, kernels.py:805-815).  GPMPC_KP_SUM / _PROD combine the two values
 * on top of the stack.  E.g. SumKernel(SE_ARD(d), WhiteNoise(s)): ops = {0,0, 4,d+1, 10,0},
 * par = {sigma2, l_0..l_{d-1}, s}.  At most GPMPC_KP_MAXOPS pairs, stack depth 8. */
enum { GPMPC_KP_WHITE = 4, GPMPC_KP_SUM = 10, GPMPC_KP_PROD = 11 };
#define GPMPC_KP_MAXOPS 64
#define GPMPC_KP_MAXSTACK 8

/* OSQP-style status values (OSQP 0.6 constants.h), reported by the ADMM. */
enum {
  GPMPC_QP_SOLVED = 1, GPMPC_QP_SOLVED_INACCURATE = 2, GPMPC_QP_MAX_ITER_REACHED = -2,
  GPMPC_QP_PRIMAL_INFEASIBLE = -3, GPMPC_QP_PRIMAL_INFEASIBLE_INACCURATE = 3,
  GPMPC_QP_DUAL_INFEASIBLE = -4, GPMPC_QP_DUAL_INFEASIBLE_INACCURATE = 4,
  GPMPC_QP_NON_CVX = -7, GPMPC_QP_UNSOLVED = -10
};

int gpmpc_abi_version(void);
const char *gpmpc_last_error(void);

/* ---- context ---------------------------------------------------------- */
int gpmpc_ctx_create(int device, gpmpc_ctx **out);
int gpmpc_ctx_destroy(gpmpc_ctx *ctx);
int gpmpc_ctx_sync(gpmpc_ctx *ctx);
/* the HIP stream the context launches on (hipStream_t as void*) */
void *gpmpc_ctx_stream(gpmpc_ctx *ctx);

/* ---- a2/a3: kernel Gram matrix -----------------------------------------
 * Replaces SquaredExponentialARD.__call__ / Matern32/52.__call__ /
 * SquaredExponential.__call__ (kernels.py:238-262, :532-545, :625-637,
 * :417-432): K[i,j] = k(X1[i], X2[j]).  X2 == NULL means X2 = X1.
 * ls: d lengthscales (SE_ISO reads ls[0]). */
int gpmpc_gram(gpmpc_ctx *ctx, int kind, const double *X1, int n1, const double *X2, int n2,
               int d, const double *ls, double sigma2, double *K, int ldk);
/* Hyperparameter gradients of the Gram, d K / d(log theta)
 * (SquaredExponentialARD.gradients kernels.py:279-318: K (x1_i - x2_i)^2 / l_i^2
 * for every input dimension i; SquaredExponential.gradients :438-456:
 * K r^2 / l^2).  kind SE_ARD writes d matrices, SE_ISO one, each n1 x n2
 * row-major, stacked in G; K (n1 x n2) is written too unless NULL.  The
 * log-signal-variance gradient is K itself (and the only one the reference's
 * Matern kernels define). */
int gpmpc_gram_grad(gpmpc_ctx *ctx, int kind, const double *X1, int n1, const double *X2, int n2,
                    int d, const double *ls, double sigma2, double *K, double *G);

/* ---- Cholesky factor / solve -------------------------------------------
 * Replaces np.linalg.cholesky (exact_gp.py:164,170; sparse_gp.py:187,205).
 * In place on the lower triangle; info = 1-based first non-positive pivot
 * (returned as well).  info = -1: the factor kernel's bounded internal wait
 * expired (a broken invariant, factor unreliable); the call then returns -1
 * with gpmpc_last_error naming it. */
int gpmpc_potrf(gpmpc_ctx *ctx, int n, double *A, int lda, int *info);
/* batch x (n x n) SPD matrices, device-resident, stride elements apart;
 * dinfo: device int[batch], with gpmpc_potrf's meaning per matrix (the caller
 * reads it; -1 marks an unreliable factor). */
int gpmpc_potrf_batched_dev(gpmpc_ctx *ctx, int n, int batch, double *dA, int lda, int64_t stride,
                            int *dinfo);
/* C = alpha A A^T + beta C on the lower triangle (dsyrk 'L','N') for batch
 * device matrices: A (n x k, lda), C (n x n, ldc); the trailing update of the
 * blocked potrf (FP64 MFMA). */
int gpmpc_syrk_batched_dev(gpmpc_ctx *ctx, int n, int k, int batch, const double *dA, int lda,
                           int64_t strideA, double *dC, int ldc, int64_t strideC, double alpha,
                           double beta);
/* Replaces scipy.linalg.solve_triangular(L, B, lower=True) (exact_gp.py:251,260;
 * sparse_gp.py:190,293,296): B (n x nrhs) overwritten by L^-1 B. */
int gpmpc_trsm_lower(gpmpc_ctx *ctx, int n, int nrhs, const double *L, int ldl, double *B, int ldb);
/* Replaces scipy.linalg.cho_solve((L, True), B) (exact_gp.py:179; sparse_gp.py:210,214). */
int gpmpc_potrs(gpmpc_ctx *ctx, int n, int nrhs, const double *L, int ldl, double *B, int ldb);

/* ---- a4-a6: exact GP ------------------------------------------------------
 * MultiOutputExactGP.fit (exact_gp.py:476-499 -> ExactGP.fit :118-184) for
 * n_out outputs sharing one kernel (one Gram + one Cholesky).
 * Y is (n x n_out) row-major.  Reproduces the jitter ladder of
 * exact_gp.py:163-175; jitter_steps = 0 (none) .. 6, and the function returns
 * GPMPC_ERR_NOT_PD (-100) when the ladder is exhausted (the reference raises
 * ValueError).  Outputs per output: y_mean, y_std, lml. */
#define GPMPC_ERR_NOT_PD (-100)
int gpmpc_gp_fit_exact(gpmpc_ctx *ctx, int kind, const double *X, int n, int d, const double *Y,
                       int n_out, const double *ls, double sigma2, double noise, gpmpc_gp **out,
                       double *y_mean, double *y_std, double *lml, int *jitter_steps);
/* gpmpc_gp_fit_exact with any kernel (ExactGP(kernel=...) fits whatever Kernel it is
 * given, exact_gp.py:157): the Gram from a composite-kernel program over the raw rows
 * (GPMPC_KP_*); predict / predict_cov then form K* and K** from the same program, and
 * the prior variance k(x, x) is the program's diagonal (a constant: the sum / product
 * of its leaves' sigma2).  -2 for a malformed program.  gpmpc_gp_append refits such a
 * GP (returns GPMPC_ERR_NOT_PD). */
int gpmpc_gp_fit_exact_prog(gpmpc_ctx *ctx, const int *ops, int nops, const double *par, int npar,
                            const double *X, int n, int d, const double *Y, int n_out, double noise,
                            gpmpc_gp **out, double *y_mean, double *y_std, double *lml, int *jitter_steps);
/* ExactGP.predict (exact_gp.py:213-268) for all outputs: mean/var (p x n_out). */
int gpmpc_gp_predict(gpmpc_ctx *ctx, gpmpc_gp *gp, const double *Xq, int p, double *mean,
                     double *var);
/* ExactGP.predict(return_cov=True) (exact_gp.py:247-254): cov (p x p) of the
 * latent posterior in normalised units (caller multiplies by y_std^2). */
int gpmpc_gp_predict_cov(gpmpc_ctx *ctx, gpmpc_gp *gp, const double *Xq, int p, double *mean,
                         double *cov);
/* append k training rows Xnew (k x d) to a fitted GP in O(n^2 k)
 * -- the result of gpmpc_gp_fit_exact on the concatenated data without the
 * O(n^3) refit (SparseGP.update's refit-with-concatenation semantics,
 * sparse_gp.py:328-353; online_update.py:361-408).  Yall holds the targets of
 * all n + k rows ((n + k) x n_out, old rows first): normalisation, alpha and
 * lml are recomputed over all of them.  Returns GPMPC_ERR_NOT_PD, with the
 * handle unchanged, when the GP was fitted with jitter or the new rows' Schur
 * complement is not positive definite: the caller refits the whole set (which
 * reruns the exact_gp.py:163-175 ladder).  A fleet built on the GP must be
 * recreated after an append (its scratch is sized for the old row count). */
int gpmpc_gp_append(gpmpc_ctx *ctx, gpmpc_gp *gp, const double *Xnew, int k, const double *Yall,
                    double *y_mean, double *y_std, double *lml);
/* Copies of the device state (L lower, n x n; alpha n x n_out). Either may be NULL. */
int gpmpc_gp_get_state(gpmpc_ctx *ctx, gpmpc_gp *gp, double *L, double *alpha);
int gpmpc_gp_destroy(gpmpc_gp *gp);

/* ---- 8f-3: batched log marginal likelihood (hyperparameter search) --------
 * Replaces the objective of ExactGP.optimize_hyperparameters
 * (exact_gp.py:357-421), each call of which is a full ExactGP.fit
 * (exact_gp.py:118-204), for B parameter sets at once: per set b the Gram of
 * X (n x d) with lengthscales ls[b*d .. b*d+d) (SE_ISO: ls[b*d]) and signal
 * variance sigma2[b], + noise[b] I, Cholesky (one batched launch; the
 * exact_gp.py:163-175 jitter ladder for sets that fail), and
 * lml[b] = -1/2 y^T alpha - sum log L_ii - n/2 log 2 pi on the normalised y.
 * jitter_steps[b] = 0..6, or -1 (and lml[b] = -inf) when the ladder is
 * exhausted -- the reference objective's ValueError -> inf. */
int gpmpc_gp_lml_batched(gpmpc_ctx *ctx, int kind, const double *X, int n, int d,
                         const double *y, int B, const double *ls, const double *sigma2,
                         const double *noise, double *lml, int *jitter_steps);

/* ---- a8-a10: FITC sparse GP ----------------------------------------------
 * MultiOutputSparseGP.fit (sparse_gp.py:430-456 -> SparseGP.fit FITC :150-219)
 * with caller-supplied inducing points Z (m x d) shared by all outputs.
 * Outputs per output: y_mean, y_std, lml.  Lambda (n) optional. */
int gpmpc_fitc_fit(gpmpc_ctx *ctx, const double *Z, int m, const double *X, int n, int d,
                   const double *Y, int n_out, const double *ls, double sigma2, double noise,
                   double jitter, gpmpc_fitc **out, double *y_mean, double *y_std, double *lml,
                   double *lambda_diag);
/* SparseGP(method="vfe").fit (sparse_gp.py:221-249 after the shared :181-188):
 * B = K_uu + K_uf K_fu / noise + jitter I, alpha = B^-1 K_uf y / noise, the VFE
 * lower bound as lml.  Same handle type as gpmpc_fitc_fit: gpmpc_fitc_predict
 * evaluates it with the reference's one predict body (sparse_gp.py:255-305). */
int gpmpc_vfe_fit(gpmpc_ctx *ctx, const double *Z, int m, const double *X, int n, int d,
                  const double *Y, int n_out, const double *ls, double sigma2, double noise,
                  double jitter, gpmpc_fitc **out, double *y_mean, double *y_std, double *lml);
/* SparseGP(kernel=any).fit (sparse_gp.py:182-183: K_uu = kernel(Z), K_uf = kernel(Z, X),
 * the diagonal kernel.diagonal(X)) with a composite-kernel program (above); method 0 =
 * FITC (lambda_diag optional), 1 = VFE. */
int gpmpc_sparse_fit_prog(gpmpc_ctx *ctx, int method, const int *ops, int nops, const double *par, int npar,
                          const double *Z, int m, const double *X, int n, int d, const double *Y, int n_out,
                          double noise, double jitter, gpmpc_fitc **out, double *y_mean, double *y_std,
                          double *lml, double *lambda_diag);
/* SparseGP.predict (sparse_gp.py:255-305), mean as written. */
int gpmpc_fitc_predict(gpmpc_ctx *ctx, gpmpc_fitc *gp, const double *Xq, int p, double *mean,
                       double *var);
/* copy of the fitted alpha (m x n_out: L_B^-T L_B^-1 A Lambda^-1 y per output,
 * sparse_gp.py:208-210) */
int gpmpc_fitc_get_state(gpmpc_ctx *ctx, gpmpc_fitc *gp, double *alpha);
int gpmpc_fitc_destroy(gpmpc_fitc *gp);

/* ---- a15: batched OSQP-style ADMM ------------------------------------------
 * Replaces osqp.OSQP().setup / update / warm_start / solve
 * (osqp_rti.py:464-478, 496, 517, 524, 527) for a batch of QPs
 *     min 1/2 x'Px + q'x  s.t.  l <= Ax <= u
 * sharing one sparsity pattern of A (CSR: rowptr m+1, colidx nnz) and a
 * diagonal P.  Per problem: Aval (nnz), Pdiag (n), q (n), l/u (m).  The
 * reduced KKT matrix M = P + sigma I + A' diag(rho) A is factored either
 * block-tridiagonally (the MPC stage structure: blocks of 10 variables
 * coupled through their first 7, n <= 216) or, for any other pattern, as a
 * banded LDL^T with half-bandwidth <= 16.  Caps: n <= 216, m <= 360,
 * nnz <= 736, <= 8 entries per row and <= 12 per column of A.
 * State carried between solves (OSQP keeps it in its workspace):
 *   rho (batch), y_scaled (batch x m).  x_ws: warm-start primal (unscaled).
 * Outputs: x (batch x n), y (batch x m) unscaled, iters, status, obj. */
typedef struct {
  double rho, sigma, alpha;
  double eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
  int max_iter, check_termination, adaptive_rho, adaptive_rho_interval;
  double adaptive_rho_tolerance;
  int scaling, warm_start;
} gpmpc_qp_settings;
void gpmpc_qp_default_settings(gpmpc_qp_settings *s); /* osqp_rti.py:54-60 + OSQP 0.6 defaults */
int gpmpc_qp_solve_batched(gpmpc_ctx *ctx, int batch, int n, int m, int nnz, const int *rowptr,
                           const int *colidx, const double *Aval, const double *Pdiag,
                           const double *q, const double *l, const double *u,
                           const gpmpc_qp_settings *s, const double *x_ws, double *rho,
                           double *y_scaled, double *x, double *y, int *iters, int *status,
                           double *obj);

/* ---- the control step: a fleet of closed-loop 3-DoF GP-MPC landings -------
 * One "step" = for every landing: GP posterior (mean + variance) at the N
 * horizon points of its linearisation trajectory, RTI QP assembly with the GP
 * mean on the velocity rows (gp_mpc.py:303-320, correct sign), batched ADMM
 * (osqp_rti.py:501-567 protocol), plant step and Monte-Carlo termination
 * (monte_carlo.py:455-537).  Everything stays device-resident. */
typedef struct {
  int horizon;           /* N (osqp_rti.py OSQPRTIConfig.N / MPCConfig.N) */
  double dt;             /* control period */
  int target_mode;       /* must be 1: the solve protocol of monte_carlo.py:495-512 with its
                            incremental target (:497-500); the step protocol of
                            FastRTI3DoF is the host mirror (mpc/osqp_rti.py) */
  int use_gp;            /* add GP mean to c_k */
  int residual_model;    /* 1: plant gets the aero-drag residual (dispersion.py:349-360) */
  int max_steps;         /* max_time / dt */
  gpmpc_qp_settings qp;
  int sqp_iters;         /* 1: RTI, one QP per control step (the bench metric).
                            > 1: GPMPC.solve's loop (gp_mpc.py:296-345): up to sqp_iters
                            re-linearise -> GP posterior -> QP passes around the last QP
                            solution, stop when max|dX|, max|dU| < sqp_tol; not converged
                            -> MPCSolution.success False -> DIVERGENCE (monte_carlo.py
                            :506-508).  The warm start is the unshifted plan (gp_mpc.py
                            :358-359). */
  double sqp_tol;        /* 1e-4 (gp_mpc.py:343) */
  gpmpc_qp_settings sqp_qp;  /* QP settings of the SQP passes (sqp_iters > 1).  sqp_qp.max_iter
                                = 0 (the default) means "the same as qp", resolved when the fleet
                                launches, so a caller that edits only qp changes the passes too.
                                With sqp_iters > 1 and max_iter 0, an sqp_qp that equals neither
                                the defaults nor qp (a field edited alongside max_iter 0, which
                                would be ignored) makes gpmpc_fleet_create fail (-2): set
                                sqp_qp.max_iter to give the passes their own settings.
                                The reference solves this subproblem with IPOPT (gp_mpc.py:462-470) */
} gpmpc_fleet_config;
void gpmpc_fleet_default_config(gpmpc_fleet_config *c);
int gpmpc_fleet_create(gpmpc_ctx *ctx, gpmpc_gp *gp, const gpmpc_fleet_config *cfg, int batch,
                       gpmpc_fleet **out);
/* A shard of batch landings of a Monte-Carlo fleet of fleet_batch landings (>= batch;
 * gpmpc_fleet_create = fleet_batch equal to batch).  Every size-dependent path choice
 * (the posterior GEMM's kernel, the few-query posterior launch, the control kernel's
 * build) is made once, here, for fleet_batch landings -- never from the running count --
 * so each landing's results are bit-identical whatever the shard size and however many
 * landings still fly beside it. */
int gpmpc_fleet_create_shard(gpmpc_ctx *ctx, gpmpc_gp *gp, const gpmpc_fleet_config *cfg, int batch,
                             int fleet_batch, gpmpc_fleet **out);
/* The same fleet over a sparse GP (gpmpc_fitc_fit / gpmpc_vfe_fit, 11 features, 3
 * outputs): the reference-default Simple3DoFGP() is MultiOutputSparseGP FITC with 50
 * inducing points (structured_gp.py:423-428, sparse_gp.py:400-456).  Every step's
 * posterior is the reference's SparseGP.predict (sparse_gp.py:255-305) at every horizon
 * point: the mean K*u alpha as written (what GPMPC consumes through
 * gp.predict), the variance sigma2 - |L_uu^-1 k*|^2 + |L_B^-1 L_uu^-1 k*|^2.  The
 * sparse GP must outlive the fleet. */
int gpmpc_fleet_create_fitc(gpmpc_ctx *ctx, gpmpc_fitc *gp, const gpmpc_fleet_config *cfg, int batch,
                            int fleet_batch, gpmpc_fleet **out);
/* (re)initialise landings [first, first+count) from x0 (count x 7) */
int gpmpc_fleet_reset(gpmpc_fleet *f, int first, int count, const double *x0);
/* advance every active landing by nsteps control steps (async on the ctx stream) */
int gpmpc_fleet_step(gpmpc_fleet *f, int nsteps);
/* one step split in its phases, launched in the order 0, 2, 3, 1:
 * bit 0: horizon features + K* = k(Z*, X) Gram; bit 2: one FP64-MFMA pass
 * over K* with [L^-1; alpha^T]: variance partial sums |L^-1 K*^T|^2 and the
 * means alpha^T K*^T; bit 3: posterior finish;
 * bit 1: QP assembly + ADMM + plant step.  A full step = phases(15). */
int gpmpc_fleet_step_phases(gpmpc_fleet *f, int phase_mask);
/* records (batch x GPMPC_REC_LEN doubles): 0 outcome (0 running, 1..6 =
 * LandingOutcome of monte_carlo.py:25-33), 1 steps, 2 fuel used, 3 flight time,
 * 4..10 state, 11 total ADMM iterations, 12 solves with status "solved",
 * 13 initial mass, 14 last QP status, 15 last rho */
#define GPMPC_REC_LEN 16
int gpmpc_fleet_read(gpmpc_fleet *f, double *records, double *x /* batch x 7, may be NULL */);
/* the rest of every landing's controller state, any pointer may be NULL:
 * linearisation / warm-start trajectory Xw (batch x (N+1) x 7) and Uw
 * (batch x N x 3), the ADMM's persistent scaled duals (batch x m) and rho
 * (batch) -- what OSQP keeps between solves (osqp_rti.py:517-527) */
int gpmpc_fleet_get_state(gpmpc_fleet *f, double *Xw, double *Uw, double *y_scaled, double *rho);
/* the last control step's GP posterior at every landing's N horizon points
 * (ExactGP.predict, exact_gp.py:256-266, over the step's linearisation
 * trajectory): mean and variance, batch x N x 3 each, in landing order (either
 * may be NULL).  The step covers the running prefix of its dispatch order (every
 * landing running at its start, plus terminated ones the host had not yet read):
 * those read the posterior at their own trajectory, landings past it read NaN.
 * -2 when use_gp = 0. */
int gpmpc_fleet_get_posterior(gpmpc_fleet *f, double *mean, double *var);
/* diagnostic: accumulate s_memtime cycles of landing 0's control kernel per
 * phase into dev_u64x16 (16 x uint64 device buffer; NULL disables):
 * 0 assembly, 1 scaling, 2 factor, 3 A' rhs, 4 KKT solve (band path, or the
 * block path's barrier tail), 5 fused z/y update, 6 checks + adaptive rho,
 * 7 tail (plant step, records), 8/9/10 block KKT solve forward / diagonal /
 * backward; 14 s_memrealtime ticks (100 MHz) and 15 shader-clock ticks over
 * the same solves */
int gpmpc_fleet_set_stamps(gpmpc_fleet *f, void *dev_u64x16);
/* diagnostic: per-landing control-kernel trace into dev_u64xbx4 (batch x 4
 * uint64 device buffer; NULL disables): start and end s_memrealtime (100 MHz),
 * HW_ID and XCC_ID of the landing's first wave */
int gpmpc_fleet_set_trace(gpmpc_fleet *f, void *dev_u64xbx4);
/* ---- uncertainty propagation (uncertainty_prop.py:117-177) ------------------
 * Replaces the covariance recursion of UncertaintyPropagator._propagate_linear
 * (Sigma_next = A_d @ Sigma_k @ A_d.T + Q_gp, uncertainty_prop.py:163-167) for
 * batch trajectories at once: A (batch x N x nx x nx), q (batch x N x nx, the
 * diagonal of Q_gp), S0 (batch x nx x nx, or NULL for s0_diag * I, the
 * reference's default 1e-6 I), out (batch x (N+1) x nx x nx), all row-major;
 * nx <= 16.  The host version copies in and out; _dev takes device pointers and
 * is asynchronous on the context stream. */
int gpmpc_cov_propagate(gpmpc_ctx *ctx, int batch, int N, int nx, const double *A, const double *q,
                        const double *S0, double s0_diag, double *out);
int gpmpc_cov_propagate_dev(gpmpc_ctx *ctx, int batch, int N, int nx, const double *dA,
                            const double *dq, const double *dS0, double s0_diag, double *dout);
/* UncertaintyPropagator._propagate_linear (uncertainty_prop.py:117-177) of the 3-DoF model
 * on the device, for batch trajectories in one call (what GPMPC.solve runs on every call,
 * gp_mpc.py:284-290, with N sequential GP predictions on the host): the explicit-Euler
 * dynamics of rocket_3dof.py (x+ = x + dt f, f = [-alpha |u|, v, u / m + g3]) plus dt times
 * the exact GP's mean on the velocity rows, A_k = I + dt J(x_k, u_k), q_k = dt^2 times the
 * GP variance on the velocity rows, Sigma_0 = S0 (batch x 7 x 7) or s0_diag I.  gp: the
 * 3-DoF exact GP (11 features, 3 outputs, a leaf kernel; else -2).  Host buffers: x0
 * (batch x 7), U (batch x N x 3) in; means (batch x (N+1) x 7), covs (batch x (N+1) x 7 x 7)
 * out.  (Round 6, ABI 4: an added entry point.) */
int gpmpc_uprop3_linear(gpmpc_ctx *ctx, gpmpc_gp *gp, int batch, int N, double dt, double alpha,
                        const double *g3, const double *x0, const double *U, const double *S0,
                        double s0_diag, double *means, double *covs);
/* The same for the 14-state model (uncertainty_prop.py:117-177 as GPMPC.solve runs it for
 * Rocket6DoFDynamics, gp_mpc.py:284-290): RK4 with quaternion normalisation
 * (rocket_6dof.py step) plus dt times the StructuredRocketGP means on the velocity
 * (rows 4-6, d_v) and rate rows (11-13, d_omega), A_k = I + dt J(x_k, u_k), q_k = dt^2 times
 * the GP variances on those rows.  gp_v / gp_w: the pair's device GPs, gpmpc_gp * (exact = 1)
 * or gpmpc_fitc * (exact = 0), 13 / 12 features and 3 outputs each, leaf kernels (else -2).
 * rocket: J_B (9, row-major; invertible), r_T_B (3), g_I (3), alpha = 1 / (I_sp g0), g0.
 * Host buffers: x0 (batch x 14), U (batch x N x 3), S0 (batch x 14 x 14) or NULL (s0_diag I)
 * in; means (batch x (N+1) x 14), covs (batch x (N+1) x 14 x 14) out.  (Round 6, ABI 4: an
 * added entry point.) */
int gpmpc_uprop6_linear(gpmpc_ctx *ctx, void *gp_v, void *gp_w, int exact, const double *rocket,
                        int batch, int N, double dt, const double *x0, const double *U,
                        const double *S0, double s0_diag, double *means, double *covs);

/* ---- BASELINE configs[4]: batched 6-DoF GP-MPC rollouts --------------------
 * gpmpc_rollout_batched of SURVEY 8b.  One step = for every running rollout:
 * the Monte-Carlo termination rules (monte_carlo.py:455-488 on [m, r, v]),
 * GPMPC.solve's forward simulation with the StructuredRocketGP FITC means
 * (gp_mpc.py:258-281; RK4 of nominal_mpc.py:163-203), the QP subproblem of
 * gp_mpc.py:394-460 in deviation variables with its QCQP rows made linear
 * (DESIGN.md section 9), the OSQP-0.6 ADMM on the block-tridiagonal reduced
 * KKT matrix, the truth plant step (RK4 + the dispersion.py:349-360 drag) and
 * the plan kept unshifted as the next warm start.  State 14 = [m, r_I, v_I,
 * q_BI (w, x, y, z), omega_B]; horizon 20 (GPMPCConfig's N, gp_mpc.py:110 /
 * nominal_mpc.py:47) or 30 (BASELINE configs[4]), each a compiled instance. */
typedef struct gpmpc_rollout6 gpmpc_rollout6;
typedef struct {
  int horizon;           /* 20 or 30 (the compiled instances); default 30 */
  double dt;
  int max_steps;
  gpmpc_qp_settings qp;  /* osqp_rti.py:54-60 defaults */
  int fitc_mean_as_written;  /* 1 (default since round 6): the reference's K*u alpha
                                (sparse_gp.py:280-283, SURVEY D1 kept); 0: the FITC
                                posterior mean K*u L_uu^-T alpha (D1 fixed) */
  /* GPMPC's problem data (ABI 2).  Defaults: CostWeights (cost_functions.py:39-98),
   * ConstraintParams (constraints.py:35-50), gp_mpc.py:432-435. */
  double q_diag[14];     /* stage cost Q (diagonal) */
  double p_diag[14];     /* terminal cost P (diagonal; 10 Q) */
  double r_diag[3];      /* control cost R (diagonal) */
  double t_min, t_max;   /* thrust magnitude bounds */
  double tan_gamma_gs;   /* tan of the glide-slope angle, np.tan(np.deg2rad(30)) */
  double trust_x2, trust_u2;  /* squared trust radii 10, 5 */
  int use_gp_mean;       /* GPMPCConfig.use_gp_mean: 0 drops the GP from the simulation and c_k */
  int upright_target;    /* rollouts: 0 = monte_carlo.py:497-500 as written (x copied, v = 0,
                            altitude - 2); 1 = also q = (1, 0, 0, 0), omega = 0 */
  /* the rocket (ABI 3): Rocket6DoFConfig (rocket_6dof.py:36-84) as the dynamics of
   * nominal_mpc.py:163-203 use it.  Defaults J_B = diag(0.02, 1, 1) 0.168 (a full
   * tensor: rocket_J below), r_T_B = (-0.25, 0, 0), g_I = (-1, 0, 0), I_sp 30, g0 1:
   * alpha = 1 / (I_sp g0); g0 also sets the hover guess [0, 0, m g0] (gp_mpc.py:271-275) */
  double rocket_j[3];    /* diagonal of J_B */
  double rocket_r_t[3];  /* thrust application point r_T_B */
  double rocket_g_i[3];  /* gravity g_I */
  double rocket_alpha;   /* 1 / (I_sp g0) */
  double rocket_g0;
  /* ABI 4: the full inertia tensor J_B (row-major 3 x 3, rocket_6dof.py:44, 77-78, 147:
   * any invertible matrix; nominal_mpc.py:196-199 solves with it).  All zeros (the
   * default) = diag(rocket_j).  A diagonal tensor runs exactly as its diagonal would. */
  double rocket_J[9];
} gpmpc_rollout6_config;
void gpmpc_rollout6_default_config(gpmpc_rollout6_config *c);
/* gp_v: FITC on the 13 translational features, gp_w: on the 12 rotational
 * ones (features.py:149-365), 3 outputs each; both must outlive the batch */
int gpmpc_rollout6_create(gpmpc_ctx *ctx, gpmpc_fitc *gp_v, gpmpc_fitc *gp_w,
                          const gpmpc_rollout6_config *cfg, int batch, gpmpc_rollout6 **out);
/* the same over a pair of exact GPs (StructuredRocketGP(use_sparse=False),
 * exact_gp.py:213-268: mean K* alpha over the training rows) */
int gpmpc_rollout6_create_exact(gpmpc_ctx *ctx, gpmpc_gp *gp_v, gpmpc_gp *gp_w,
                                const gpmpc_rollout6_config *cfg, int batch, gpmpc_rollout6 **out);
/* GPMPC.solve (gp_mpc.py:229-369) for every rollout b of the batch at x0[b]
 * (batch x 14) with target x_target[b] (batch x 14), X_ref = x_target, U_ref = 0:
 *   pass 1: forward simulation of the warm-start controls with the GP mean
 *           (gp_mpc.py:258-281), the QP around it (:394-460, made linear as the
 *           rollouts), plan <- X_pred + dX, U_pred + dU;
 *   pass p > 1: GP means and Jacobians at the last plan (:299-320), QP, plan;
 *   stop after max_sqp_iter passes or when max|X_new - X_pred| and
 *   max|U_new - U_pred| are both < sqp_tol (:336-345).
 * A QP without a solution returns the nominal trajectory (:478-482: X_new =
 * X_pred, so the loop stops as converged) with qp_status < 0 (not -2).
 * cold = 1: the hover guess [0, 0, m0 g0] at every stage and fresh ADMM duals /
 * rho (first call, GPMPC.reset_warm_start); cold = 2: fresh duals / rho, the
 * controls already set (gpmpc_rollout6_set_state: U_ref, :268-269); cold = 0:
 * the previous call's plan U, unshifted (:266-267, :358-359).  The batch's Monte-Carlo records are not
 * touched except rec[11] (ADMM iterations of this call), rec[12] (solves with
 * status solved), rec[14] (last QP status), rec[15] (rho).
 * Outputs (any may be NULL): X (batch x (N+1) x 14), U (batch x N x 3), passes,
 * converged (0 / 1), qp_status of the last pass, qp_iters summed over passes. */
int gpmpc_rollout6_solve(gpmpc_rollout6 *r, const double *x0, const double *x_target, int cold,
                         int max_sqp_iter, double sqp_tol, double *X, double *U, int *passes,
                         int *converged, int *qp_status, int *qp_iters);
/* the same with the QP cost's reference trajectory (gp_mpc.py:442-453): X_ref
 * (batch x (N+1) x 14; NULL = x_target on every stage) and U_ref (batch x N x 3;
 * NULL = 0) in sum_k |x_k - X_ref[k]|_Q^2 + |u_k - U_ref[k]|_R^2 + |x_N - X_ref[N]|_P^2.
 * (U_ref's other use, the first guess of :268-269, is cold = 2 after
 * gpmpc_rollout6_set_state.) */
int gpmpc_rollout6_solve_ref(gpmpc_rollout6 *r, const double *x0, const double *x_target, const double *X_ref,
                             const double *U_ref, int cold, int max_sqp_iter, double sqp_tol, double *X,
                             double *U, int *passes, int *converged, int *qp_status, int *qp_iters);
/* (re)start rollouts [first, first+count) at x0 (count x 14) */
int gpmpc_rollout6_reset(gpmpc_rollout6 *r, int first, int count, const double *x0);
/* nsteps control steps of every running rollout (async on the ctx stream) */
int gpmpc_rollout6_step(gpmpc_rollout6 *r, int nsteps);
/* one step split in its kernels, launched in order: bit 0 termination rules +
 * forward simulation + GP means + Jacobians (k_r6_predict), bit 1 QP + ADMM +
 * plan (k_r6_control), bit 2 truth plant step (k_r6_plant); a full step = 7 */
int gpmpc_rollout6_step_phases(gpmpc_rollout6 *r, int mask);
/* records (batch x GPMPC_REC_LEN, the fleet layout; state slots hold [m, r, v])
 * and the full states (batch x 14, may be NULL) */
int gpmpc_rollout6_read(gpmpc_rollout6 *r, double *records, double *x);
/* controller state, any pointer may be NULL: warm-start controls U (batch x N
 * x 3), last QP plan X (batch x (N+1) x 14), forward-simulated X_pred (batch x
 * (N+1) x 14), its GP means (batch x N x 6: d_v, d_omega), the ADMM's persistent
 * scaled duals (batch x M, M = 36 N + 24: 1104 at N = 30, 744 at N = 20) and rho (batch) */
int gpmpc_rollout6_get_state(gpmpc_rollout6 *r, double *U, double *X_plan, double *X_pred,
                             double *gp_mean, double *y_scaled, double *rho);
/* set controller state (any pointer may be NULL): U (batch x N x 3), scaled
 * duals (batch x M), rho (batch) -- e.g. to carry a warm start across a GP
 * refit, or to start GPMPC.solve from caller-given controls */
int gpmpc_rollout6_set_state(gpmpc_rollout6 *r, const double *U, const double *y_scaled, const double *rho);
int gpmpc_rollout6_destroy(gpmpc_rollout6 *r);

/* device pointer of the record array (for collectives) */
double *gpmpc_fleet_records_dev(gpmpc_fleet *f);
double *gpmpc_rollout6_records_dev(gpmpc_rollout6 *r);

/* ---- (e) the one collective: shard records to the root over RCCL -----------
 * SURVEY 8b gpmpc_gather_results.  Landings are sharded in contiguous blocks,
 * one process per GPU, with no data-path collective (monte_carlo.py:401-583 is
 * per landing); at the end one ncclGather over xGMI brings every rank's record
 * block to the root.  The communicator is bootstrapped from a ncclUniqueId
 * that rank 0 creates (gpmpc_comm_unique_id) and the caller distributes (a
 * file on local disk, or the process group it already has).  RCCL is loaded at
 * run time (librccl.so.1; the copy torch loaded when there is one). */
typedef struct gpmpc_comm gpmpc_comm;
#define GPMPC_COMM_ID_BYTES 128
int gpmpc_comm_unique_id(unsigned char *id /* GPMPC_COMM_ID_BYTES */);
int gpmpc_comm_init(gpmpc_ctx *ctx, const unsigned char *id, int nranks, int rank, gpmpc_comm **out);
int gpmpc_comm_destroy(gpmpc_comm *c);
/* ranks the RCCL communicator spans (ncclCommCount) */
int gpmpc_comm_count(gpmpc_comm *c, int *nranks);
/* d_records: this rank's counts[rank] x GPMPC_REC_LEN records (device, e.g.
 * gpmpc_fleet_records_dev); counts: every rank's shard size (host, nranks).
 * On the root, out (host) receives sum(counts) x GPMPC_REC_LEN doubles in
 * rank order; elsewhere out may be NULL.  Collective: every rank calls it.
 * = gpmpc_gather_prepare + gpmpc_gather_collective. */
int gpmpc_gather_results(gpmpc_ctx *ctx, gpmpc_comm *c, const double *d_records, const int *counts, int root,
                         double *out);
/* The same gather in two steps, so that the ranks can agree in between: prepare is
 * local (argument checks, send/receive buffers, the device padding of the ragged
 * block; the stream is drained before it returns), so every failure a rank can
 * meet alone is reported by it; collective issues only the ncclGather and the
 * root's compaction, and fails with -2 unless prepare succeeded since the last
 * collective with the same counts and root (the buffers were sized and padded for
 * them; a call with other arguments leaves the prepared block for the right one).  Agree on every rank's prepare status before any rank calls
 * collective (sharding.gather_shard_records does, with one all-reduce). */
int gpmpc_gather_prepare(gpmpc_ctx *ctx, gpmpc_comm *c, const double *d_records, const int *counts, int root);
int gpmpc_gather_collective(gpmpc_ctx *ctx, gpmpc_comm *c, const int *counts, int root, double *out);
int gpmpc_fleet_destroy(gpmpc_fleet *f);

#ifdef __cplusplus
}
#endif
#endif /* GPMPC_H */
