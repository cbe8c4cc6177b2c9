/*
 * admm_ref.c -- plain-C restatement of the OSQP 0.6 ADMM (TEST INFRASTRUCTURE /
 * CPU BASELINE ONLY; never linked into the product).
 *
 * Same algorithm as oracle/admm_oracle.py (see its header for the OSQP
 * behaviour pinned and why parity against OSQP itself is unpinned), written
 * the way the reference's hot loop would run on a CPU core: sequential,
 * fp64, with the KKT system eliminated to the reduced (normal-equation) form
 *     (P + sigma I + A' diag(rho) A) x~ = sigma x - q + A'(rho z - y),   z~ = A x~
 * which is algebraically identical to OSQP's quasi-definite KKT solve.  The
 * reduced matrix of an MPC QP is banded, so it is factored by a banded
 * Cholesky (LAPACK dpbtrf-style, row oriented).  Compiled with
 * -ffp-contract=off so every product and sum rounds as written.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define OSQP_INFTY 1e30
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_TOL 1e-4
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define DIVISION_TOL (1.0 / OSQP_INFTY)

enum { SOLVED = 1, SOLVED_INACCURATE = 2, MAX_ITER_REACHED = -2, PRIMAL_INFEASIBLE = -3,
       PRIMAL_INFEASIBLE_INACCURATE = 3, DUAL_INFEASIBLE = -4, DUAL_INFEASIBLE_INACCURATE = 4,
       NON_CVX = -7, UNSOLVED = -10 };

typedef struct {
  double rho, sigma, alpha;
  double eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
  int max_iter, check_termination, adaptive_rho, adaptive_rho_interval;
  double adaptive_rho_tolerance;
  int scaling, warm_start;
} ref_settings;

typedef struct {
  int n, m, nnz, w;
  const int *rp, *ci;
  double *A, *P, *q, *l, *u, *D, *E, c;
  double *rho, *x, *y, *z, *xt, *zt, *dx, *dy, *rhs, *Ax, *Px, *Aty, *tmp, *adx, *band;
  double rho_s;
  double pri, dua;
  int status, iter;
} ws_t;

static double dmax(double a, double b) { return a > b ? a : b; }
static double dmin(double a, double b) { return a < b ? a : b; }
static double limit(double v) {
  if (v < MIN_SCALING) v = 1.0;
  if (v > MAX_SCALING) v = MAX_SCALING;
  return v;
}
static double norm_inf(const double *v, int k) {
  double r = 0.0;
  for (int i = 0; i < k; ++i) r = dmax(r, fabs(v[i]));
  return r;
}
static double scaled_norm_inf(const double *s, const double *v, int k) { /* |s.*v| */
  double r = 0.0;
  for (int i = 0; i < k; ++i) r = dmax(r, fabs(s[i] * v[i]));
  return r;
}
static double inv_scaled_norm_inf(const double *s, const double *v, int k) { /* |v./s| */
  double r = 0.0;
  for (int i = 0; i < k; ++i) r = dmax(r, fabs(v[i] / s[i]));
  return r;
}
static void spmv(const ws_t *w, const double *x, double *out) { /* out = A x */
  for (int r = 0; r < w->m; ++r) {
    double s = 0.0;
    for (int k = w->rp[r]; k < w->rp[r + 1]; ++k) s += w->A[k] * x[w->ci[k]];
    out[r] = s;
  }
}
static void spmv_t(const ws_t *w, const double *y, double *out) { /* out = A' y */
  memset(out, 0, sizeof(double) * w->n);
  for (int r = 0; r < w->m; ++r)
    for (int k = w->rp[r]; k < w->rp[r + 1]; ++k) out[w->ci[k]] += w->A[k] * y[r];
}

/* scaling.c scale_data: Ruiz on [[P A'],[A 0]] + cost scaling */
static void scale_data(ws_t *w, int iters) {
  int n = w->n, m = w->m;
  for (int j = 0; j < n; ++j) w->D[j] = 1.0;
  for (int i = 0; i < m; ++i) w->E[i] = 1.0;
  w->c = 1.0;
  double *dt = w->tmp, *et = w->zt; /* scratch */
  for (int it = 0; it < iters; ++it) {
    for (int j = 0; j < n; ++j) dt[j] = fabs(w->P[j]);
    for (int r = 0; r < m; ++r) {
      double rn = 0.0;
      for (int k = w->rp[r]; k < w->rp[r + 1]; ++k) {
        double a = fabs(w->A[k]);
        rn = dmax(rn, a);
        dt[w->ci[k]] = dmax(dt[w->ci[k]], a);
      }
      et[r] = rn;
    }
    for (int j = 0; j < n; ++j) dt[j] = 1.0 / sqrt(limit(dt[j]));
    for (int r = 0; r < m; ++r) et[r] = 1.0 / sqrt(limit(et[r]));
    for (int j = 0; j < n; ++j) w->P[j] = dt[j] * w->P[j] * dt[j];
    for (int r = 0; r < m; ++r)
      for (int k = w->rp[r]; k < w->rp[r + 1]; ++k) w->A[k] = et[r] * w->A[k] * dt[w->ci[k]];
    for (int j = 0; j < n; ++j) w->q[j] = dt[j] * w->q[j];
    for (int j = 0; j < n; ++j) w->D[j] *= dt[j];
    for (int r = 0; r < m; ++r) w->E[r] *= et[r];
    double s = 0.0;
    for (int j = 0; j < n; ++j) s += fabs(w->P[j]);
    double ct = s / n;
    double nq = limit(norm_inf(w->q, n));
    ct = limit(dmax(ct, nq));
    ct = 1.0 / ct;
    for (int j = 0; j < n; ++j) w->P[j] *= ct;
    for (int j = 0; j < n; ++j) w->q[j] *= ct;
    w->c *= ct;
  }
  for (int r = 0; r < m; ++r) {
    w->l[r] = w->E[r] * w->l[r];
    w->u[r] = w->E[r] * w->u[r];
  }
}

static void set_rho_vec(ws_t *w) {
  w->rho_s = dmin(dmax(w->rho_s, RHO_MIN), RHO_MAX);
  for (int r = 0; r < w->m; ++r) {
    if (w->l[r] < -OSQP_INFTY * MIN_SCALING && w->u[r] > OSQP_INFTY * MIN_SCALING)
      w->rho[r] = RHO_MIN;
    else if (w->u[r] - w->l[r] < RHO_TOL)
      w->rho[r] = RHO_EQ_OVER_RHO_INEQ * w->rho_s;
    else
      w->rho[r] = w->rho_s;
  }
}

/* band[i*(w+1) + (i-j)] = M[i][j] / L[i][j] for j in [i-w, i] */
#define BAND(i, j) w->band[(size_t)(i) * (w->w + 1) + ((i) - (j))]
static int factor(ws_t *w, double sigma) {
  int n = w->n, bw = w->w;
  memset(w->band, 0, sizeof(double) * (size_t)n * (bw + 1));
  for (int j = 0; j < n; ++j) BAND(j, j) = w->P[j] + sigma;
  for (int r = 0; r < w->m; ++r)
    for (int a = w->rp[r]; a < w->rp[r + 1]; ++a)
      for (int b = w->rp[r]; b < w->rp[r + 1]; ++b) {
        int i = w->ci[a], j = w->ci[b];
        if (j > i) continue;
        BAND(i, j) += w->rho[r] * w->A[a] * w->A[b];
      }
  for (int i = 0; i < n; ++i) {
    int j0 = i - bw < 0 ? 0 : i - bw;
    for (int j = j0; j <= i; ++j) {
      double s = BAND(i, j);
      int k0 = (j - bw > j0) ? j - bw : j0;
      for (int k = k0; k < j; ++k) s -= BAND(i, k) * BAND(j, k);
      if (j < i) BAND(i, j) = s / BAND(j, j);
      else {
        if (!(s > 0.0)) return i + 1;
        BAND(i, i) = sqrt(s);
      }
    }
  }
  return 0;
}
static void band_solve(ws_t *w, double *b) { /* b <- M^-1 b */
  int n = w->n, bw = w->w;
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    int k0 = i - bw < 0 ? 0 : i - bw;
    for (int k = k0; k < i; ++k) s -= BAND(i, k) * b[k];
    b[i] = s / BAND(i, i);
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    int k1 = i + bw > n - 1 ? n - 1 : i + bw;
    for (int k = i + 1; k <= k1; ++k) s -= BAND(k, i) * b[k];
    b[i] = s / BAND(i, i);
  }
}
#undef BAND

static void update_info(ws_t *w) {
  spmv(w, w->x, w->Ax);
  for (int j = 0; j < w->n; ++j) w->Px[j] = w->P[j] * w->x[j];
  spmv_t(w, w->y, w->Aty);
  double pr = 0.0, du = 0.0;
  for (int r = 0; r < w->m; ++r) pr = dmax(pr, fabs((w->Ax[r] - w->z[r]) / w->E[r]));
  for (int j = 0; j < w->n; ++j) du = dmax(du, fabs((w->q[j] + w->Px[j] + w->Aty[j]) / w->D[j]));
  w->pri = pr;
  w->dua = du / w->c;
}

static int primal_infeasible(ws_t *w, double eps) {
  int m = w->m;
  double *dy = w->zt; /* projected copy */
  for (int r = 0; r < m; ++r) {
    double v = w->dy[r];
    int bu = w->u[r] > OSQP_INFTY * MIN_SCALING, bl = w->l[r] < -OSQP_INFTY * MIN_SCALING;
    if (bu && bl) v = 0.0;
    else if (bu) v = dmin(v, 0.0);
    else if (bl) v = dmax(v, 0.0);
    dy[r] = v;
  }
  double nrm = scaled_norm_inf(w->E, dy, m);
  if (nrm > DIVISION_TOL) {
    double lhs = 0.0;
    for (int r = 0; r < m; ++r) lhs += w->u[r] * dmax(dy[r], 0.0) + w->l[r] * dmin(dy[r], 0.0);
    if (lhs < -eps * nrm) {
      spmv_t(w, dy, w->tmp);
      return inv_scaled_norm_inf(w->D, w->tmp, w->n) < eps * nrm;
    }
  }
  return 0;
}

static int dual_infeasible(ws_t *w, double eps) {
  int n = w->n, m = w->m;
  double nrm = scaled_norm_inf(w->D, w->dx, n);
  if (nrm > DIVISION_TOL) {
    double qdx = 0.0;
    for (int j = 0; j < n; ++j) qdx += w->q[j] * w->dx[j];
    if (qdx < w->c * eps * nrm) {
      double pn = 0.0;
      for (int j = 0; j < n; ++j) pn = dmax(pn, fabs(w->P[j] * w->dx[j] / w->D[j]));
      if (pn < w->c * eps * nrm) {
        spmv(w, w->dx, w->adx);
        for (int r = 0; r < m; ++r) {
          double v = w->adx[r] / w->E[r];
          if ((w->u[r] < OSQP_INFTY * MIN_SCALING && v > eps * nrm) ||
              (w->l[r] > -OSQP_INFTY * MIN_SCALING && v < -eps * nrm))
            return 0;
        }
        return 1;
      }
    }
  }
  return 0;
}

static double pri_tol(ws_t *w, double ea, double er) {
  return ea + er * dmax(inv_scaled_norm_inf(w->E, w->z, w->m), inv_scaled_norm_inf(w->E, w->Ax, w->m));
}
static double dua_tol(ws_t *w, double ea, double er) {
  double mx = inv_scaled_norm_inf(w->D, w->q, w->n);
  mx = dmax(mx, inv_scaled_norm_inf(w->D, w->Aty, w->n));
  mx = dmax(mx, inv_scaled_norm_inf(w->D, w->Px, w->n));
  return ea + er * mx / w->c;
}

/* auxil.c check_termination */
static int check_termination(ws_t *w, const ref_settings *s, int approx) {
  double ea = s->eps_abs, er = s->eps_rel, epi = s->eps_prim_inf, edi = s->eps_dual_inf;
  if (w->pri > OSQP_INFTY || w->dua > OSQP_INFTY) { w->status = NON_CVX; return 1; }
  if (approx) { ea *= 10; er *= 10; epi *= 10; edi *= 10; }
  int prim_ok = 0, prim_inf = 0, dual_ok = 0, dual_inf = 0;
  if (w->pri < pri_tol(w, ea, er)) prim_ok = 1;
  else prim_inf = primal_infeasible(w, epi);
  if (w->dua < dua_tol(w, ea, er)) dual_ok = 1;
  else dual_inf = dual_infeasible(w, edi);
  if (prim_ok && dual_ok) { w->status = approx ? SOLVED_INACCURATE : SOLVED; return 1; }
  if (prim_inf) { w->status = approx ? PRIMAL_INFEASIBLE_INACCURATE : PRIMAL_INFEASIBLE; return 1; }
  if (dual_inf) { w->status = approx ? DUAL_INFEASIBLE_INACCURATE : DUAL_INFEASIBLE; return 1; }
  return 0;
}

/* auxil.c compute_rho_estimate / adapt_rho (residuals in the scaled space) */
static int adapt_rho(ws_t *w, const ref_settings *s) {
  double pr = 0.0, du = 0.0;
  for (int r = 0; r < w->m; ++r) pr = dmax(pr, fabs(w->Ax[r] - w->z[r]));
  for (int j = 0; j < w->n; ++j) du = dmax(du, fabs(w->q[j] + w->Px[j] + w->Aty[j]));
  double pn = dmax(norm_inf(w->z, w->m), norm_inf(w->Ax, w->m));
  double dn = dmax(dmax(norm_inf(w->q, w->n), norm_inf(w->Aty, w->n)), norm_inf(w->Px, w->n));
  pr /= (pn + 1e-10);
  du /= (dn + 1e-10);
  double est = w->rho_s * sqrt(pr / (du + 1e-10));
  est = dmin(dmax(est, RHO_MIN), RHO_MAX);
  if (est > w->rho_s * s->adaptive_rho_tolerance || est < w->rho_s / s->adaptive_rho_tolerance) {
    w->rho_s = est;
    set_rho_vec(w);
    return factor(w, s->sigma) ? -1 : 1;
  }
  return 0;
}

void ref_qp_default_settings(ref_settings *s) {
  s->rho = 0.1; s->sigma = 1e-6; s->alpha = 1.6;
  s->eps_abs = 1e-4; s->eps_rel = 1e-4; s->eps_prim_inf = 1e-4; s->eps_dual_inf = 1e-4;
  s->max_iter = 50; s->check_termination = 25; s->adaptive_rho = 1;
  s->adaptive_rho_interval = 25; s->adaptive_rho_tolerance = 5.0; s->scaling = 3;
  s->warm_start = 1;
}

/* One OSQP "update + warm_start(x) + solve" on fresh data.  rho_state and
 * y_state carry OSQP's persistent workspace values between calls (y scaled).
 * Returns 0, or -1 when the reduced KKT matrix is not positive definite. */
int ref_qp_solve(int n, int m, const int *rowptr, const int *colidx, const double *Aval,
                 const double *Pdiag, const double *q, const double *l, const double *u,
                 const ref_settings *s, const double *x_ws, double *rho_state, double *y_state,
                 double *x_out, double *y_out, int *iters, int *status, double *obj,
                 double *res /* [pri, dua] or NULL */) {
  ws_t W;
  ws_t *w = &W;
  memset(w, 0, sizeof(W));
  w->n = n; w->m = m; w->rp = rowptr; w->ci = colidx; w->nnz = rowptr[m];
  int bw = 0;
  for (int r = 0; r < m; ++r)
    for (int a = rowptr[r]; a < rowptr[r + 1]; ++a)
      for (int b = rowptr[r]; b < rowptr[r + 1]; ++b) {
        int d = colidx[a] - colidx[b];
        if (d > bw) bw = d;
      }
  w->w = bw;
  double *mem = (double *)calloc((size_t)w->nnz + 12 * (size_t)n + 12 * (size_t)m +
                                     (size_t)n * (bw + 1), sizeof(double));
  double *p = mem;
  w->A = p; p += w->nnz;
  w->P = p; p += n; w->q = p; p += n; w->D = p; p += n; w->x = p; p += n; w->xt = p; p += n;
  w->dx = p; p += n; w->rhs = p; p += n; w->Px = p; p += n; w->Aty = p; p += n; w->tmp = p; p += n;
  w->l = p; p += m; w->u = p; p += m; w->E = p; p += m; w->rho = p; p += m; w->y = p; p += m;
  w->z = p; p += m; w->zt = p; p += m; w->dy = p; p += m; w->Ax = p; p += m; w->adx = p; p += m;
  w->band = p;
  memcpy(w->A, Aval, sizeof(double) * w->nnz);
  memcpy(w->P, Pdiag, sizeof(double) * n);
  memcpy(w->q, q, sizeof(double) * n);
  for (int r = 0; r < m; ++r) {
    w->l[r] = dmax(l[r], -OSQP_INFTY);
    w->u[r] = dmin(u[r], OSQP_INFTY);
  }
  if (s->scaling) scale_data(w, s->scaling);
  else { for (int j = 0; j < n; ++j) w->D[j] = 1.0; for (int r = 0; r < m; ++r) w->E[r] = 1.0; w->c = 1.0; }
  w->rho_s = *rho_state;
  set_rho_vec(w);
  if (factor(w, s->sigma)) { free(mem); return -1; }
  if (s->warm_start) {
    for (int j = 0; j < n; ++j) w->x[j] = x_ws ? x_ws[j] / w->D[j] : 0.0;
    spmv(w, w->x, w->z);
    memcpy(w->y, y_state, sizeof(double) * m);
  }
  w->status = UNSOLVED;
  int can_check = 0, it = 0;
  for (it = 1; it <= s->max_iter; ++it) {
    /* rhs = sigma x - q + A'(rho z - y) */
    for (int r = 0; r < m; ++r) w->zt[r] = w->rho[r] * w->z[r] - w->y[r];
    spmv_t(w, w->zt, w->rhs);
    for (int j = 0; j < n; ++j) w->rhs[j] = s->sigma * w->x[j] - w->q[j] + w->rhs[j];
    band_solve(w, w->rhs); /* x~ */
    spmv(w, w->rhs, w->zt); /* z~ = A x~ */
    for (int j = 0; j < n; ++j) {
      double xn = s->alpha * w->rhs[j] + (1.0 - s->alpha) * w->x[j];
      w->dx[j] = xn - w->x[j];
      w->x[j] = xn;
    }
    for (int r = 0; r < m; ++r) {
      double zr = s->alpha * w->zt[r] + (1.0 - s->alpha) * w->z[r];
      double zn = zr + w->y[r] / w->rho[r];
      zn = dmin(dmax(zn, w->l[r]), w->u[r]);
      w->dy[r] = w->rho[r] * (zr - zn);
      w->y[r] += w->dy[r];
      w->z[r] = zn;
    }
    can_check = s->check_termination && (it % s->check_termination == 0);
    if (can_check) {
      w->iter = it;
      update_info(w);
      if (check_termination(w, s, 0)) break;
    }
    if (s->adaptive_rho && s->adaptive_rho_interval && (it % s->adaptive_rho_interval == 0)) {
      if (!can_check) { w->iter = it; update_info(w); }
      if (adapt_rho(w, s) < 0) { free(mem); return -1; }
    }
  }
  if (!can_check) {
    w->iter = it - 1;
    update_info(w);
    check_termination(w, s, 0);
  }
  if (w->status == UNSOLVED && !check_termination(w, s, 1)) w->status = MAX_ITER_REACHED;
  int has_sol = (w->status == SOLVED || w->status == SOLVED_INACCURATE || w->status == MAX_ITER_REACHED);
  double ob = 0.0;
  for (int j = 0; j < n; ++j) ob += 0.5 * w->x[j] * (w->P[j] * w->x[j]) + w->q[j] * w->x[j];
  *obj = has_sol ? ob / w->c : NAN;
  for (int j = 0; j < n; ++j) x_out[j] = has_sol ? w->D[j] * w->x[j] : NAN;
  for (int r = 0; r < m; ++r) y_out[r] = has_sol ? w->E[r] * w->y[r] / w->c : NAN;
  memcpy(y_state, w->y, sizeof(double) * m);
  *rho_state = w->rho_s;
  *iters = w->iter;
  *status = w->status;
  if (res) { res[0] = w->pri; res[1] = w->dua; }
  free(mem);
  return 0;
}
