"""numpy restatement of the OSQP 0.6 ADMM solve (TEST INFRASTRUCTURE ONLY).

The reference (src/mpc/osqp_rti.py:454-567) drives the third-party ``osqp``
package (declared ``osqp>=0.6.0``, requirements.txt:9).  Its C sources are not
under /root/reference and the package is not installed, so the behaviour below
is restated from Stellato et al. 2020 (cited at osqp_rti.py:16-17) and the OSQP
0.6 C sources as published (scaling.c scale_data, auxil.c update_* /
compute_*_res / check_termination / is_*_infeasible, osqp.c osqp_solve /
osqp_update_rho).  Parity against OSQP itself is therefore *unpinned*; this
module is the parity oracle for the HIP ADMM.

Solver settings pinned by the reference (osqp_rti.py:54-60): max_iter=50,
eps_abs=eps_rel=1e-4, polish off, warm_start on, scaling=3.  OSQP defaults
(not passed by the reference) are pinned explicitly: rho=0.1, sigma=1e-6,
alpha=1.6, adaptive_rho on with tolerance 5 and a FIXED interval of 25
(OSQP's profiling builds choose it from wall time),
check_termination=25, eps_prim_inf=eps_dual_inf=1e-4, scaled_termination off.

The linear system is the quasi-definite KKT matrix
[[P + sigma I, A^T], [A, -diag(rho)^-1]] solved by a dense LU here (QDLDL's
LDL^T in OSQP); z_tilde is formed exactly as OSQP's QDLDL solve does.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.linalg as la
import scipy.sparse as sp

OSQP_INFTY = 1e30
MIN_SCALING, MAX_SCALING = 1e-4, 1e4
RHO_MIN, RHO_MAX, RHO_TOL, RHO_EQ_OVER_RHO_INEQ = 1e-6, 1e6, 1e-4, 1e3
DIVISION_TOL = 1.0 / OSQP_INFTY

SOLVED, SOLVED_INACCURATE, MAX_ITER_REACHED = 1, 2, -2
PRIMAL_INFEASIBLE, PRIMAL_INFEASIBLE_INACCURATE = -3, 3
DUAL_INFEASIBLE, DUAL_INFEASIBLE_INACCURATE = -4, 4
NON_CVX, UNSOLVED = -7, -10
STATUS_STRINGS = {
    SOLVED: "solved", SOLVED_INACCURATE: "solved inaccurate",
    MAX_ITER_REACHED: "maximum iterations reached", PRIMAL_INFEASIBLE: "primal infeasible",
    PRIMAL_INFEASIBLE_INACCURATE: "primal infeasible inaccurate",
    DUAL_INFEASIBLE: "dual infeasible", DUAL_INFEASIBLE_INACCURATE: "dual infeasible inaccurate",
    NON_CVX: "problem non convex", UNSOLVED: "unsolved",
}


@dataclass
class Settings:
    rho: float = 0.1
    sigma: float = 1e-6
    alpha: float = 1.6
    eps_abs: float = 1e-4
    eps_rel: float = 1e-4
    eps_prim_inf: float = 1e-4
    eps_dual_inf: float = 1e-4
    max_iter: int = 50
    check_termination: int = 25
    adaptive_rho: bool = True
    adaptive_rho_interval: int = 25
    adaptive_rho_tolerance: float = 5.0
    scaling: int = 3
    warm_start: bool = True


def _limit(v):
    v = np.where(v < MIN_SCALING, 1.0, v)
    return np.where(v > MAX_SCALING, MAX_SCALING, v)


def _colnorm_inf(M):
    M = sp.csc_matrix(M)
    return np.asarray(abs(M).max(axis=0).todense()).ravel()


def _rownorm_inf(M):
    M = sp.csr_matrix(M)
    return np.asarray(abs(M).max(axis=1).todense()).ravel()


def scale_data(P, q, A, l, u, iters):
    """Ruiz equilibration + cost scaling (OSQP scaling.c scale_data)."""
    P = sp.csc_matrix(P, dtype=float).copy(); A = sp.csc_matrix(A, dtype=float).copy()
    q = q.astype(float).copy()
    n, m = P.shape[0], A.shape[0]
    D = np.ones(n); E = np.ones(m); c = 1.0
    for _ in range(iters):
        dt = np.maximum(_colnorm_inf(P), _colnorm_inf(A))   # P stored full (symmetric)
        et = _rownorm_inf(A)
        dt = 1.0 / np.sqrt(_limit(dt)); et = 1.0 / np.sqrt(_limit(et))
        P = sp.diags(dt) @ P @ sp.diags(dt)
        A = sp.diags(et) @ A @ sp.diags(dt)
        q = dt * q
        D = D * dt; E = E * et
        ct = np.mean(_colnorm_inf(P))
        nq = float(_limit(np.array([np.max(np.abs(q))]))[0])
        ct = float(_limit(np.array([max(ct, nq)]))[0])
        ct = 1.0 / ct
        P = P * ct; q = q * ct; c *= ct
    return sp.csc_matrix(P), q, sp.csc_matrix(A), E * l, E * u, D, E, c


class OSQPOracle:
    """One OSQP workspace: setup once, then per-RTI-step ``update`` + ``warm_start`` + ``solve``.

    Every ``update`` re-derives the scaling from the new unscaled data (OSQP does
    unscale_data + scale_data inside osqp_update_A; the only difference is the
    1-ulp rounding of that unscale/rescale round trip).  The dual iterate y is
    kept in scaled form across solves, as OSQP keeps work->y.
    """

    def __init__(self, P, q, A, l, u, settings: Settings | None = None):
        self.s = settings or Settings()
        self.rho = self.s.rho
        n, m = P.shape[0], A.shape[0]
        self.n, self.m = n, m
        self.x = np.zeros(n); self.y = np.zeros(m); self.z = np.zeros(m)
        self._load(P, q, A, l, u)

    # -- data ------------------------------------------------------------
    def _load(self, P, q, A, l, u):
        l = np.maximum(np.asarray(l, float), -OSQP_INFTY)
        u = np.minimum(np.asarray(u, float), OSQP_INFTY)
        self.P, self.q, self.A, self.l, self.u, self.D, self.E, self.c = scale_data(
            sp.csc_matrix(P), np.asarray(q, float), sp.csc_matrix(A), l, u, self.s.scaling)
        self._set_rho_vec()

    def _set_rho_vec(self):
        self.rho = min(max(self.rho, RHO_MIN), RHO_MAX)
        loose = (self.l < -OSQP_INFTY * MIN_SCALING) & (self.u > OSQP_INFTY * MIN_SCALING)
        eq = (~loose) & (self.u - self.l < RHO_TOL)
        self.rho_vec = np.where(loose, RHO_MIN, np.where(eq, RHO_EQ_OVER_RHO_INEQ * self.rho, self.rho))
        self.loose = loose
        self._factor()

    def _factor(self):
        n = self.n
        Pd = self.P.toarray(); Ad = self.A.toarray()
        K = np.block([[Pd + self.s.sigma * np.eye(n), Ad.T], [Ad, -np.diag(1.0 / self.rho_vec)]])
        self.lu = la.lu_factor(K)

    def update(self, P, q, A, l, u):
        self._load(P, q, A, l, u)

    def warm_start_x(self, x):
        self.x = np.asarray(x, float) / self.D
        self.z = self.A @ self.x

    # -- residuals (auxil.c) ----------------------------------------------
    def _info(self, x, y, z):
        Ax = self.A @ x
        Px = self.P @ x
        Aty = self.A.T @ y
        self.Ax, self.Px, self.Aty = Ax, Px, Aty
        self.pri_vec = Ax - z
        self.dua_vec = self.q + Px + Aty
        pri = np.max(np.abs(self.pri_vec / self.E))
        dua = np.max(np.abs(self.dua_vec / self.D)) / self.c
        return pri, dua

    def _pri_tol(self, ea, er):
        return ea + er * max(np.max(np.abs(self.z / self.E)), np.max(np.abs(self.Ax / self.E)))

    def _dua_tol(self, ea, er):
        mx = max(np.max(np.abs(self.q / self.D)), np.max(np.abs(self.Aty / self.D)),
                 np.max(np.abs(self.Px / self.D)))
        return ea + er * mx / self.c

    def _primal_infeasible(self, eps):
        """auxil.c is_primal_infeasible: project delta_y onto the polar of the recession
        cone of [l,u], then u'max(dy,0) + l'min(dy,0) < -eps|dy| and |A'dy| < eps|dy|
        (Stellato et al. 2020, eq. (9)); norms unscaled."""
        dy = self.delta_y
        big_u = self.u > OSQP_INFTY * MIN_SCALING
        big_l = self.l < -OSQP_INFTY * MIN_SCALING
        dy = np.where(big_u & big_l, 0.0, np.where(big_u, np.minimum(dy, 0.0),
                                                   np.where(big_l, np.maximum(dy, 0.0), dy)))
        nrm = np.max(np.abs(self.E * dy))
        if nrm > DIVISION_TOL:
            lhs = np.sum(self.u * np.maximum(dy, 0.0) + self.l * np.minimum(dy, 0.0))
            if lhs < -eps * nrm:
                return np.max(np.abs((self.A.T @ dy) / self.D)) < eps * nrm
        return False

    def _dual_infeasible(self, eps):
        dx = self.delta_x
        nrm = np.max(np.abs(self.D * dx))
        if nrm > DIVISION_TOL:
            if np.dot(self.q, dx) < self.c * eps * nrm:
                if np.max(np.abs((self.P @ dx) / self.D)) < self.c * eps * nrm:
                    Adx = (self.A @ dx) / self.E
                    fin_u = self.u < OSQP_INFTY * MIN_SCALING
                    fin_l = self.l > -OSQP_INFTY * MIN_SCALING
                    bad = (fin_u & (Adx > eps * nrm)) | (fin_l & (Adx < -eps * nrm))
                    return not bool(np.any(bad))
        return False

    def _check(self, approx):
        s = self.s
        ea, er, epi, edi = s.eps_abs, s.eps_rel, s.eps_prim_inf, s.eps_dual_inf
        if self.pri > OSQP_INFTY or self.dua > OSQP_INFTY:
            self.status = NON_CVX
            return True
        if approx:
            ea, er, epi, edi = 10 * ea, 10 * er, 10 * epi, 10 * edi
        prim_ok = prim_inf = dual_ok = dual_inf = False
        if self.pri < self._pri_tol(ea, er):
            prim_ok = True
        else:
            prim_inf = self._primal_infeasible(epi)
        if self.dua < self._dua_tol(ea, er):
            dual_ok = True
        else:
            dual_inf = self._dual_infeasible(edi)
        if prim_ok and dual_ok:
            self.status = SOLVED_INACCURATE if approx else SOLVED
            return True
        if prim_inf:
            self.status = PRIMAL_INFEASIBLE_INACCURATE if approx else PRIMAL_INFEASIBLE
            return True
        if dual_inf:
            self.status = DUAL_INFEASIBLE_INACCURATE if approx else DUAL_INFEASIBLE
            return True
        return False

    def _adapt_rho(self):
        pri = np.max(np.abs(self.pri_vec)) / (max(np.max(np.abs(self.z)), np.max(np.abs(self.Ax))) + 1e-10)
        dua = np.max(np.abs(self.dua_vec)) / (max(np.max(np.abs(self.q)), np.max(np.abs(self.Aty)),
                                                  np.max(np.abs(self.Px))) + 1e-10)
        new = self.rho * np.sqrt(pri / (dua + 1e-10))
        new = min(max(new, RHO_MIN), RHO_MAX)
        self.rho_estimate = new
        if new > self.rho * self.s.adaptive_rho_tolerance or new < self.rho / self.s.adaptive_rho_tolerance:
            self.rho = new
            self._set_rho_vec()
            self.rho_updates += 1

    # -- solve (osqp.c osqp_solve) -----------------------------------------
    def solve(self):
        s = self.s; n = self.n
        if not s.warm_start:
            self.x[:] = 0; self.y[:] = 0; self.z[:] = 0
        self.status = UNSOLVED; self.rho_updates = 0
        can_check = False
        it = 0
        for it in range(1, s.max_iter + 1):
            xp, zp = self.x, self.z
            rhs = np.concatenate([s.sigma * xp - self.q, zp - self.y / self.rho_vec])
            sol = la.lu_solve(self.lu, rhs)
            xt = sol[:n]
            zt = rhs[n:] + sol[n:] / self.rho_vec
            x = s.alpha * xt + (1 - s.alpha) * xp
            self.delta_x = x - xp
            zr = s.alpha * zt + (1 - s.alpha) * zp
            z = np.minimum(np.maximum(zr + self.y / self.rho_vec, self.l), self.u)
            self.delta_y = self.rho_vec * (zr - z)
            self.y = self.y + self.delta_y
            self.x, self.z = x, z
            can_check = s.check_termination and it % s.check_termination == 0
            if can_check:
                self.iter = it
                self.pri, self.dua = self._info(self.x, self.y, self.z)
                if self._check(False):
                    break
            if s.adaptive_rho and s.adaptive_rho_interval and it % s.adaptive_rho_interval == 0:
                if not can_check:
                    self.iter = it
                    self.pri, self.dua = self._info(self.x, self.y, self.z)
                self._adapt_rho()
        if not can_check:
            self.iter = it
            self.pri, self.dua = self._info(self.x, self.y, self.z)
            self._check(False)
        if self.status == UNSOLVED:
            if not self._check(True):
                self.status = MAX_ITER_REACHED
        has_sol = self.status in (SOLVED, SOLVED_INACCURATE, MAX_ITER_REACHED)
        xbar = self.x
        self.obj_val = (0.5 * xbar @ (self.P @ xbar) + self.q @ xbar) / self.c if has_sol else np.nan
        if has_sol:
            x_out = self.D * self.x
            y_out = self.E * self.y / self.c
        else:
            x_out = np.full(n, np.nan); y_out = np.full(self.m, np.nan)
        return dict(x=x_out, y=y_out, status=self.status, status_str=STATUS_STRINGS[self.status],
                    iter=self.iter, obj_val=self.obj_val, rho=self.rho, pri_res=self.pri, dua_res=self.dua)
