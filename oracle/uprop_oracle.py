"""numpy restatement of the reference's linear uncertainty propagation
(TEST INFRASTRUCTURE ONLY).

UncertaintyPropagator._propagate_linear, uncertainty_prop.py:117-177:

    x_{k+1} = step(x_k, u_k) + dt * d(x_k, u_k)        on the residual rows
    Sigma_{k+1} = A_k Sigma_k A_k^T + diag(var(x_k, u_k) * dt^2)

with the residual rows 4:7 (v-dot) and, for the 14-state model, 11:14
(omega-dot).  Pinned to the reference's own output in
tests/golden/f9_uncertainty_prop.npz.
"""
from __future__ import annotations

import numpy as np

from . import gp_oracle


def propagate_linear(dynamics, gp_predict, x0, U, Sigma_0=None, dt=0.1):
    """uncertainty_prop.py:117-177.  gp_predict(x, u) -> (d_v, d_w, var_v, var_w)
    with d_w / var_w None for a 3-DoF (velocity-only) GP."""
    x0 = np.asarray(x0, float); U = np.atleast_2d(np.asarray(U, float))
    n, N = x0.size, len(U)
    S = np.eye(n) * 1e-6 if Sigma_0 is None else np.array(Sigma_0, float)
    means = np.zeros((N + 1, n)); covs = np.zeros((N + 1, n, n))
    means[0] = x0; covs[0] = S
    x = x0.copy()
    for k in range(N):
        A, _ = dynamics.linearize(x, U[k], dt=dt)
        d_v, d_w, var_v, var_w = gp_predict(x, U[k])
        Q = np.zeros((n, n))
        Q[4:7, 4:7] = np.diag(var_v) * dt ** 2
        xn = dynamics.step(x, U[k], dt).copy()
        xn[4:7] += d_v * dt
        if d_w is not None:
            Q[11:14, 11:14] = np.diag(var_w) * dt ** 2
            xn[11:14] += d_w * dt
        S = A @ S @ A.T + Q                       # uncertainty_prop.py:167
        means[k + 1] = xn; covs[k + 1] = S
        x = xn
    return means, covs


def structured_exact_predictor(X, U, Dv, Dw, noise=1e-4):
    """StructuredRocketGP(use_sparse=False) fit on (X, U, Dv, Dw) as a gp_predict
    callable (structured_gp.py:206-268 over exact_gp.py:118-268)."""
    sv = gp_oracle.exact_fit(gp_oracle.features_translational(X, U), Dv, noise=noise)
    sw = gp_oracle.exact_fit(gp_oracle.features_rotational(X, U), Dw, noise=noise)

    def predict(x, u):
        x = np.atleast_2d(x); u = np.atleast_2d(u)
        mv, vv = gp_oracle.exact_predict(sv, gp_oracle.features_translational(x, u))
        mw, vw = gp_oracle.exact_predict(sw, gp_oracle.features_rotational(x, u))
        return mv[0], mw[0], vv[0], vw[0]
    return predict


def simple3dof_exact_predictor(X, U, D, noise=1e-4):
    """Simple3DoFGP(use_sparse=False) as a gp_predict callable (velocity residual only)."""
    st = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D, noise=noise)

    def predict(x, u):
        m, v = gp_oracle.exact_predict(st, gp_oracle.features_3dof(np.atleast_2d(x), np.atleast_2d(u)))
        return m[0], None, v[0], None
    return predict
