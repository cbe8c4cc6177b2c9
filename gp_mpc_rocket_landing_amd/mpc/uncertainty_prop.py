"""Uncertainty propagation for GP-MPC (reference src/mpc/uncertainty_prop.py).

Same classes, arguments and results as the reference:

* ``UncertaintyPropagator`` -- linear (uncertainty_prop.py:117-177), unscented
  (:179-264) and Monte-Carlo (:266-315) propagation of the state distribution
  along a control sequence, with the GP variance as process noise;
* ``ConstraintTightening`` (:318-411) and ``TubeBasedRobustness`` (:414-468).

The linear method is the one GPMPC calls (gp_mpc.py:284-290, 348-353).  Its
mean recursion needs one GP evaluation per horizon step -- a device call,
batched over trajectories in ``propagate_batch`` -- and its covariance
recursion Sigma_{k+1} = A_k Sigma_k A_k^T + Q_k runs for every trajectory in
one launch of the device kernel (``gpmpc_cov_propagate``, csrc/uprop.hip).

Both model shapes work: the reference's 14-state 6-DoF model with a 4-tuple GP
(StructuredRocketGP: residuals on v-dot 4:7 and omega-dot 11:14), and the
7-state 3-DoF model with a 2-tuple GP (Simple3DoFGP: residual on v-dot only).
The reference hard-codes n_x = 14 (uncertainty_prop.py:87); here n_x is the
dynamics' ``n_state`` (default 14).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

import numpy as np

from .. import _lib


@dataclass
class PropagatedUncertainty:
    """uncertainty_prop.py:35-55."""
    means: np.ndarray        # (N+1, n_x)
    covariances: np.ndarray  # (N+1, n_x, n_x)

    def get_std(self, k: int) -> np.ndarray:
        return np.sqrt(np.diag(self.covariances[k]))

    def get_confidence_bounds(self, k: int, confidence: float = 0.95) -> Tuple[np.ndarray, np.ndarray]:
        from scipy.stats import norm
        kappa = norm.ppf((1 + confidence) / 2)
        std = self.get_std(k)
        return self.means[k] - kappa * std, self.means[k] + kappa * std


def _gp_batch(gp, X, U):
    """GP residual mean/variance at P points -> (d_v, d_w, var_v, var_w); d_w and
    var_w are None for a 2-tuple (3-DoF) GP.  One device call when the GP has
    predict_batch."""
    X = np.atleast_2d(X); U = np.atleast_2d(U)
    if hasattr(gp, "predict_batch"):
        r = gp.predict_batch(X, U)
    else:
        rows = [gp.predict(X[i], U[i]) for i in range(X.shape[0])]
        r = tuple(np.array([row[j] for row in rows]) for j in range(len(rows[0])))
    if len(r) == 4:
        return (np.atleast_2d(r[0]), np.atleast_2d(r[1]), np.atleast_2d(r[2]), np.atleast_2d(r[3]))
    return np.atleast_2d(r[0]), None, np.atleast_2d(r[1]), None


class UncertaintyPropagator:
    """uncertainty_prop.py:58-315."""

    def __init__(self, dynamics, gp_model, method: str = "linear", ctx=None):
        self.dynamics = dynamics
        self.gp = gp_model
        self.method = method
        self.n_x = int(getattr(dynamics, "n_state", 14))
        self.n_u = 3
        self._ctx = ctx

    @property
    def ctx(self):
        return self._ctx or _lib.default_context()

    # residual rows of the state: v-dot, and omega-dot for the 14-state model
    def _rows(self):
        return (slice(4, 7), slice(11, 14)) if self.n_x == 14 else (slice(4, 7), None)

    def propagate(self, x0, U, Sigma_0=None, dt: float = 0.1) -> PropagatedUncertainty:
        """uncertainty_prop.py:91-115."""
        if self.method == "linear":
            return self._propagate_linear(x0, U, Sigma_0, dt)
        if self.method == "unscented":
            return self._propagate_unscented(x0, U, Sigma_0, dt)
        if self.method == "monte_carlo":
            return self._propagate_monte_carlo(x0, U, Sigma_0, dt)
        raise ValueError(f"Unknown method: {self.method}")

    # the whole linear propagation in one device call (gpmpc_uprop3_linear) for the 3-DoF
    # explicit-Euler model over the 3-DoF exact GP: the N sequential GP predictions of the
    # host loop below become one kernel; the same recursion, rounding aside
    use_device = True

    def _device_6dof(self, X0, U, Sigma_0, dt):
        """gpmpc_uprop6_linear for Rocket6DoFDynamics over a fitted StructuredRocketGP at its
        default feature set (the device features are features.py's at reference velocity
        10 with altitude and density), its residual groups each one shared device GP."""
        if not self.use_device or self.n_x != 14:
            return None
        from ..dynamics.rocket_6dof import Rocket6DoFDynamics
        from ..gp.structured_gp import StructuredRocketGP
        gp = self.gp
        if type(self.dynamics) is not Rocket6DoFDynamics or type(gp) is not StructuredRocketGP:
            return None
        c = gp.config
        if not (gp._is_fitted and c.reference_velocity == 10.0 and c.include_altitude and c.include_density):
            return None
        hv, hw = gp.gp_v.device_handle, gp.gp_omega.device_handle
        if hv is None or hw is None:
            return None
        p = self.dynamics.params
        rocket = np.concatenate([np.asarray(p.J_B, float).reshape(9), np.asarray(p.r_T_B, float).reshape(3),
                                 np.asarray(p.g_I, float).reshape(3),
                                 [float(p.alpha), float(p.g0)]])
        S0 = None
        if Sigma_0 is not None:
            S0 = np.broadcast_to(np.asarray(Sigma_0, float), (X0.shape[0], 14, 14))
        try:
            return _lib.uprop6_linear(self.ctx, hv, hw, not c.use_sparse, rocket, X0, U, S0, dt)
        except _lib.HIPError:
            return None   # (a composite-kernel GP: the host loop)

    def _device_3dof(self, X0, U, Sigma_0, dt):
        if not self.use_device or self.n_x != 7:
            return None
        from ..dynamics.rocket_3dof import Rocket3DoFDynamics
        from ..gp.exact_gp import MultiOutputExactGP
        from ..gp.features import Simple3DoFFeatureExtractor
        gp = self.gp
        inner = getattr(gp, "gp", None)
        # (only the exact GP's handle is a gpmpc_gp; a FITC handle is another type)
        if (type(self.dynamics) is not Rocket3DoFDynamics or not isinstance(inner, MultiOutputExactGP)
                or type(getattr(gp, "feature_extractor", None)) is not Simple3DoFFeatureExtractor
                or not getattr(gp, "_is_fitted", False)):
            return None
        h = inner.device_handle
        if h is None:
            return None
        p = self.dynamics.params
        S0 = None
        if Sigma_0 is not None:
            S0 = np.broadcast_to(np.asarray(Sigma_0, float), (X0.shape[0], 7, 7))
        try:
            return _lib.uprop3_linear(self.ctx, h, X0, U, S0, dt, float(p.alpha), np.asarray(p.g_vec, float))
        except _lib.HIPError:
            return None   # (a composite-kernel GP: the host loop)

    # ------------------------------------------------------------------ linear
    def _propagate_linear(self, x0, U, Sigma_0, dt) -> PropagatedUncertainty:
        """uncertainty_prop.py:117-177 for one trajectory (a batch of one)."""
        S0 = None if Sigma_0 is None else np.asarray(Sigma_0, float)[None]
        means, covs = self.propagate_batch(np.asarray(x0, float)[None], np.asarray(U, float)[None], S0, dt)
        return PropagatedUncertainty(means=means[0], covariances=covs[0])

    def propagate_batch(self, X0, U, Sigma_0=None, dt: float = 0.1):
        """Linear propagation of B trajectories at once.

        X0 (B, n_x), U (B, N, n_u), Sigma_0 None (the reference's 1e-6 I),
        (n_x, n_x) or (B, n_x, n_x) -> means (B, N+1, n_x), covariances
        (B, N+1, n_x, n_x).  Per horizon step: one batched GP evaluation on the
        device and the nominal step / Jacobian of every trajectory; then one
        device launch for all covariance recursions."""
        X0 = np.atleast_2d(np.asarray(X0, float)); U = np.asarray(U, float)
        if U.ndim == 2:
            U = U[None]
        B, N = U.shape[0], U.shape[1]
        nx = self.n_x
        if X0.shape != (B, nx):
            raise ValueError(f"X0 shape {X0.shape}, expected {(B, nx)}")
        dev = self._device_3dof(X0, U, Sigma_0, dt)
        if dev is None:
            dev = self._device_6dof(X0, U, Sigma_0, dt)
        if dev is not None:
            return dev
        rv, rw = self._rows()
        means = np.zeros((B, N + 1, nx)); means[:, 0] = X0
        A = np.zeros((B, N, nx, nx)); q = np.zeros((B, N, nx))
        x = X0.copy()
        for k in range(N):
            u = U[:, k]
            d_v, d_w, var_v, var_w = _gp_batch(self.gp, x, u)
            xn = np.empty_like(x)
            for b in range(B):
                A[b, k], _ = self.dynamics.linearize(x[b], u[b], dt=dt)
                xn[b] = self.dynamics.step(x[b], u[b], dt)
            xn[:, rv] += d_v * dt
            q[:, k, rv] = var_v * dt ** 2
            if rw is not None:
                xn[:, rw] += d_w * dt
                q[:, k, rw] = var_w * dt ** 2
            means[:, k + 1] = xn
            x = xn
        S0 = None
        if Sigma_0 is not None:
            S0 = np.asarray(Sigma_0, float)
            if S0.ndim == 2:
                S0 = np.broadcast_to(S0, (B, nx, nx))
        covs = _lib.cov_propagate(self.ctx, A, q, S0, 1e-6)
        return means, covs

    # --------------------------------------------------------------- unscented
    def _propagate_unscented(self, x0, U, Sigma_0, dt) -> PropagatedUncertainty:
        """uncertainty_prop.py:179-264; the 2n+1 sigma points and the mean point
        of a step go to the GP as one batch."""
        U = np.atleast_2d(np.asarray(U, float))
        N, n = len(U), self.n_x
        if Sigma_0 is None:
            Sigma_0 = np.eye(n) * 1e-6
        alpha, beta, kappa = 1e-3, 2, 0
        lam = alpha ** 2 * (n + kappa) - n
        w_m = np.full(2 * n + 1, 1 / (2 * (n + lam)))
        w_c = w_m.copy()
        w_m[0] = lam / (n + lam)
        w_c[0] = lam / (n + lam) + (1 - alpha ** 2 + beta)
        rv, rw = self._rows()
        means = np.zeros((N + 1, n)); covs = np.zeros((N + 1, n, n))
        means[0] = x0; covs[0] = Sigma_0
        x_k = np.array(x0, float); S_k = np.array(Sigma_0, float)
        for k in range(N):
            u_k = U[k]
            sq = np.linalg.cholesky((n + lam) * S_k + 1e-10 * np.eye(n))
            sp = np.zeros((2 * n + 1, n))
            sp[0] = x_k
            for i in range(n):
                sp[i + 1] = x_k + sq[:, i]
                sp[n + i + 1] = x_k - sq[:, i]
            pts = np.vstack([sp, x_k[None]])
            d_v, d_w, var_v, var_w = _gp_batch(self.gp, pts, np.broadcast_to(u_k, (len(pts), 3)))
            spn = np.array([self.dynamics.step(sp[i], u_k, dt) for i in range(2 * n + 1)])
            spn[:, rv] += d_v[:-1] * dt
            if rw is not None:
                spn[:, rw] += d_w[:-1] * dt
            x_next = np.sum(w_m[:, None] * spn, axis=0)
            S_next = np.zeros((n, n))
            for i in range(2 * n + 1):
                diff = spn[i] - x_next
                S_next += w_c[i] * np.outer(diff, diff)
            Q = np.zeros((n, n))
            Q[rv, rv] = np.diag(var_v[-1]) * dt ** 2
            if rw is not None:
                Q[rw, rw] = np.diag(var_w[-1]) * dt ** 2
            S_next += Q
            means[k + 1] = x_next; covs[k + 1] = S_next
            x_k, S_k = x_next, S_next
        return PropagatedUncertainty(means=means, covariances=covs)

    # ------------------------------------------------------------- Monte Carlo
    def _propagate_monte_carlo(self, x0, U, Sigma_0, dt, n_samples: int = 100) -> PropagatedUncertainty:
        """uncertainty_prop.py:266-315.  Draws from numpy's global RNG in the
        reference's order (per particle: 3 normals for d_v, then 3 for d_omega;
        the 3-DoF model draws only the d_v ones); the particles' GP evaluations
        are one batch per step."""
        U = np.atleast_2d(np.asarray(U, float))
        N, n = len(U), self.n_x
        if Sigma_0 is None:
            Sigma_0 = np.eye(n) * 1e-6
        rv, rw = self._rows()
        particles = np.random.multivariate_normal(x0, Sigma_0, n_samples)
        means = np.zeros((N + 1, n)); covs = np.zeros((N + 1, n, n))
        means[0] = x0; covs[0] = Sigma_0
        for k in range(N):
            u_k = U[k]
            d_v, d_w, var_v, var_w = _gp_batch(self.gp, particles, np.broadcast_to(u_k, (n_samples, 3)))
            nxt = np.array([self.dynamics.step(particles[i], u_k, dt) for i in range(n_samples)])
            z = np.random.randn(n_samples, 2 if rw is not None else 1, 3)
            nxt[:, rv] += (d_v + np.sqrt(var_v) * z[:, 0]) * dt
            if rw is not None:
                nxt[:, rw] += (d_w + np.sqrt(var_w) * z[:, 1]) * dt
            means[k + 1] = np.mean(nxt, axis=0)
            diff = nxt - means[k + 1]
            covs[k + 1] = (diff.T @ diff) / (n_samples - 1)
            particles = nxt
        return PropagatedUncertainty(means=means, covariances=covs)


class ConstraintTightening:
    """uncertainty_prop.py:318-411."""

    def __init__(self, confidence: float = 0.95):
        from scipy.stats import norm
        self.confidence = confidence
        self.kappa = norm.ppf(confidence)

    def tighten_linear_constraint(self, a, b: float, mu, Sigma) -> float:
        """a^T x >= b under x ~ N(mu, Sigma): returns b + kappa sqrt(a^T Sigma a)."""
        a = np.asarray(a, float)
        return b + self.kappa * np.sqrt(a.T @ np.asarray(Sigma, float) @ a)

    def tighten_quadratic_constraint(self, x_mu, x_Sigma, constraint_func: Callable, n_samples: int = 100) -> float:
        samples = np.random.multivariate_normal(x_mu, x_Sigma, n_samples)
        g = np.array([constraint_func(s) for s in samples])
        return np.percentile(g, (1 - self.confidence) * 100)

    def compute_back_offs(self, uncertainty: PropagatedUncertainty, constraint_gradients: List) -> np.ndarray:
        N = len(uncertainty.means) - 1
        n_c = len(constraint_gradients[0]) if constraint_gradients else 0
        back = np.zeros((N, n_c))
        for k in range(N):
            S = uncertainty.covariances[k]
            for j, grad in enumerate(constraint_gradients[k] if k < len(constraint_gradients) else []):
                back[k, j] = self.kappa * np.sqrt(grad.T @ S @ grad)
        return back


class TubeBasedRobustness:
    """uncertainty_prop.py:414-468: w_{k+1} = |A_k| w_k + d_max dt on the residual rows."""

    def __init__(self, dynamics, d_max: float = 0.1):
        self.dynamics = dynamics
        self.d_max = d_max

    def compute_tube(self, X_nom, U_nom, dt: float) -> np.ndarray:
        X_nom = np.asarray(X_nom, float)
        N, n_x = len(U_nom), X_nom.shape[1]
        widths = np.zeros((N + 1, n_x))
        w = np.zeros(n_x)
        for k in range(N):
            A_d, _ = self.dynamics.linearize(X_nom[k], U_nom[k], dt=dt)
            w = np.abs(A_d) @ w
            w[4:7] += self.d_max * dt
            if n_x >= 14:
                w[11:14] += self.d_max * dt
            widths[k + 1] = w
        return widths
