"""GPMPC surface of reference src/mpc/gp_mpc.py:66-497, 3-DoF mode.

The reference GPMPC is written for the 14-state 6-DoF model with a CasADi/
IPOPT QP subproblem; its 3-DoF use needs an adapter.  This one
is the control step the fleet runs on the device for every landing (SURVEY
8d C3), for one landing from the host:

  * linearisation trajectory = the shifted previous solution (or the
    linear-interpolation / hover guess on the first call, osqp_rti.py:425-446);
  * GP mean d_v at the N horizon points of that trajectory, one device call
    (Simple3DoFGP.predict_batch) -- gp_mpc.py:309-314 adds dt*d_v to c_k;
  * RTI QP with x+ = A x + B u + c (gp_mpc.py:410-411 sign), warm-started,
    solved by the device ADMM whose rho / scaled y persist across calls;
  * success = the ADMM returned a solution (solved, solved inaccurate or max
    iterations reached); the shifted solution becomes the next linearisation.

``max_sqp_iter`` > 1 re-linearises around each QP solution like the
reference's outer loop (gp_mpc.py:296-345, stop at 1e-4), success = converged.
With ``use_gp_uncertainty`` (the default) each solve also propagates the
state covariance along the linearisation trajectory (UncertaintyPropagator,
linear: one batched GP call per step + the device covariance kernel;
gp_mpc.py:284-290) and derives the step-0 tightened constraint parameters
(gp_mpc.py:177-215, 414).  As in the reference these change nothing the QP
uses (only thrust bounds and the glideslope enter it, and neither
is tightened); they are exposed through ``last_uncertainty``,
``last_tightened_params`` and ``get_uncertainty_at_horizon(k)``.  Propagation
uses the propagator's default dt = 0.1 like the reference (D6).
"""
from __future__ import annotations

import dataclasses
import time
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .. import _lib
from .. import rollouts6 as _r6
from .constraints import ConstraintParams, TightenedConstraints
from .cost_functions import CostWeights
from .nominal_mpc import MPCConfig, MPCSolution, _SQPBase, trajectory_cost
from .qp_builder import solution_to_vector, vector_to_solution
from .uncertainty_prop import PropagatedUncertainty, UncertaintyPropagator


@dataclass
class GPMPCConfig(MPCConfig):
    """gp_mpc.py:48-63."""
    use_gp_mean: bool = True
    use_gp_uncertainty: bool = True
    confidence_level: float = 0.95
    max_variance_for_constraint: float = 1.0
    robust_horizon: int = -1
    max_sqp_iter: int = 1
    # QP settings of the loop's passes (max_sqp_iter > 1); None = qp_max_iter / qp_eps.
    # The reference solves this subproblem with IPOPT (gp_mpc.py:462-470).
    sqp_qp_max_iter: Optional[int] = None
    sqp_qp_eps: Optional[float] = None

    def qp_settings(self):
        """(max_iter, eps) of the QP solves this configuration runs."""
        if self.max_sqp_iter > 1:
            return (self.qp_max_iter if self.sqp_qp_max_iter is None else self.sqp_qp_max_iter,
                    self.qp_eps if self.sqp_qp_eps is None else self.sqp_qp_eps)
        return self.qp_max_iter, self.qp_eps


class GPMPC(_SQPBase):
    """``GPMPC(dynamics, gp_model, config, constraint_params, cost_weights)``.

    A 14-state plant (``dynamics.n_state == 14``, the reference's own use with
    StructuredRocketGP) constructs the 6-DoF device controller, GPMPC6DoF; a
    7-state plant the 3-DoF adapter below."""

    def __new__(cls, dynamics=None, *args, **kwargs):
        if cls is GPMPC and getattr(dynamics, "n_state", 7) == 14:
            return super().__new__(GPMPC6DoF)
        return super().__new__(cls)

    def __init__(self, dynamics, gp_model, config: Optional[GPMPCConfig] = None,
                 constraint_params=None, cost_weights=None, ctx=None):
        n_state = getattr(dynamics, "n_state", 7)
        if n_state != 7:
            raise NotImplementedError("the 3-DoF adapter runs n_x = 7; 14 states go to GPMPC6DoF")
        config = config or GPMPCConfig()
        mi, eps = config.qp_settings()
        super().__init__(dynamics, dataclasses.replace(config, qp_max_iter=mi, qp_eps=eps), ctx=ctx)
        self.config = config
        self.gp = gp_model
        self.constraint_params = constraint_params or ConstraintParams()
        self.cost_weights = cost_weights or CostWeights()
        self._tightened_constraints = TightenedConstraints(base_params=self.constraint_params,
                                                           confidence_level=self.config.confidence_level)
        self._uncertainty_prop = UncertaintyPropagator(dynamics, gp_model, ctx=ctx)
        self.last_uncertainty: Optional[PropagatedUncertainty] = None
        self.last_tightened_params: Optional[ConstraintParams] = None
        self._last_var = None
        self._is_setup = False

    def setup(self) -> None:
        self._is_setup = True

    def _gp_mean(self, X, U):
        if not self.config.use_gp_mean or self.gp is None:
            return None
        N = self.config.N
        if hasattr(self.gp, "predict_batch"):
            mean, var = self.gp.predict_batch(X[:N], U[:N])
        else:
            mv = [self.gp.predict(X[k], U[k]) for k in range(N)]
            mean = np.array([m for m, _ in mv]); var = np.array([v for _, v in mv])
        self._last_var = np.asarray(var)
        return np.asarray(mean)

    def _initial(self, x0, x_target, U_ref=None):
        N = self.config.N
        if self._X_warm is not None:
            return self._X_warm.copy(), self._U_warm.copy()
        a = (np.arange(N + 1) / N)[:, None]
        X = (1 - a) * x0 + a * x_target
        if U_ref is not None:   # gp_mpc.py:268-269: U_ref as the first guess
            return X, np.array(U_ref, float)[:N].copy()
        U = np.zeros((N, self.n_u)); U[:, 0] = x0[0] * 1.0
        return X, U

    def _references(self, x_target, X_ref, U_ref):
        """(X_ref (N+1, n_x), U_ref (N, 3) or None) of gp_mpc.py:442-453: x_target on
        every stage by default; a reference of N rows takes x_target as its
        terminal row (:452)."""
        N = self.config.N
        if X_ref is None:
            Xr = np.tile(x_target, (N + 1, 1))
        else:
            Xr = np.asarray(X_ref, float).reshape(-1, self.n_x)
            if Xr.shape[0] < N:
                raise ValueError(f"X_ref needs at least N = {N} rows, got {Xr.shape[0]}")
            Xr = np.vstack([Xr[:N], Xr[N:N + 1] if Xr.shape[0] > N else x_target[None]])
        if U_ref is None:
            return Xr, None
        Ur = np.asarray(U_ref, float).reshape(-1, self.n_u)
        if Ur.shape[0] < N:
            raise ValueError(f"U_ref needs at least N = {N} rows, got {Ur.shape[0]}")
        return Xr, Ur[:N]

    def _get_tightened_params(self, unc: PropagatedUncertainty, k: int) -> ConstraintParams:
        """gp_mpc.py:177-215; the 7-state model has no attitude / rate rows (0 std)."""
        if not self.config.use_gp_uncertainty:
            return self.constraint_params
        std = np.sqrt(np.diag(unc.covariances[k]))
        position_std = float(np.mean(std[1:4]))
        velocity_std = float(np.mean(std[4:7]))
        attitude_std = float(np.mean(std[8:10])) if std.size >= 14 else 0.0
        omega_std = float(np.mean(std[11:14])) if std.size >= 14 else 0.0
        if velocity_std > self.config.max_variance_for_constraint:
            return self.constraint_params
        return self._tightened_constraints.get_tightened_params(position_std=position_std,
                                                                velocity_std=velocity_std,
                                                                attitude_std=attitude_std,
                                                                omega_std=omega_std)

    def _propagate(self, x0, U):
        if not (self.config.use_gp_uncertainty and self.gp is not None):
            self.last_uncertainty = None
            self.last_tightened_params = self.constraint_params
            return
        self.last_uncertainty = self._uncertainty_prop.propagate(
            x0=x0, U=U[: self.config.N], Sigma_0=np.eye(self.n_x) * 1e-6)
        self.last_tightened_params = self._get_tightened_params(self.last_uncertainty, 0)

    def solve(self, x0, x_target, X_ref=None, U_ref=None) -> MPCSolution:
        """X_ref / U_ref: the QP cost's reference trajectory and controls
        (gp_mpc.py:442-453); U_ref also seeds the first guess (:268-269)."""
        if not self._is_setup:
            self.setup()
        x0 = np.asarray(x0, float); x_target = np.asarray(x_target, float)
        Xr, Ur = self._references(x_target, X_ref, U_ref)
        X, U = self._initial(x0, x_target, Ur)
        self._propagate(x0, U)
        if self.config.max_sqp_iter <= 1:
            t0 = time.perf_counter()
            P, q = self._qp.cost(Xr, Ur)
            Aval, l, u = self._qp.constraints(X, U, x0, gp_dv=self._gp_mean(X, U), sign=-1.0)
            r = self._ws.solve(Aval, P, q, l, u, solution_to_vector(X, U))
            st = int(r["status"][0])
            self.last_status, self.last_iterations = st, int(r["iter"][0])
            ok = st in (1, 2, -2)
            if ok:
                X, U = vector_to_solution(r["x"][0], self.config.N)
                self._X_warm = np.vstack([X[1:], X[-1:]])
                self._U_warm = np.vstack([U[1:], U[-1:]])
            return MPCSolution(success=ok, X_opt=X, U_opt=U,
                               cost=trajectory_cost(X, U, Xr, Ur) if ok else np.inf,
                               solve_time=time.perf_counter() - t0, iterations=int(r["iter"][0]),
                               status=_lib.QP_STATUS_TEXT.get(st, str(st)))
        X[0] = x0   # X_pred[0] = x0 (gp_mpc.py:263)
        X, U, conv, it, st, dt = self._sqp(x0, x_target, X, U, self.config.max_sqp_iter, -1.0, Xr, Ur)
        self._X_warm, self._U_warm = X.copy(), U.copy()
        return MPCSolution(success=conv, X_opt=X, U_opt=U, cost=trajectory_cost(X, U, Xr, Ur),
                           solve_time=dt, iterations=it, status="Converged" if conv else "Max iterations")

    def get_uncertainty_at_horizon(self, k: Optional[int] = None):
        """gp_mpc.py:486-492 (a stub returning None in the reference): the propagated
        covariance (n_x, n_x) at horizon step k of the last solve; with no k, the
        GP variances (N, 3) at the last solve's horizon points."""
        if k is None:
            return None if self._last_var is None else self._last_var.copy()
        return None if self.last_uncertainty is None else self.last_uncertainty.covariances[k].copy()


class GPMPC6DoF(GPMPC):
    """The reference's own GPMPC: the 14-state rocket with StructuredRocketGP
    (gp_mpc.py:66-497), one control solve on the device (csrc/fleet6.hip
    through gpmpc_rollout6_solve, a batch of one).

    ``solve(x0, x_target)`` = gp_mpc.py:229-369: forward simulation of the
    warm-start controls with the GP mean (RK4 of nominal_mpc.py:163-203 +
    [.., d_v dt, .., d_w dt]), then up to ``max_sqp_iter`` passes of
    linearise (A_d = I + A_c dt, B_d = B_c dt) -> c_k = GP mean dt -> QP
    subproblem (:394-460) -> plan, stopping when max|dX|, max|dU| < sqp_tol.
    The QP subproblem is the reference's with its quadratic constraints made
    linear (thrust ball -> box, |u| >= T_min linearised at
    U_nom, glide-slope cone -> 4 half-planes, trust balls -> boxes), solved by
    the OSQP-0.6 ADMM (osqp_rti.py settings: the reference's IPOPT/CasADi are
    absent) with OSQP's persistent rho / duals across passes and calls.

    Defaults and semantics as the 3-DoF adapter (D14): ``max_sqp_iter = 1``
    (the RTI control step; success = the ADMM returned a solution); ``> 1``
    runs the reference loop (success = converged, status "Converged" / "Max
    iterations"; a QP without a solution returns the nominal, which the
    reference's loop counts as converged, gp_mpc.py:478-482 + :343).

    The GP must be a fitted StructuredRocketGP (FITC or exact); its means are
    what ``gp.predict`` returns (FITC: K*u alpha as written).
    Cost weights must be diagonal (CostWeights builds them so).  ``X_ref`` /
    ``U_ref`` enter the QP cost as the reference writes it (:442-453: x_k -
    X_ref[k], u_k - U_ref[k], terminal X_ref[N] or x_target when X_ref has N
    rows); U_ref also seeds the first guess when there is no warm start
    (:268-269).  The horizon is ``config.N`` -- ``GPMPCConfig()`` is the
    reference's N = 20 (gp_mpc.py:110, nominal_mpc.py:47); the device
    controller is compiled for every N from 2 to 30 (BASELINE configs[4]: 30).  The
    rocket is ``dynamics.params`` (J_B, r_T_B, g_I, I_sp, g0 of
    Rocket6DoFConfig); J_B may be any invertible tensor (ABI 4 rocket_J).
    """
    n_x, n_u = 14, 3

    def __init__(self, dynamics, gp_model, config: Optional[GPMPCConfig] = None,
                 constraint_params=None, cost_weights=None, ctx=None):
        config = config or GPMPCConfig()
        if int(config.N) not in _r6.HORIZONS:
            raise NotImplementedError(f"the 6-DoF device controller is compiled for N = {_r6.HORIZONS[0]} .. "
                                      f"{_r6.HORIZONS[-1]} (two QP items per thread of its 512-thread "
                                      f"workgroup), not {config.N}")
        params = getattr(dynamics, "params", None)
        if params is None:
            raise TypeError("dynamics must expose the rocket's params (Rocket6DoFDynamics)")
        self._rocket_kw = _r6.rocket_config(params)
        self.dynamics = dynamics
        self.config = config
        self.gp = gp_model
        self.constraint_params = constraint_params or ConstraintParams()
        self.cost_weights = cost_weights or CostWeights()
        self._ctx = ctx   # the device context is taken at the first solve
        self._tightened_constraints = TightenedConstraints(base_params=self.constraint_params,
                                                           confidence_level=self.config.confidence_level)
        self._uncertainty_prop = UncertaintyPropagator(dynamics, gp_model, ctx=ctx)
        self.last_uncertainty: Optional[PropagatedUncertainty] = None
        self.last_tightened_params: Optional[ConstraintParams] = None
        self._last_var = None
        self._X_warm = self._U_warm = None
        self._ro = None
        self._ro_key = None
        self._is_setup = False
        self.last_status, self.last_iterations, self.last_passes = -10, 0, 0
        self._cfg_kw = self._device_problem()

    def _device_problem(self):
        cw, cp = self.cost_weights, self.constraint_params
        Q, R, P = (np.asarray(M, float) for M in (cw.Q, cw.R, cw.P))
        for M in (Q, R, P):
            if np.any(M - np.diag(np.diag(M))):
                raise NotImplementedError("the device QP takes diagonal cost weights (CostWeights' own)")
        return dict(horizon=int(self.config.N), **self._rocket_kw,
                    q_diag=np.diag(Q), p_diag=np.diag(P), r_diag=np.diag(R), t_min=float(cp.T_min),
                    t_max=float(cp.T_max), tan_gamma_gs=float(np.tan(cp.gamma_gs_rad)),
                    dt=float(self.config.dt), use_gp_mean=int(bool(self.config.use_gp_mean)),
                    fitc_mean_as_written=1,   # gp.predict's mean (sparse_gp.py:280-283, D1)
                    max_iter=int(self.config.qp_settings()[0]), eps_abs=float(self.config.qp_settings()[1]),
                    eps_rel=float(self.config.qp_settings()[1]))

    def _rollout(self):
        """The batch-of-one device controller over the GP's current device pair;
        rebuilt (carrying U, duals and rho) when the GP has been refitted."""
        hv, hw, _ = _r6.device_handles(self.gp)
        key = (id(hv), id(hw))
        if self._ro is not None and key == self._ro_key:
            return self._ro
        old = self._ro.state() if self._ro is not None else None
        if self._ctx is None:
            self._ctx = _lib.default_context()
        ro = _r6.Rollouts6(self._ctx, hv, hw, 1, **self._cfg_kw)
        if old is not None:
            ro.set_state(U=old["U"], y=old["y"], rho=old["rho"])
            self._ro.close()
        self._ro, self._ro_key = ro, key
        return ro

    def reset_warm_start(self) -> None:
        """gp_mpc.py:494-497 (+ the ADMM's persistent duals / rho)."""
        self._X_warm = self._U_warm = None

    def _references(self, x_target, X_ref, U_ref):
        """The QP cost's (X_ref (N+1, 14), U_ref (N, 3)) of gp_mpc.py:442-453: X_ref
        defaults to x_target on every stage, a reference of N rows takes x_target as
        its terminal row (:452), U_ref defaults to zero."""
        N = self.config.N
        if X_ref is None:
            Xr = np.tile(x_target, (N + 1, 1))
        else:
            Xr = np.asarray(X_ref, float).reshape(-1, 14)
            if Xr.shape[0] < N:
                raise ValueError(f"X_ref needs at least N = {N} rows, got {Xr.shape[0]}")
            Xr = np.vstack([Xr[:N], Xr[N:N + 1] if Xr.shape[0] > N else x_target[None]])
        Ur = np.zeros((N, 3)) if U_ref is None else np.asarray(U_ref, float).reshape(-1, 3)[:N]
        if Ur.shape[0] < N:
            raise ValueError(f"U_ref needs at least N = {N} rows, got {Ur.shape[0]}")
        return Xr, Ur

    def solve(self, x0, x_target, X_ref=None, U_ref=None) -> MPCSolution:
        if not self._is_setup:
            self.setup()
        t0 = time.perf_counter()
        N = self.config.N
        x0 = np.asarray(x0, float).reshape(14); x_target = np.asarray(x_target, float).reshape(14)
        Xr, Ur = self._references(x_target, X_ref, U_ref)
        ro = self._rollout()
        if self._U_warm is not None:
            cold = 0
        elif U_ref is not None:  # gp_mpc.py:268-269: U_ref as the first guess
            ro.set_state(U=Ur.reshape(1, N, 3))
            cold = 2
        else:
            cold = 1
        max_sqp = max(1, int(self.config.max_sqp_iter))
        r = ro.solve(x0[None], x_target[None], cold, max_sqp_iter=max_sqp, sqp_tol=float(self.config.sqp_tol),
                     X_ref=None if X_ref is None else Xr[None], U_ref=None if U_ref is None else Ur[None])
        X, U = r["X"][0], r["U"][0]
        st, passes = int(r["qp_status"][0]), int(r["passes"][0])
        has = st in (1, 2, -2)
        self.last_status, self.last_iterations, self.last_passes = st, int(r["qp_iters"][0]), passes
        self._X_warm, self._U_warm = X.copy(), U.copy()
        self._propagate(x0, U)
        cost = self._cost(X, U, Xr, Ur) if has else np.inf
        if max_sqp <= 1:
            return MPCSolution(success=has, X_opt=X, U_opt=U, cost=cost, solve_time=time.perf_counter() - t0,
                               iterations=self.last_iterations, status=_lib.QP_STATUS_TEXT.get(st, str(st)))
        conv = bool(r["converged"][0])
        return MPCSolution(success=conv, X_opt=X, U_opt=U, cost=cost, solve_time=time.perf_counter() - t0,
                           iterations=passes, status="Converged" if conv else "Max iterations")

    def _cost(self, X, U, Xr, Ur):
        """gp_mpc.py:447-458 at the returned plan against (X_ref, U_ref)."""
        cw = self.cost_weights
        e = X - Xr
        du = U - Ur
        return float(np.einsum("ki,ij,kj->", e[:-1], cw.Q, e[:-1]) + np.einsum("ki,ij,kj->", du, cw.R, du)
                     + e[-1] @ cw.P @ e[-1])

    def _get_tightened_params(self, unc: PropagatedUncertainty, k: int) -> ConstraintParams:
        return GPMPC._get_tightened_params(self, unc, k)

    def _propagate(self, x0, U):
        """gp_mpc.py:284-290 with the returned controls.  The re-propagations
        of :347-353 are not repeated per pass: their only consumer,
        _get_tightened_params(uncertainty, 0) (:414), reads covariances[0] =
        Sigma_0 and tightens none of the rows the QP has (D14)."""
        GPMPC._propagate(self, x0, U)

    def close(self):
        if self._ro is not None:
            self._ro.close()
            self._ro = None


class SimpleGPPredictor:
    """gp_mpc.py:505-574: GP-augmented one-step prediction and rollout.

    Works with either GP surface: a 4-tuple GP (StructuredRocketGP, 14 states:
    residuals on v-dot 4:7 and omega-dot 11:14, as the reference) or a 2-tuple
    GP (Simple3DoFGP, 7 states: residual on v-dot only).  ``simulate`` evaluates
    the GP one step at a time like the reference (each step depends on the last).
    """

    def __init__(self, dynamics, gp_model):
        self.dynamics = dynamics
        self.gp = gp_model

    def predict(self, x, u, dt: float):
        x = np.asarray(x, float)
        x_nom = np.asarray(self.dynamics.step(x, u, dt), float)
        r = self.gp.predict(x, u)
        n = x.size
        x_next = x_nom.copy()
        d_mean = np.zeros(14 if len(r) == 4 else n)
        d_var = np.zeros_like(d_mean)
        if len(r) == 4:
            d_v, d_w, var_v, var_w = r
            x_next[4:7] += d_v * dt
            x_next[11:14] += d_w * dt
            d_mean[4:7] = d_v; d_mean[11:14] = d_w
            d_var[4:7] = var_v; d_var[11:14] = var_w
        else:
            d_v, var_v = r
            x_next[4:7] += d_v * dt
            d_mean[4:7] = d_v; d_var[4:7] = var_v
        return x_next, d_mean, d_var

    def simulate(self, x0, U, dt: float):
        x0 = np.asarray(x0, float)
        N = len(U)
        X = np.zeros((N + 1, x0.size))
        X[0] = x0
        D_mean, D_var = [], []
        for k in range(N):
            X[k + 1], dm, dv = self.predict(X[k], U[k], dt)
            D_mean.append(dm); D_var.append(dv)
        width = D_mean[0].size if N else 14
        return X, np.array(D_mean).reshape(N, width), np.array(D_var).reshape(N, width)
