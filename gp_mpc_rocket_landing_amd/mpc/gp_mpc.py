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

import time
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .. import _lib
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


class GPMPC(_SQPBase):
    def __init__(self, dynamics, gp_model, config: Optional[GPMPCConfig] = None,
                 constraint_params=None, cost_weights=None, ctx=None):
        n_state = getattr(dynamics, "n_state", 7)
        if n_state != 7:
            raise NotImplementedError("this GPMPC runs the 3-DoF model (n_x = 7)")
        super().__init__(dynamics, config or GPMPCConfig(), ctx=ctx)
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

    def _initial(self, x0, x_target):
        N = self.config.N
        if self._X_warm is not None:
            return self._X_warm.copy(), self._U_warm.copy()
        a = (np.arange(N + 1) / N)[:, None]
        X = (1 - a) * x0 + a * x_target
        U = np.zeros((N, self.n_u)); U[:, 0] = x0[0] * 1.0
        return X, U

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

    def solve(self, x0, x_target, X_ref=None, U_ref=None) -> MPCSolution:  # noqa: ARG002
        if not self._is_setup:
            self.setup()
        x0 = np.asarray(x0, float); x_target = np.asarray(x_target, float)
        X, U = self._initial(x0, x_target)
        self._propagate(x0, U)
        if self.config.max_sqp_iter <= 1:
            t0 = time.perf_counter()
            P, q = self._qp.cost(np.tile(x_target, (self.config.N + 1, 1)))
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
                               cost=trajectory_cost(X, U, x_target) if ok else np.inf,
                               solve_time=time.perf_counter() - t0, iterations=int(r["iter"][0]),
                               status=_lib.QP_STATUS_TEXT.get(st, str(st)))
        X, U, conv, it, st, dt = self._sqp(x0, x_target, X, U, self.config.max_sqp_iter, -1.0)
        self._X_warm, self._U_warm = X.copy(), U.copy()
        return MPCSolution(success=conv, X_opt=X, U_opt=U, cost=trajectory_cost(X, U, x_target),
                           solve_time=dt, iterations=it, status="Converged" if conv else "Max iterations")

    def get_uncertainty_at_horizon(self, k: Optional[int] = None):
        """gp_mpc.py:486-492 (a stub returning None in the reference): the propagated
        covariance (n_x, n_x) at horizon step k of the last solve; with no k, the
        GP variances (N, 3) at the last solve's horizon points."""
        if k is None:
            return None if self._last_var is None else self._last_var.copy()
        return None if self.last_uncertainty is None else self.last_uncertainty.covariances[k].copy()


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
