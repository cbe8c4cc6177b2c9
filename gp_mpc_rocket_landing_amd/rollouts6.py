"""Device-resident batch of closed-loop 6-DoF GP-MPC rollouts (BASELINE configs[4]).

The batched form of the reference's 6-DoF ``GPMPC.solve`` loop (gp_mpc.py:229-369
on the 14-state rocket, nominal_mpc.py:151-261) with the ``StructuredRocketGP``
FITC residuals (structured_gp.py:66-411, n_inducing = 2000 at config 5): every
control step runs, for every rollout, GPMPC's forward simulation with the GP
mean, the QP subproblem around it, the OSQP-style ADMM and the plant step on
the GPU (libgpmpc_hip.so, csrc/fleet6.hip; DESIGN.md section 9 states the
QCQP-to-QP choices).  Rollouts shard across ranks like the 3-DoF fleet.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .data import synthetic_6dof_training_data
from .gp.features import CombinedFeatureExtractor

NX6 = 14
# the compiled horizons of csrc/fleet6_n.h: every N from 2 to 30 (one instance each,
# csrc/fleet6_h*.hip; 30 = the two-items-per-thread cap of the 512-thread control kernel)
HORIZONS = tuple(range(2, 31))


def qp_rows(N: int) -> int:
    """Rows of the 6-DoF QP at horizon N: x0 + dynamics 14 (N+1), one bound row per
    variable (17 N + 14), N thrust rows and 4 (N-1) glide-slope rows."""
    return 14 * (N + 1) + (17 * N + 14) + N + 4 * (N - 1)


def rocket_config(params) -> dict:
    """Rollout6Config rocket fields from a Rocket6DoFParams-like object
    (rocket_6dof.py:36-84: J_B, r_T_B, g_I, I_sp, g0).  J_B is any invertible 3 x 3
    tensor (rocket_6dof.py:44, 77-78, 147): a diagonal one goes as its diagonal
    (rocket_j), any other as the full tensor (rocket_J, ABI 4), which the device
    inverts once and applies as nominal_mpc.py:196-199's ca.solve(J, .)."""
    J = np.asarray(params.J_B, float)
    if J.shape != (3, 3):
        raise ValueError(f"J_B must be 3 x 3, got {J.shape}")
    kw = dict(rocket_j=np.diag(J).copy(), rocket_r_t=np.asarray(params.r_T_B, float).reshape(3),
              rocket_g_i=np.asarray(params.g_I, float).reshape(3),
              rocket_alpha=1.0 / (float(params.I_sp) * float(params.g0)), rocket_g0=float(params.g0))
    if np.any(J - np.diag(np.diag(J))):
        kw["rocket_J"] = J.reshape(9).copy()
    return kw


def fit_structured_gp(n_train=4000, n_inducing=2000, seed=0, use_sparse=True):
    """The config-5 ``StructuredRocketGP`` (structured_gp.py:66-411) fitted on
    generator-G6 data (data.synthetic_6dof_training_data): d_v on the 13
    translational, d_w on the 12 rotational features, unit SE-ARD kernels and
    noise 1e-4 as the surface builds them, ``max_data_points = n_train`` (else
    add_data keeps only the newest 1000).  The inducing points are
    the surface's own: scipy kmeans2 on the global RNG (sparse_gp.py:122-148),
    seeded here by ``np.random.seed(seed)``."""
    from .gp.structured_gp import StructuredGPConfig, StructuredRocketGP
    X, U, Dv, Dw = synthetic_6dof_training_data(n_train, seed=seed)
    gp = StructuredRocketGP(StructuredGPConfig(n_inducing=n_inducing, max_data_points=n_train,
                                               use_sparse=use_sparse))
    gp.add_data(X, U, Dv, Dw)
    np.random.seed(seed)
    gp.fit()
    return gp


def device_handles(gp):
    """The fitted StructuredRocketGP's device GP pair (FITCHandle or
    ExactGPHandle each) and whether it is exact."""
    if not gp._is_fitted:
        gp.fit()
    hv, hw = gp.gp_v.device_handle, gp.gp_omega.device_handle
    if hv is None or hw is None:
        raise ValueError("the StructuredRocketGP's outputs must share one device GP per residual group")
    return hv, hw, not gp.config.use_sparse


def fit_structured_fitc(ctx=None, n_train=4000, n_inducing=2000, seed=0):
    """The config-5 FITC pair as device handles, through the StructuredRocketGP
    surface (fit_structured_gp).  Returns (gp_v handle, gp_w handle); the
    surface object stays alive on the first handle (``.surface``)."""
    gp = fit_structured_gp(n_train, n_inducing, seed)
    hv, hw, _ = device_handles(gp)
    hv.surface = gp
    return hv, hw


def initial_conditions_6dof(count, seed0=42, first=0):
    """Rollout starts: the run_experiments draw of [m, r, v] (monte_carlo.py:368-399,
    seed 42 + global index), a tilt of N(0, 5 deg) about a random horizontal body
    axis (its own RandomState(seed + 7919)), at rest in rotation."""
    from .experiments.monte_carlo import SimulationConfig, sample_initial_condition
    cfg = SimulationConfig.run_experiments()
    out = np.zeros((count, NX6))
    for i in range(count):
        seed = seed0 + first + i
        out[i, :7] = sample_initial_condition(seed, cfg)
        rs = np.random.RandomState(seed + 7919)
        ang = np.deg2rad(5.0) * rs.randn()
        phi = 2 * np.pi * rs.rand()
        out[i, 7] = np.cos(ang / 2)
        out[i, 8:11] = np.array([0.0, np.cos(phi), np.sin(phi)]) * np.sin(ang / 2)
    return out


class Rollouts6:
    """B rollouts on one device.  ``gp_v`` / ``gp_w``: FITCHandles (13 / 12
    features), or ExactGPHandles (the exact StructuredRocketGP)."""

    def __init__(self, ctx, gp_v, gp_w, batch, **config):
        self.ctx = ctx
        self.gp_v, self.gp_w = gp_v, gp_w  # keep alive: the kernels read their device state
        self.cfg = _lib.rollout6_default_config(**config)
        if int(self.cfg.horizon) not in HORIZONS:
            raise ValueError(f"horizon {int(self.cfg.horizon)}: the device controller is compiled for "
                             f"N = {HORIZONS[0]} .. {HORIZONS[-1]}")
        self.batch = int(batch)
        self.N = int(self.cfg.horizon)
        self.M = qp_rows(self.N)
        h = ctypes.c_void_p()
        exact = isinstance(gp_v, _lib.ExactGPHandle)
        if exact != isinstance(gp_w, _lib.ExactGPHandle):
            raise TypeError("gp_v and gp_w must both be FITC or both exact")
        create = _lib._L.gpmpc_rollout6_create_exact if exact else _lib._L.gpmpc_rollout6_create
        _lib._chk(create(ctx.h, gp_v.h, gp_w.h, ctypes.byref(self.cfg), self.batch, ctypes.byref(h)),
                  "rollout6_create")
        self.h = h

    def reset(self, x0, first=0):
        x0 = _lib.f64(np.atleast_2d(x0))
        _lib._chk(_lib._L.gpmpc_rollout6_reset(self.h, int(first), x0.shape[0], _lib._d(x0)), "rollout6_reset")

    def step(self, nsteps=1):
        _lib._chk(_lib._L.gpmpc_rollout6_step(self.h, int(nsteps)), "rollout6_step")

    def phases(self, mask):
        """gpmpc_rollout6_step_phases: 1 predict, 2 control, 4 plant (7 = a step)."""
        _lib._chk(_lib._L.gpmpc_rollout6_step_phases(self.h, int(mask)), "rollout6_step_phases")

    @property
    def records_dev(self):
        return _lib._L.gpmpc_rollout6_records_dev(self.h)

    def read(self):
        rec = np.empty((self.batch, _lib.REC_LEN)); x = np.empty((self.batch, NX6))
        _lib._chk(_lib._L.gpmpc_rollout6_read(self.h, _lib._d(rec), _lib._d(x)), "rollout6_read")
        return rec, x

    def state(self):
        """Records, states and each rollout's controller state: warm-start U,
        last plan X, forward-simulated X_pred and its GP means, scaled duals, rho."""
        rec, x = self.read()
        B, N = self.batch, self.N
        U = np.empty((B, N, 3)); X = np.empty((B, N + 1, NX6)); Xp = np.empty((B, N + 1, NX6))
        gm = np.empty((B, N, 6)); y = np.empty((B, self.M)); rho = np.empty(B)
        _lib._chk(_lib._L.gpmpc_rollout6_get_state(self.h, _lib._d(U), _lib._d(X), _lib._d(Xp), _lib._d(gm),
                                                   _lib._d(y), _lib._d(rho)), "rollout6_get_state")
        return dict(rec=rec, x=x, U=U, X=X, X_pred=Xp, gm=gm, y=y, rho=rho)

    def set_state(self, U=None, y=None, rho=None):
        """gpmpc_rollout6_set_state (None leaves a part unchanged)."""
        B, N = self.batch, self.N
        a = [None if v is None else _lib.f64(np.reshape(v, shape))
             for v, shape in ((U, (B, N, 3)), (y, (B, self.M)), (rho, (B,)))]
        _lib._chk(_lib._L.gpmpc_rollout6_set_state(self.h, *[None if v is None else _lib._d(v) for v in a]),
                  "rollout6_set_state")

    def solve(self, x0, x_target, cold, max_sqp_iter=10, sqp_tol=1e-4, X_ref=None, U_ref=None):
        """GPMPC.solve (gp_mpc.py:229-369) for every rollout (gpmpc_rollout6_solve_ref).
        X_ref (B, N+1, 14) / U_ref (B, N, 3): the QP cost's reference trajectory
        (gp_mpc.py:442-453; None = x_target on every stage / zero).
        Returns dict(X (B, N+1, 14), U (B, N, 3), passes, converged, qp_status,
        qp_iters) of int arrays (B,)."""
        B, N = self.batch, self.N
        x0 = _lib.f64(np.reshape(x0, (B, NX6))); xt = _lib.f64(np.reshape(x_target, (B, NX6)))
        xr = None if X_ref is None else _lib.f64(np.reshape(X_ref, (B, N + 1, NX6)))
        ur = None if U_ref is None else _lib.f64(np.reshape(U_ref, (B, N, 3)))
        X = np.empty((B, N + 1, NX6)); U = np.empty((B, N, 3))
        ps, cv, qs, qi = (np.zeros(B, np.int32) for _ in range(4))
        _lib._chk(_lib._L.gpmpc_rollout6_solve_ref(self.h, _lib._d(x0), _lib._d(xt),
                                                   None if xr is None else _lib._d(xr),
                                                   None if ur is None else _lib._d(ur), int(cold),
                                                   int(max_sqp_iter), float(sqp_tol), _lib._d(X), _lib._d(U),
                                                   _lib._i(ps), _lib._i(cv), _lib._i(qs), _lib._i(qi)),
                  "rollout6_solve")
        return dict(X=X, U=U, passes=ps, converged=cv.astype(bool), qp_status=qs, qp_iters=qi)

    def close(self):
        if getattr(self, "h", None):
            _lib._L.gpmpc_rollout6_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
