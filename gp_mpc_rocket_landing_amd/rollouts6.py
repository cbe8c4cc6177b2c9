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


def fit_structured_fitc(ctx, n_train=4000, n_inducing=2000, seed=0):
    """The config-5 StructuredRocketGP pair as device FITC handles: d_v on the 13
    translational, d_w on the 12 rotational features of generator-G6 data
    (data.synthetic_6dof_training_data), unit SE-ARD kernels and noise 1e-4 as
    StructuredRocketGP builds them; the inducing points are a seeded random
    subset of the training rows (kmeans2's, sparse_gp.py:122-148, is host work
    outside the hot path)."""
    X, U, Dv, Dw = synthetic_6dof_training_data(n_train, seed=seed)
    fe = CombinedFeatureExtractor()
    Zv = fe.extract_batch_translational(X, U)
    Zw = fe.extract_batch_rotational(X, U)
    idx = np.sort(np.random.RandomState(seed + 3).choice(n_train, min(n_inducing, n_train), replace=False))
    gv = _lib.FITCHandle(ctx, Zv[idx], Zv, Dv, np.ones(Zv.shape[1]), 1.0, 1e-4)
    gw = _lib.FITCHandle(ctx, Zw[idx], Zw, Dw, np.ones(Zw.shape[1]), 1.0, 1e-4)
    return gv, gw


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
    """B rollouts on one device.  ``gp_v`` / ``gp_w``: FITCHandles (13 / 12 features)."""

    def __init__(self, ctx, gp_v, gp_w, batch, **config):
        self.ctx = ctx
        self.gp_v, self.gp_w = gp_v, gp_w  # keep alive: the kernels read their device state
        self.cfg = _lib.rollout6_default_config(**config)
        self.batch = int(batch)
        h = ctypes.c_void_p()
        _lib._chk(_lib._L.gpmpc_rollout6_create(ctx.h, gp_v.h, gp_w.h, ctypes.byref(self.cfg), self.batch,
                                                ctypes.byref(h)), "rollout6_create")
        self.h = h

    def reset(self, x0, first=0):
        x0 = _lib.f64(np.atleast_2d(x0))
        _lib._chk(_lib._L.gpmpc_rollout6_reset(self.h, int(first), x0.shape[0], _lib._d(x0)), "rollout6_reset")

    def step(self, nsteps=1):
        _lib._chk(_lib._L.gpmpc_rollout6_step(self.h, int(nsteps)), "rollout6_step")

    def read(self):
        rec = np.empty((self.batch, _lib.REC_LEN)); x = np.empty((self.batch, NX6))
        _lib._chk(_lib._L.gpmpc_rollout6_read(self.h, _lib._d(rec), _lib._d(x)), "rollout6_read")
        return rec, x

    def state(self):
        """Records, states and each rollout's controller state: warm-start U,
        last plan X, forward-simulated X_pred and its GP means, scaled duals, rho."""
        rec, x = self.read()
        B, N = self.batch, int(self.cfg.horizon)
        U = np.empty((B, N, 3)); X = np.empty((B, N + 1, NX6)); Xp = np.empty((B, N + 1, NX6))
        gm = np.empty((B, N, 6)); y = np.empty((B, 1104)); rho = np.empty(B)
        _lib._chk(_lib._L.gpmpc_rollout6_get_state(self.h, _lib._d(U), _lib._d(X), _lib._d(Xp), _lib._d(gm),
                                                   _lib._d(y), _lib._d(rho)), "rollout6_get_state")
        return dict(rec=rec, x=x, U=U, X=X, X_pred=Xp, gm=gm, y=y, rho=rho)

    def close(self):
        if getattr(self, "h", None):
            _lib._L.gpmpc_rollout6_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
