"""Device-resident batch ("fleet") of closed-loop 3-DoF GP-MPC landings.

The fleet is the batched form of ``MonteCarloSimulator.run_single``
(monte_carlo.py:401-583) driving the 3-DoF ``GPMPC`` surface: every control
step runs the GP posterior at the N horizon points of every landing, the RTI
QP assembly with the GP mean, the batched OSQP-style ADMM, the plant step and
the termination rules -- all on the GPU (libgpmpc_hip.so, csrc/fleet.hip).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .data import synthetic_training_data
from .gp.features import Simple3DoFFeatureExtractor

# record layout (GPMPC_REC_LEN = 16 doubles per landing)
REC_OUTCOME, REC_STEPS, REC_FUEL, REC_TIME = 0, 1, 2, 3
REC_STATE = slice(4, 11)
REC_ADMM_ITERS, REC_SOLVED, REC_M0, REC_LAST_STATUS, REC_RHO = 11, 12, 13, 14, 15
OUTCOMES = {0: "RUNNING", 1: "SUCCESS", 2: "CRASH", 3: "FUEL_EXHAUSTED",
            4: "CONSTRAINT_VIOLATION", 5: "TIMEOUT", 6: "DIVERGENCE"}


def fit_gp(ctx, n_train=1000, seed=0, noise=1e-4):
    """Exact Simple3DoF GP on generator G -- the GP every landing shares."""
    X, U, D = synthetic_training_data(n_train, seed=seed)
    Z = Simple3DoFFeatureExtractor().extract_batch(X, U)
    return _lib.ExactGPHandle(ctx, _lib.SE_ARD, Z, D, np.ones(Z.shape[1]), 1.0, noise)


def fit_gp_sparse(n_train=1000, n_inducing=50, seed=0):
    """The reference-default ``Simple3DoFGP()`` (structured_gp.py:423-428: a
    MultiOutputSparseGP, FITC, 50 inducing points shared by the 3 outputs, kmeans2 on
    the global RNG, sparse_gp.py:122-148, seeded here by ``np.random.seed(seed)``)
    fitted through the surface on generator G data.  Returns its device FITCHandle
    (``.surface`` keeps the surface alive)."""
    from .gp.structured_gp import Simple3DoFGP
    X, U, D = synthetic_training_data(n_train, seed=seed)
    gp = Simple3DoFGP(n_inducing=n_inducing)
    gp.add_data(X, U, D)
    np.random.seed(seed)
    gp.fit()
    h = gp.gp.device_handle
    if h is None:
        raise RuntimeError("the Simple3DoFGP's outputs must share one device GP")
    h.surface = gp
    return h


class Fleet:
    """``gp``: an exact GP (ExactGPHandle) or a sparse one (FITCHandle: FITC or VFE,
    gpmpc_fleet_create_fitc -- the reference-default ``Simple3DoFGP()`` is FITC with
    50 inducing points).  ``fleet_batch``: the size of the whole Monte-Carlo fleet when
    this one is a shard of it (gpmpc_fleet_create_shard): every size-dependent kernel
    choice is made for that size, so the shard's landings come out bit-identical to
    the same landings in the whole fleet.  Default: the fleet is whole."""

    def __init__(self, ctx, gp, batch, fleet_batch=None, **config):
        self.ctx = ctx
        self.gp = gp  # keep the GP alive: the fleet reads its device factor
        self.cfg = _lib.fleet_default_config(**config)
        self.batch = int(batch)
        self.fleet_batch = int(fleet_batch) if fleet_batch is not None else self.batch
        h = ctypes.c_void_p()
        create = (_lib._L.gpmpc_fleet_create_fitc if isinstance(gp, _lib.FITCHandle)
                  else _lib._L.gpmpc_fleet_create_shard)
        _lib._chk(create(ctx.h, gp.h, ctypes.byref(self.cfg), self.batch, self.fleet_batch, ctypes.byref(h)),
                  "fleet_create")
        self.h = h

    def reset(self, x0, first=0):
        x0 = _lib.f64(np.atleast_2d(x0))
        _lib._chk(_lib._L.gpmpc_fleet_reset(self.h, int(first), x0.shape[0], _lib._d(x0)), "fleet_reset")

    def step(self, nsteps=1):
        _lib._chk(_lib._L.gpmpc_fleet_step(self.h, int(nsteps)), "fleet_step")

    def phases(self, mask):
        _lib._chk(_lib._L.gpmpc_fleet_step_phases(self.h, int(mask)), "fleet_step_phases")

    def read(self):
        rec = np.empty((self.batch, _lib.REC_LEN)); x = np.empty((self.batch, 7))
        _lib._chk(_lib._L.gpmpc_fleet_read(self.h, _lib._d(rec), _lib._d(x)), "fleet_read")
        return rec, x

    def state(self):
        """Every landing's full controller state: x, records, the linearisation /
        warm-start trajectory Xw, Uw, the ADMM's persistent scaled duals and rho."""
        rec, x = self.read()
        B, N = self.batch, int(self.cfg.horizon)
        m = 7 * (N + 1) + 10 * N + 7
        Xw = np.empty((B, N + 1, 7)); Uw = np.empty((B, N, 3)); y = np.empty((B, m)); rho = np.empty(B)
        _lib._chk(_lib._L.gpmpc_fleet_get_state(self.h, _lib._d(Xw), _lib._d(Uw), _lib._d(y),
                                                _lib._d(rho)), "fleet_get_state")
        return dict(rec=rec, x=x, Xw=Xw, Uw=Uw, y=y, rho=rho)

    def posterior(self):
        """The last control step's GP posterior at every landing's N horizon points
        (ExactGP.predict, exact_gp.py:256-266): mean and variance, (batch, N, 3) each,
        in landing order."""
        B, N = self.batch, int(self.cfg.horizon)
        mean = np.empty((B, N, 3)); var = np.empty((B, N, 3))
        _lib._chk(_lib._L.gpmpc_fleet_get_posterior(self.h, _lib._d(mean), _lib._d(var)),
                  "fleet_get_posterior")
        return mean, var

    @property
    def records_dev(self):
        return _lib._L.gpmpc_fleet_records_dev(self.h)

    def close(self):
        if getattr(self, "h", None):
            _lib._L.gpmpc_fleet_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def initial_conditions(count, seed0=42, first=0):
    from .experiments.monte_carlo import SimulationConfig, sample_initial_condition
    cfg = SimulationConfig.run_experiments()
    return np.array([sample_initial_condition(seed0 + first + i, cfg) for i in range(count)])


def run_fleet(ctx, batch, steps, seed0=42, gp=None, **config):
    gp = gp or fit_gp(ctx)
    f = Fleet(ctx, gp, batch, **config)
    f.reset(initial_conditions(batch, seed0))
    f.step(steps)
    rec, x = f.read()
    f.close()
    return dict(records=rec, x=x)
