"""Synthetic, seeded inputs for the GP + QP hot path (generator G).

There is no dataset in the reference (and no network), so training data for the
residual GP are drawn from the envelope of the Monte-Carlo landings of
scripts/run_experiments.py:359-371, and the learned residual is the aero drag
of experiments/dispersion.py:349-360 (rho = 0.02, Cd = A = 1, applied when
|v| > 1) expressed as an acceleration, plus N(0, 0.01^2) noise.
"""
from __future__ import annotations

import numpy as np

DRAG_RHO, DRAG_CD, DRAG_A = 0.02, 1.0, 1.0


def drag_accel(X):
    """Aero residual (N, 3) of dispersion.py:349-360 for states X (N, 7)."""
    X = np.atleast_2d(X)
    v = X[:, 4:7]
    speed = np.sqrt(np.sum(v * v, axis=1))
    safe = np.where(speed > 1.0, speed, 1.0)
    drag = 0.5 * DRAG_RHO * DRAG_CD * DRAG_A * speed ** 2
    acc = -(drag / X[:, 0])[:, None] * (v / safe[:, None])
    return np.where((speed > 1.0)[:, None], acc, 0.0)


def synthetic_training_data(n=1000, seed=0, noise_seed=1):
    """Generator G: (X (n,7), U (n,3), D (n,3)) fp64."""
    rs = np.random.RandomState(seed)
    m = rs.uniform(1.0, 2.0, n)
    rx = rs.uniform(0.0, 100.0, n)
    ry = rs.normal(0.0, 3.0, n)
    rz = rs.normal(0.0, 3.0, n)
    vx = rs.normal(-3.0, 1.0, n)
    vy = rs.normal(0.0, 0.5, n)
    vz = rs.normal(0.0, 0.5, n)
    u0 = rs.uniform(0.3, 5.0, n)
    u1 = rs.normal(0.0, 0.5, n)
    u2 = rs.normal(0.0, 0.5, n)
    X = np.stack([m, rx, ry, rz, vx, vy, vz], axis=1)
    U = np.stack([u0, u1, u2], axis=1)
    D = drag_accel(X) + np.random.RandomState(noise_seed).normal(0.0, 0.01, (n, 3))
    return X, U, D


def synthetic_6dof_training_data(n=300, seed=0, noise_seed=1):
    """6-DoF analogue for StructuredRocketGP (x = [m, r(3), v(3), q(4), w(3)]):
    (X (n,14), U (n,3), D_v (n,3), D_w (n,3))."""
    rs = np.random.RandomState(seed)
    X3, U, D = synthetic_training_data(n, seed, noise_seed)
    q = rs.normal(0.0, 0.05, (n, 4))
    q[:, 0] += 1.0
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    w = rs.normal(0.0, 0.1, (n, 3))
    X = np.concatenate([X3, q, w], axis=1)
    Dw = -0.05 * w + np.random.RandomState(noise_seed + 1).normal(0.0, 0.01, (n, 3))
    return X, U, D, Dw


def query_points(X, U, p, seed=7):
    """Rows of the training envelope used as kernel-bench queries."""
    idx = np.random.RandomState(seed).choice(X.shape[0], p, replace=p > X.shape[0])
    return X[idx].copy(), U[idx].copy()
