"""Physics features for the residual GPs (reference src/gp/features.py).

Host-side preprocessing of the GP inputs (the per-step features of the
closed-loop path are computed on the device inside the fleet step).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np


@dataclass
class AtmosphereModel:
    """features.py:46-63: rho(h) = rho0 exp(-h/H)."""
    rho_0: float = 1.225
    scale_height: float = 8500.0

    def density(self, altitude):
        return self.rho_0 * np.exp(-altitude / self.scale_height)

    def density_array(self, altitude):
        return self.rho_0 * np.exp(-np.asarray(altitude) / self.scale_height)


def _dcm(q):
    """Body-from-inertial DCM of quaternions [w, x, y, z] (features.py:265-270), (P,3,3)."""
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y + w * z), 2 * (x * z - w * y)], -1),
        np.stack([2 * (x * y - w * z), 1 - 2 * (x * x + z * z), 2 * (y * z + w * x)], -1),
        np.stack([2 * (x * z + w * y), 2 * (y * z - w * x), 1 - 2 * (x * x + y * y)], -1),
    ], axis=1)


class RocketFeatureExtractor:
    """features.py:71-146: extract(x, u) for one point, extract_batch(X, U) for many."""

    _names: List[str] = []

    def __init__(self, atmosphere: Optional[AtmosphereModel] = None, include_altitude=True,
                 include_density=True, reference_velocity=10.0):
        self.atmosphere = atmosphere or AtmosphereModel()
        self.include_altitude = include_altitude
        self.include_density = include_density
        self.v_ref = reference_velocity

    @property
    def feature_names(self):
        return list(self._names)

    @property
    def n_features(self):
        return len(self._names)

    def extract(self, x, u):
        return self.extract_batch(np.atleast_2d(x), np.atleast_2d(u))[0]

    def _common(self, X):
        alt = X[:, 1]; v = X[:, 4:7]
        speed = np.sqrt(np.sum(v * v, axis=1))
        rho = self.atmosphere.density_array(alt)
        qn = (0.5 * rho * speed ** 2) / (0.5 * self.atmosphere.rho_0 * self.v_ref ** 2)
        return alt, v, speed, rho, qn


class Simple3DoFFeatureExtractor(RocketFeatureExtractor):
    """features.py:368-444: [v/10, |v|/10, q_dyn, u/10, |u|/10, alt/100, rho/rho0]."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._names = ["v_x", "v_y", "v_z", "speed", "q_dyn", "T_x", "T_y", "T_z", "T_mag"]
        if self.include_altitude:
            self._names.append("altitude")
        if self.include_density:
            self._names.append("density")

    def extract_batch(self, X, U):
        X = np.atleast_2d(np.asarray(X, float)); U = np.atleast_2d(np.asarray(U, float))
        alt, v, speed, rho, qn = self._common(X)
        tm = np.sqrt(np.sum(U * U, axis=1))
        cols = [v[:, 0] / self.v_ref, v[:, 1] / self.v_ref, v[:, 2] / self.v_ref,
                speed / self.v_ref, qn, U[:, 0] / 10.0, U[:, 1] / 10.0, U[:, 2] / 10.0, tm / 10.0]
        if self.include_altitude:
            cols.append(alt / 100.0)
        if self.include_density:
            cols.append(rho / self.atmosphere.rho_0)
        return np.stack(cols, axis=1)


class TranslationalFeatureExtractor(RocketFeatureExtractor):
    """features.py:149-270: 13 features for d_v (6-DoF state)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._names = ["v_x", "v_y", "v_z", "speed", "q_dyn", "alpha", "beta", "T_x", "T_y",
                       "T_z", "T_mag"]
        if self.include_altitude:
            self._names.append("altitude")
        if self.include_density:
            self._names.append("density")

    def extract_batch(self, X, U):
        X = np.atleast_2d(np.asarray(X, float)); U = np.atleast_2d(np.asarray(U, float))
        alt, v, speed, rho, qn = self._common(X)
        vB = np.einsum("pij,pj->pi", _dcm(X[:, 7:11]), v)
        moving = speed > 1e-3
        aoa = np.where(moving, np.arctan2(-vB[:, 2], vB[:, 0]), 0.0)
        beta = np.where(moving, np.arcsin(np.clip(vB[:, 1] / np.where(moving, speed, 1.0), -1, 1)), 0.0)
        tm = np.sqrt(np.sum(U * U, axis=1))
        cols = [v[:, 0] / self.v_ref, v[:, 1] / self.v_ref, v[:, 2] / self.v_ref,
                speed / self.v_ref, qn, aoa, beta, U[:, 0] / 10.0, U[:, 1] / 10.0,
                U[:, 2] / 10.0, tm / 10.0]
        if self.include_altitude:
            cols.append(alt / 100.0)
        if self.include_density:
            cols.append(rho / self.atmosphere.rho_0)
        return np.stack(cols, axis=1)


class RotationalFeatureExtractor(RocketFeatureExtractor):
    """features.py:273-365: 12 features for d_omega."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._names = ["omega_x", "omega_y", "omega_z", "omega_mag", "T_x", "T_y", "T_z",
                       "v_Bx", "v_By", "v_Bz", "speed", "q_dyn"]

    def extract_batch(self, X, U):
        X = np.atleast_2d(np.asarray(X, float)); U = np.atleast_2d(np.asarray(U, float))
        alt, v, speed, rho, qn = self._common(X)
        w = X[:, 11:14]
        wm = np.sqrt(np.sum(w * w, axis=1))
        vB = np.einsum("pij,pj->pi", _dcm(X[:, 7:11]), v)
        cols = [w[:, 0], w[:, 1], w[:, 2], wm, U[:, 0] / 10.0, U[:, 1] / 10.0, U[:, 2] / 10.0,
                vB[:, 0] / self.v_ref, vB[:, 1] / self.v_ref, vB[:, 2] / self.v_ref,
                speed / self.v_ref, qn]
        return np.stack(cols, axis=1)


class CombinedFeatureExtractor:
    """features.py:447-491."""

    def __init__(self, atmosphere=None, reference_velocity=10.0):
        self.translational = TranslationalFeatureExtractor(atmosphere=atmosphere,
                                                           reference_velocity=reference_velocity)
        self.rotational = RotationalFeatureExtractor(atmosphere=atmosphere,
                                                     reference_velocity=reference_velocity)

    @property
    def n_features_translational(self):
        return self.translational.n_features

    @property
    def n_features_rotational(self):
        return self.rotational.n_features

    def extract_translational(self, x, u):
        return self.translational.extract(x, u)

    def extract_rotational(self, x, u):
        return self.rotational.extract(x, u)

    def extract_batch_translational(self, X, U):
        return self.translational.extract_batch(X, U)

    def extract_batch_rotational(self, X, U):
        return self.rotational.extract_batch(X, U)
