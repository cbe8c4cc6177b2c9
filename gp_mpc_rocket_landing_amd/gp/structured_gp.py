"""Structured GPs: the 6-DoF StructuredRocketGP (structured_gp.py:43-411) and
the 3-DoF Simple3DoFGP (structured_gp.py:414-496).

Same construction, data handling and error behaviour as the reference; the
multi-output GPs underneath are the device ones (exact: one shared Gram +
Cholesky for the three outputs; sparse: one FITC fit with shared inducing
points).  ``predict_batch`` evaluates many (x, u) pairs -- e.g. a whole MPC
horizon -- in one device call per residual group.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass
from typing import Any, Dict, Optional, Tuple

import numpy as np

from .exact_gp import MultiOutputExactGP
from .features import AtmosphereModel, CombinedFeatureExtractor, Simple3DoFFeatureExtractor
from .sparse_gp import MultiOutputSparseGP


@dataclass
class StructuredGPConfig:
    """structured_gp.py:43-63 (same fields and defaults)."""
    n_inducing: int = 50
    noise_variance: float = 1e-4
    use_sparse: bool = True
    reference_velocity: float = 10.0
    include_altitude: bool = True
    include_density: bool = True
    signal_variance: float = 0.1
    lengthscales_translational: Optional[np.ndarray] = None
    lengthscales_rotational: Optional[np.ndarray] = None
    max_data_points: int = 1000
    novelty_threshold: float = 0.1


class StructuredRocketGP:
    """6-DoF physics-structured GP: d_v (13 translational features) and d_omega
    (12 rotational features), three outputs each (structured_gp.py:66-411).

    As in the reference, the SE-ARD kernels built from ``signal_variance`` and
    the configured length-scales are not handed to the multi-output GPs
    (structured_gp.py:117-129, ``noqa: F841``): both GPs use their default
    unit kernels, and ``signal_variance`` only sets the unfitted prior.
    """

    def __init__(self, config: Optional[StructuredGPConfig] = None):
        self.config = config or StructuredGPConfig()
        self.feature_extractor = CombinedFeatureExtractor(atmosphere=AtmosphereModel(),
                                                          reference_velocity=self.config.reference_velocity)
        n_v = self.feature_extractor.n_features_translational
        n_w = self.feature_extractor.n_features_rotational
        if self.config.use_sparse:
            self.gp_v = MultiOutputSparseGP(input_dim=n_v, output_dim=3, n_inducing=self.config.n_inducing,
                                            noise_variance=self.config.noise_variance)
            self.gp_omega = MultiOutputSparseGP(input_dim=n_w, output_dim=3,
                                                n_inducing=self.config.n_inducing,
                                                noise_variance=self.config.noise_variance)
        else:
            self.gp_v = MultiOutputExactGP(input_dim=n_v, output_dim=3,
                                           noise_variance=self.config.noise_variance)
            self.gp_omega = MultiOutputExactGP(input_dim=n_w, output_dim=3,
                                               noise_variance=self.config.noise_variance)
        self.X_data: list = []
        self.U_data: list = []
        self.D_v_data: list = []
        self.D_omega_data: list = []
        self._is_fitted = False

    @property
    def n_data(self) -> int:
        return len(self.X_data)

    def add_data(self, X, U, D_v, D_omega) -> None:
        """structured_gp.py:170-204: append, then keep the newest max_data_points."""
        X = np.atleast_2d(X); U = np.atleast_2d(U)
        D_v = np.atleast_2d(D_v); D_omega = np.atleast_2d(D_omega)
        for i in range(X.shape[0]):
            self.X_data.append(X[i])
            self.U_data.append(U[i])
            self.D_v_data.append(D_v[i])
            self.D_omega_data.append(D_omega[i])
        excess = len(self.X_data) - self.config.max_data_points
        if excess > 0:
            self.X_data = self.X_data[excess:]
            self.U_data = self.U_data[excess:]
            self.D_v_data = self.D_v_data[excess:]
            self.D_omega_data = self.D_omega_data[excess:]
        self._is_fitted = False

    def fit(self) -> None:
        """structured_gp.py:206-223."""
        if self.n_data == 0:
            raise RuntimeError("No data to fit")
        X = np.array(self.X_data); U = np.array(self.U_data)
        Z_v = self.feature_extractor.extract_batch_translational(X, U)
        Z_w = self.feature_extractor.extract_batch_rotational(X, U)
        self.gp_v.fit(Z_v, np.array(self.D_v_data))
        self.gp_omega.fit(Z_w, np.array(self.D_omega_data))
        self._is_fitted = True

    def _ensure_fitted(self) -> bool:
        if not self._is_fitted:
            if self.n_data == 0:
                return False
            self.fit()
        return True

    def predict(self, x, u) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """structured_gp.py:225-268 -> (d_v mean, d_omega mean, d_v var, d_omega var), each (3,)."""
        if not self._ensure_fitted():
            zero = np.zeros(3)
            prior = np.full(3, self.config.signal_variance)
            return zero, zero, prior, prior
        z_v = self.feature_extractor.extract_translational(x, u)
        z_w = self.feature_extractor.extract_rotational(x, u)
        mv, vv = self.gp_v.predict(z_v.reshape(1, -1))
        mw, vw = self.gp_omega.predict(z_w.reshape(1, -1))
        return mv.flatten(), mw.flatten(), vv.flatten(), vw.flatten()

    def predict_batch(self, X, U) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """structured_gp.py:270-305 -> four (P, 3) arrays; one device call per residual group."""
        X = np.atleast_2d(X); U = np.atleast_2d(U)
        if not self._ensure_fitted():
            zero = np.zeros((X.shape[0], 3))
            prior = np.full((X.shape[0], 3), self.config.signal_variance)
            return zero, zero, prior, prior
        Z_v = self.feature_extractor.extract_batch_translational(X, U)
        Z_w = self.feature_extractor.extract_batch_rotational(X, U)
        mv, vv = self.gp_v.predict(Z_v)
        mw, vw = self.gp_omega.predict(Z_w)
        return mv, mw, vv, vw

    def get_full_residual(self, x, u) -> Tuple[np.ndarray, np.ndarray]:
        """structured_gp.py:307-338: the 6 residuals placed on v-dot (4:7) and omega-dot (11:14)."""
        mv, mw, vv, vw = self.predict(x, u)
        d_mean = np.zeros(14); d_var = np.zeros(14)
        d_mean[4:7] = mv; d_mean[11:14] = mw
        d_var[4:7] = vv; d_var[11:14] = vw
        return d_mean, d_var

    def is_novel(self, x, u) -> bool:
        """structured_gp.py:340-359."""
        _, _, vv, vw = self.predict(x, u)
        return bool(max(np.max(vv), np.max(vw)) > self.config.novelty_threshold * self.config.signal_variance)

    def optimize_hyperparameters(self) -> Dict[str, Any]:
        """structured_gp.py:361-373 (the reference returns its state; no optimisation)."""
        return {"n_data": self.n_data, "is_fitted": self._is_fitted}

    def save(self, path: str) -> None:
        """structured_gp.py:375-392, as a pickle-free ``.npz``: the data arrays and the
        config as JSON (the reference's ``np.save(allow_pickle=True)`` is not used)."""
        cfg = {k: (v.tolist() if isinstance(v, np.ndarray) else v)
               for k, v in dataclasses.asdict(self.config).items()}
        with open(path, "wb") as fh:   # keep the caller's path verbatim (np.savez would add .npz)
            np.savez(fh, X=np.array(self.X_data).reshape(-1, 14), U=np.array(self.U_data).reshape(-1, 3),
                     D_v=np.array(self.D_v_data).reshape(-1, 3), D_omega=np.array(self.D_omega_data).reshape(-1, 3),
                     is_fitted=np.array(self._is_fitted), config=np.array(json.dumps(cfg)))

    def load(self, path: str) -> None:
        """structured_gp.py:394-406: restore the data, refit if the saved model was fitted."""
        with np.load(path, allow_pickle=False) as d:
            self.X_data = list(d["X"]); self.U_data = list(d["U"])
            self.D_v_data = list(d["D_v"]); self.D_omega_data = list(d["D_omega"])
            fitted = bool(d["is_fitted"])
        self._is_fitted = False
        if fitted:
            self.fit()

    def __repr__(self) -> str:
        return (f"StructuredRocketGP(n_data={self.n_data}, n_inducing={self.config.n_inducing}, "
                f"fitted={self._is_fitted})")


class Simple3DoFGP:
    def __init__(self, n_inducing: int = 50, noise_variance: float = 1e-4, use_sparse: bool = True):
        self.feature_extractor = Simple3DoFFeatureExtractor()
        n_feat = self.feature_extractor.n_features
        self.use_sparse = use_sparse
        if use_sparse:
            self.gp = MultiOutputSparseGP(input_dim=n_feat, output_dim=3, n_inducing=n_inducing,
                                          noise_variance=noise_variance)
        else:
            self.gp = MultiOutputExactGP(input_dim=n_feat, output_dim=3, noise_variance=noise_variance)
        self.X_data: list = []
        self.U_data: list = []
        self.D_data: list = []
        self._is_fitted = False

    @property
    def n_data(self) -> int:
        return len(self.X_data)

    def add_data(self, X, U, D) -> None:
        X = np.atleast_2d(X); U = np.atleast_2d(U); D = np.atleast_2d(D)
        for i in range(X.shape[0]):
            self.X_data.append(X[i])
            self.U_data.append(U[i])
            self.D_data.append(D[i])
        self._is_fitted = False

    def fit(self) -> None:
        """structured_gp.py:470-481.  With the exact GP, a refit after add_data
        only appended rows grows the device factor in O(n^2 k) (gpmpc_gp_append,
        SURVEY 8f-4) -- the same GP as the full refit, which remains the
        fallback (first fit, jitter, indefinite Schur complement)."""
        if self.n_data == 0:
            raise RuntimeError("No data")
        X = np.array(self.X_data); U = np.array(self.U_data); D = np.array(self.D_data)
        n_old = getattr(self, "_n_fitted", 0)
        if (not self.use_sparse and 0 < n_old < self.n_data
                and self.gp.device_handle is not None and self.gp.device_handle.n == n_old):
            Znew = self.feature_extractor.extract_batch(X[n_old:], U[n_old:])
            self.gp.update(Znew, D[n_old:])
        else:
            Z = self.feature_extractor.extract_batch(X, U)
            self.gp.fit(Z, D)
        self._n_fitted = self.n_data
        self._is_fitted = True

    def predict(self, x, u) -> Tuple[np.ndarray, np.ndarray]:
        if not self._is_fitted:
            if self.n_data > 0:
                self.fit()
            else:
                return np.zeros(3), np.ones(3) * 0.1
        z = self.feature_extractor.extract(x, u)
        mean, var = self.gp.predict(z.reshape(1, -1))
        return mean.flatten(), var.flatten()

    def predict_batch(self, X, U) -> Tuple[np.ndarray, np.ndarray]:
        """(P, 7), (P, 3) -> means (P, 3), variances (P, 3) in one device call."""
        X = np.atleast_2d(X); U = np.atleast_2d(U)
        if not self._is_fitted:
            if self.n_data > 0:
                self.fit()
            else:
                return np.zeros((X.shape[0], 3)), np.full((X.shape[0], 3), 0.1)
        return self.gp.predict(self.feature_extractor.extract_batch(X, U))

    def __repr__(self) -> str:
        return f"Simple3DoFGP(n_data={self.n_data}, fitted={self._is_fitted})"
