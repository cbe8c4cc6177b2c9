"""Simple3DoFGP: the GP surface of the 3-DoF GP-MPC (structured_gp.py:414-496).

Same construction, data handling and error behaviour as the reference; the
multi-output GP underneath is the device one (exact: one shared Gram +
Cholesky for the three outputs; sparse: one FITC fit with shared inducing
points).  ``predict_batch`` evaluates many (x, u) pairs -- e.g. a whole MPC
horizon -- in one device call.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .exact_gp import MultiOutputExactGP
from .features import Simple3DoFFeatureExtractor
from .sparse_gp import MultiOutputSparseGP


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
        if self.n_data == 0:
            raise RuntimeError("No data")
        X = np.array(self.X_data); U = np.array(self.U_data); D = np.array(self.D_data)
        Z = self.feature_extractor.extract_batch(X, U)
        self.gp.fit(Z, D)
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
