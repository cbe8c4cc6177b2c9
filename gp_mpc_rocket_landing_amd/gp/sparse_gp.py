"""FITC sparse GP surfaces of reference src/gp/sparse_gp.py on the GPU.

SparseGP.fit -> gpmpc_fitc_fit: K_uu + jitter I -> L_uu, A = L_uu^-1 K_uf,
Lambda = max(sigma2 - colsum(A^2) + sigma_n^2, 1e-10), B = I + A Lambda^-1 A^T
-> L_B, alpha, FITC LML (sparse_gp.py:150-219); predict -> gpmpc_fitc_predict
(mean as written; variance sigma2 - |v|^2 + |w|^2, sparse_gp.py:
255-305).  Inducing points are chosen on the host exactly like the reference
(scipy kmeans2 on the global RNG, random-subset fallback, sparse_gp.py:122-148);
MultiOutputSparseGP shares them and fits all outputs with one device call.
method="vfe" -> gpmpc_vfe_fit: B = K_uu + K_uf K_fu / sigma_n^2 + jitter I -> L_B,
alpha = B^-1 K_uf y / sigma_n^2, the VFE bound (sparse_gp.py:221-249); the
reference predicts both methods with one body, and so does the device handle.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
from scipy.cluster.vq import kmeans2

from .. import _lib
from .exact_gp import GPPrediction, _spec
from .kernels import Kernel, SquaredExponentialARD


class SparseGP:
    """sparse_gp.py:39-388."""

    def __init__(self, kernel: Kernel, n_inducing: int = 50, noise_variance: float = 1e-4,
                 method: str = "fitc", inducing_points: Optional[np.ndarray] = None,
                 jitter: float = 1e-6):
        self.kernel = kernel
        self.n_inducing = n_inducing
        self._noise_variance = noise_variance
        self.method = method
        self.jitter = jitter
        self._Z = inducing_points
        self.X_train: Optional[np.ndarray] = None
        self.y_train: Optional[np.ndarray] = None
        self.n_train = 0
        self._y_mean, self._y_std = 0.0, 1.0
        self._dev = None
        self._col = 0
        self._log_marginal_likelihood: Optional[float] = None

    @property
    def inducing_points(self):
        return self._Z

    @property
    def noise_variance(self) -> float:
        return self._noise_variance

    @noise_variance.setter
    def noise_variance(self, value: float) -> None:
        self._noise_variance = value
        self._invalidate_cache()

    def _invalidate_cache(self) -> None:
        self._dev = None
        self._log_marginal_likelihood = None

    def _initialize_inducing_points(self, X) -> np.ndarray:
        """sparse_gp.py:122-148."""
        n = X.shape[0]
        if n <= self.n_inducing:
            return X.copy()
        try:
            Z, _ = kmeans2(X, self.n_inducing, minit="points")
        except Exception:
            idx = np.random.choice(n, self.n_inducing, replace=False)
            Z = X[idx].copy()
        return Z

    def fit(self, X, y) -> "SparseGP":
        if self.method not in ("fitc", "vfe"):
            raise ValueError(f"method must be 'fitc' or 'vfe', got {self.method!r}")
        X = np.atleast_2d(X)
        y = np.atleast_1d(y).flatten()
        if self._Z is None:
            self._Z = self._initialize_inducing_points(X)
        h = _lib.FITCHandle(_lib.default_context(), self._Z, X, y[:, None], *_sparse_kernel(self.kernel),
                            self._noise_variance, self.jitter, method=self.method)
        self._attach(X, y, h, 0)
        return self

    def _attach(self, X, y, h, col):
        self.X_train = X
        self.n_train = X.shape[0]
        self._y_mean, self._y_std = float(h.y_mean[col]), float(h.y_std[col])
        self.y_train = (y - self._y_mean) / self._y_std
        self._dev, self._col = h, col
        self._log_marginal_likelihood = float(h.lml[col])

    def predict(self, X, return_std: bool = True) -> GPPrediction:
        if self._dev is None:
            raise RuntimeError("Must call fit() before predict()")
        mean, var = self._dev.predict(np.atleast_2d(X))
        mean = mean[:, self._col].copy()
        if return_std:
            v = var[:, self._col].copy()
            return GPPrediction(mean=mean, variance=v, std=np.sqrt(v))
        return GPPrediction(mean=mean, variance=np.zeros_like(mean), std=np.zeros_like(mean))

    def predict_f(self, X) -> Tuple[np.ndarray, np.ndarray]:
        pred = self.predict(X, return_std=True)
        return pred.mean, pred.variance

    @property
    def log_marginal_likelihood(self) -> float:
        if self._log_marginal_likelihood is None:
            raise RuntimeError("Must call fit() first")
        return self._log_marginal_likelihood

    def update(self, X_new, y_new) -> "SparseGP":
        """sparse_gp.py:328-353: refit on the concatenated data (same Z)."""
        if self.X_train is None:
            return self.fit(X_new, y_new)
        y_den = self.y_train * self._y_std + self._y_mean
        X_all = np.vstack([self.X_train, np.atleast_2d(X_new)])
        y_all = np.concatenate([y_den, np.atleast_1d(y_new)])
        return self.fit(X_all, y_all)

    def __repr__(self) -> str:
        return f"SparseGP(n_train={self.n_train}, n_inducing={self.n_inducing}, method={self.method})"


def _sparse_kernel(kernel):
    """(ls, sigma2) of FITCHandle: the SE-ARD fast path, or any other kernel as its
    device program (sparse_gp.py:182-183 takes any Kernel) with sigma2 unused."""
    kind, ls, s2 = _spec(kernel)
    if kind == _lib.SE_ARD:
        return ls, s2
    return kernel.device_program(), None


class _SharedFITC:
    def __init__(self, h):
        self.h = h
        self.y_mean, self.y_std, self.lml = h.y_mean, h.y_std, h.lml
        self._key = None
        self._val = None

    def predict(self, Xq):
        Xq = np.ascontiguousarray(Xq, dtype=np.float64)
        key = (Xq.shape, Xq.tobytes())
        if key != self._key:
            self._val = self.h.predict(Xq)
            self._key = key
        return self._val


class MultiOutputSparseGP:
    """sparse_gp.py:391-508."""

    def __init__(self, input_dim: int, output_dim: int, n_inducing: int = 50,
                 noise_variance: float = 1e-4, share_inducing: bool = True):
        self.input_dim, self.output_dim = input_dim, output_dim
        self.n_inducing = n_inducing
        self.share_inducing = share_inducing
        self.gps: list[SparseGP] = [SparseGP(SquaredExponentialARD(input_dim), n_inducing, noise_variance)
                                    for _ in range(output_dim)]

    def fit(self, X, Y) -> "MultiOutputSparseGP":
        X = np.atleast_2d(X)
        Y = np.atleast_2d(Y)
        if Y.shape[1] != self.output_dim:
            Y = Y.T
        if self.share_inducing:
            Z = self.gps[0]._initialize_inducing_points(X)
            for gp in self.gps:
                gp._Z = Z.copy()
            g0 = self.gps[0]
            h = _SharedFITC(_lib.FITCHandle(_lib.default_context(), Z, X, Y, *_sparse_kernel(g0.kernel),
                                            g0.noise_variance, g0.jitter))
            for i, gp in enumerate(self.gps):
                gp._attach(X, Y[:, i], h, i)
        else:
            for i, gp in enumerate(self.gps):
                gp.fit(X, Y[:, i])
        return self

    def predict(self, X) -> Tuple[np.ndarray, np.ndarray]:
        X = np.atleast_2d(X)
        means = np.zeros((X.shape[0], self.output_dim))
        variances = np.zeros((X.shape[0], self.output_dim))
        for i, gp in enumerate(self.gps):
            pred = gp.predict(X)
            means[:, i] = pred.mean
            variances[:, i] = pred.variance
        return means, variances

    def predict_f(self, X):
        return self.predict(X)

    @property
    def device_handle(self):
        """The shared device FITC GP (None before fit or with share_inducing=False)."""
        d = self.gps[0]._dev
        return d.h if isinstance(d, _SharedFITC) and all(g._dev is d for g in self.gps) else None

    def update(self, X_new, Y_new) -> "MultiOutputSparseGP":
        Y_new = np.atleast_2d(Y_new)
        if Y_new.shape[1] != self.output_dim:
            Y_new = Y_new.T
        for i, gp in enumerate(self.gps):
            gp.update(X_new, Y_new[:, i])
        return self

    def __repr__(self) -> str:
        return (f"MultiOutputSparseGP(input_dim={self.input_dim}, output_dim={self.output_dim}, "
                f"n_inducing={self.n_inducing})")
