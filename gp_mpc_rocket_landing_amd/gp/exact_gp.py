"""Exact GP surfaces of reference src/gp/exact_gp.py on the GPU.

ExactGP.fit -> gpmpc_gp_fit_exact: normalisation (population std, floor
1e-10 -> 1), Gram of the training set, K + sigma_n^2 I, Cholesky with the
exact_gp.py:163-175 jitter ladder, alpha = L^-T L^-1 y, LML, and W = L^-1 for
the posterior variance -- all on device.  ExactGP.predict -> gpmpc_gp_predict
(K*, mean, variance |L^-1 K*^T|^2 via the FP64-MFMA GEMM).  The handle keeps
L, alpha and the scaled training inputs resident in HBM.

MultiOutputExactGP fits every output with ONE Gram + ONE Cholesky when the
per-output kernels and noise are identical (the default construction; SURVEY
D13) -- the reference repeats both per output.

ExactGP.optimize_hyperparameters keeps the reference's L-BFGS-B
with finite-difference gradients, but evaluates f(x) and the n_params probes
f(x + h e_i) of each gradient as ONE batched device call
(gpmpc_gp_lml_batched: all Grams, one batched Cholesky, batched triangular
solves).

Any Kernel can be fitted, as in the reference (exact_gp.py:157): the four
stationary kernels take the fast device Gram, composites (SumKernel,
ProductKernel, WhiteNoise) their device program (Kernel.device_program,
gpmpc_gp_fit_exact_prog).  Not on this path: mean_function /
normalize_y=False (NotImplementedError).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from .. import _lib
from .kernels import Kernel, SquaredExponentialARD


@dataclass
class GPPrediction:
    """exact_gp.py:33-44."""
    mean: np.ndarray
    variance: np.ndarray
    std: np.ndarray

    @property
    def confidence_bounds(self) -> Tuple[np.ndarray, np.ndarray]:
        return self.mean - 1.96 * self.std, self.mean + 1.96 * self.std


def _spec(kernel: Kernel):
    """(kind, lengthscales, sigma2) of a stationary kernel, or (KernelProgram, None,
    None) for any other (composite) kernel: ExactGPHandle / FITCHandle take either."""
    spec = kernel._device_spec()
    if spec is None:
        return kernel.device_program(), None, None
    return spec


class _Shared:
    """A device GP fitted for several outputs at once (column j = output j)."""

    def __init__(self, handle: _lib.ExactGPHandle):
        self.h = handle
        self._cache_key = None
        self._cache = None

    def predict(self, Xq):
        Xq = np.ascontiguousarray(np.atleast_2d(Xq), dtype=np.float64)
        key = (Xq.shape, Xq.tobytes())
        if key != self._cache_key:  # one device call serves every output
            self._cache = self.h.predict(Xq)
            self._cache_key = key
        return self._cache


class ExactGP:
    """exact_gp.py:47-424."""

    def __init__(self, kernel: Kernel, noise_variance: float = 1e-4,
                 mean_function=None, normalize_y: bool = True):
        self.kernel = kernel
        self._noise_variance = noise_variance
        self.mean_function = mean_function
        self.normalize_y = normalize_y
        self.X_train: Optional[np.ndarray] = None
        self.y_train: Optional[np.ndarray] = None
        self.n_train = 0
        self._y_mean, self._y_std = 0.0, 1.0
        self._dev: Optional[_Shared] = None
        self._col = 0
        self._log_marginal_likelihood: Optional[float] = None
        self.jitter_steps = 0

    @property
    def noise_variance(self) -> float:
        return self._noise_variance

    @noise_variance.setter
    def noise_variance(self, value: float) -> None:
        assert value > 0, "Noise variance must be positive"
        self._noise_variance = value
        self._invalidate_cache()

    def _invalidate_cache(self) -> None:
        self._dev = None
        self._log_marginal_likelihood = None

    def _check_supported(self):
        if self.mean_function is not None or not self.normalize_y:
            raise NotImplementedError("mean_function / normalize_y=False are not on the device path")

    def fit(self, X, y) -> "ExactGP":
        """exact_gp.py:118-184 (ValueError when the jitter ladder is exhausted)."""
        self._check_supported()
        X = np.atleast_2d(X)
        y = np.atleast_1d(y).flatten()
        assert X.shape[0] == len(y), "X and y must have same number of samples"
        kind, ls, s2 = _spec(self.kernel)
        h = _lib.ExactGPHandle(_lib.default_context(), kind, X, y[:, None], ls, s2, self._noise_variance)
        self._attach(X, y, _Shared(h), 0)
        return self

    def _attach(self, X, y, shared: _Shared, col: int):
        h = shared.h
        self.X_train = X
        self.n_train = X.shape[0]
        self._y_mean, self._y_std = float(h.y_mean[col]), float(h.y_std[col])
        self.y_train = (y - self._y_mean) / self._y_std
        self._dev, self._col = shared, col
        self._log_marginal_likelihood = float(h.lml[col])
        self.jitter_steps = h.jitter_steps

    @property
    def log_marginal_likelihood(self) -> float:
        if self._log_marginal_likelihood is None:
            raise RuntimeError("Must call fit() before accessing log_marginal_likelihood")
        return self._log_marginal_likelihood

    @property
    def _L(self):
        """Cholesky factor of K + sigma_n^2 I (+ jitter), copied from the device."""
        if self._dev is None:
            return None
        return self._dev.h.state()[0]

    @property
    def _alpha(self):
        if self._dev is None:
            return None
        return self._dev.h.state()[1][:, self._col]

    def predict(self, X, return_std: bool = True, return_cov: bool = False):
        """exact_gp.py:213-268."""
        if self._dev is None:
            raise RuntimeError("Must call fit() before predict()")
        X = np.atleast_2d(X)
        if return_cov:
            mean, cov = self._dev.h.predict_cov(X)
            return mean[:, self._col], cov * self._y_std ** 2
        mean, var = self._dev.predict(X)
        mean = mean[:, self._col].copy()
        if return_std:
            v = var[:, self._col].copy()
            return GPPrediction(mean=mean, variance=v, std=np.sqrt(v))
        return GPPrediction(mean=mean, variance=np.zeros_like(mean), std=np.zeros_like(mean))

    def predict_f(self, X) -> Tuple[np.ndarray, np.ndarray]:
        pred = self.predict(X, return_std=True)
        return pred.mean, pred.variance

    def sample_prior(self, X, n_samples: int = 1, random_state: Optional[int] = None):
        """exact_gp.py:289-322 (Gram and Cholesky on the device)."""
        if random_state is not None:
            np.random.seed(random_state)
        X = np.atleast_2d(X)
        K = self.kernel(X) + 1e-10 * np.eye(X.shape[0])
        L, info = _lib.potrf(_lib.default_context(), K)
        if info:
            raise np.linalg.LinAlgError("Matrix is not positive definite")
        return (L @ np.random.randn(X.shape[0], n_samples)).T

    def sample_posterior(self, X, n_samples: int = 1, random_state: Optional[int] = None):
        """exact_gp.py:324-355."""
        if self._dev is None:
            raise RuntimeError("Must call fit() before sample_posterior()")
        if random_state is not None:
            np.random.seed(random_state)
        mean, cov = self.predict(X, return_cov=True)
        L, info = _lib.potrf(_lib.default_context(), cov + 1e-10 * np.eye(cov.shape[0]))
        if info:
            raise np.linalg.LinAlgError("Matrix is not positive definite")
        return (mean[:, None] + L @ np.random.randn(np.atleast_2d(X).shape[0], n_samples)).T

    def update(self, X_new, y_new) -> "ExactGP":
        """Refit on the concatenated data (the SparseGP.update semantics,
        sparse_gp.py:328-353), done incrementally on the device when possible
        (gpmpc_gp_append, SURVEY 8f-4: O(n^2 k) instead of O(n^3)); a GP fitted
        with jitter or an indefinite Schur complement falls back to the refit."""
        if self._dev is None:
            return self.fit(X_new, y_new)
        X_new = np.atleast_2d(X_new)
        y_new = np.atleast_1d(y_new).flatten()
        X = np.vstack([self.X_train, X_new])
        y = np.concatenate([self.y_train * self._y_std + self._y_mean, y_new])
        h = self._dev.h
        if h.n_out == 1 and h.append(X_new, y[:, None]):
            self._dev._cache_key = None
            self._attach(X, y, self._dev, 0)
            return self
        return self.fit(X, y)

    def _lml_batch(self, P, X, y):
        """Log marginal likelihoods at the rows of P = [kernel params (log
        space, kernels.py:320-371 order), log noise] -- the objective of
        exact_gp.py:375-386 for every row, one device call (a composite
        kernel: one device fit of its program per row)."""
        P = np.atleast_2d(P)
        nk = self.kernel.n_params
        k2 = copy.deepcopy(self.kernel)
        if k2._device_spec() is None:
            lml, steps = np.empty(len(P)), np.empty(len(P), np.int32)
            for i, p in enumerate(P):
                k2.set_params(p[:nk])
                try:
                    h = _lib.ExactGPHandle(_lib.default_context(), k2.device_program(), X, y[:, None], None,
                                           None, float(np.exp(p[nk])))
                    lml[i], steps[i] = h.lml[0], h.jitter_steps
                except ValueError:   # exact_gp.py:383-386: a failed fit is +inf for the optimiser
                    lml[i], steps[i] = -np.inf, -1
                except _lib.HIPError as e:
                    # parameters the device refuses as a kernel program (a lengthscale that
                    # underflowed to 0 from exp(p), a negative variance): the reference's
                    # fit fails on them too (a non-finite Gram), which its objective turns
                    # into +inf; any other device error propagates
                    if e.rc != -2:
                        raise
                    lml[i], steps[i] = -np.inf, -1
            return lml, steps
        kind = None
        ls, s2 = [], []
        for p in P:
            k2.set_params(p[:nk])
            kd, l, s = _spec(k2)
            kind = kd
            ls.append(np.asarray(l, float).reshape(-1)); s2.append(float(s))
        lml, steps = _lib.gp_lml_batched(_lib.default_context(), kind, X, y, np.stack(ls),
                                         np.array(s2), np.exp(P[:, nk]))
        return lml, steps

    def optimize_hyperparameters(self, n_restarts: int = 5, verbose: bool = False) -> dict:
        """exact_gp.py:357-421: maximise the LML over [kernel params, log noise]
        with L-BFGS-B (maxiter 100) from the current parameters, then
        n_restarts - 1 restarts perturbed by 0.5 * np.random.randn (global RNG);
        the best result is set and refitted.  The gradient is scipy's 2-point
        rule with L-BFGS-B's absolute step eps = 1e-8 (scipy/_numdiff.py:
        h = 1e-8, dx = (x + h) - x, g_i = (f(x + dx e_i) - f(x)) / dx), so the
        optimiser sees what the reference's sees; f(x) and the n_params probes
        are one batched device evaluation.  A failed fit (jitter ladder
        exhausted) is +inf, as in the reference."""
        if self.X_train is None:
            raise RuntimeError("Must call fit() before optimize_hyperparameters()")
        from scipy.optimize import minimize
        X = self.X_train
        y = self.y_train * self._y_std + self._y_mean  # what the objective refits with (:382)
        nk = self.kernel.n_params
        eps_fallback = np.finfo(float).eps ** 0.5

        def fun_and_grad(x):
            x = np.asarray(x, float)
            h = np.full(x.size, 1e-8)
            dx = (x + h) - x
            sign = (x >= 0).astype(float) * 2 - 1
            h = np.where(dx == 0, eps_fallback * sign * np.maximum(1.0, np.abs(x)), h)
            P = np.repeat(x[None, :], x.size + 1, axis=0)
            steps = np.empty(x.size)
            for i in range(x.size):
                P[i + 1, i] += h[i]
                steps[i] = P[i + 1, i] - x[i]
            lml, _ = self._lml_batch(P, X, y)
            f = -lml
            with np.errstate(invalid="ignore", over="ignore"):
                g = (f[1:] - f[0]) / steps
            return float(f[0]), g

        initial = np.concatenate([self.kernel.get_params(), [np.log(self._noise_variance)]])
        best_result, best_nll = None, np.inf
        for restart in range(n_restarts):
            params0 = initial if restart == 0 else initial + 0.5 * np.random.randn(len(initial))
            try:
                result = minimize(fun_and_grad, params0, jac=True, method="L-BFGS-B",
                                  options={"maxiter": 100, "disp": verbose})
                if result.fun < best_nll:
                    best_nll, best_result = result.fun, result
            except Exception as e:  # noqa: BLE001  (exact_gp.py:407-409)
                if verbose:
                    print(f"Restart {restart} failed: {e}")
        if best_result is not None:
            self.kernel.set_params(best_result.x[:nk])
            self._noise_variance = float(np.exp(best_result.x[nk]))
            try:
                self.fit(X, y)
            except ValueError:
                self._invalidate_cache()
        return {
            "success": best_result is not None and bool(best_result.success),
            "log_marginal_likelihood": -best_nll if best_result else None,
            "n_iterations": best_result.nit if best_result else 0,
        }

    def __repr__(self) -> str:
        return f"ExactGP(n_train={self.n_train}, kernel={self.kernel!r})"


def _same_kernel(a: Kernel, b: Kernel) -> bool:
    sa, sb = _spec(a), _spec(b)
    if isinstance(sa[0], _lib.KernelProgram) or isinstance(sb[0], _lib.KernelProgram):
        return sa[0] == sb[0]
    return (sa[0] == sb[0] and sa[2] == sb[2]
            and np.array_equal(np.asarray(sa[1]), np.asarray(sb[1])))


class MultiOutputExactGP:
    """exact_gp.py:427-535."""

    def __init__(self, input_dim: int, output_dim: int, kernel: Optional[Kernel] = None,
                 noise_variance: float = 1e-4, share_hyperparameters: bool = False):
        self.input_dim, self.output_dim = input_dim, output_dim
        self.share_hyperparameters = share_hyperparameters
        self.gps: list[ExactGP] = []
        for _ in range(output_dim):
            if kernel is None:
                k = SquaredExponentialARD(input_dim)
            elif share_hyperparameters:
                k = kernel
            else:
                k = SquaredExponentialARD(input_dim)
                k.set_params(kernel.get_params())
            self.gps.append(ExactGP(k, noise_variance=noise_variance))

    def fit(self, X, Y) -> "MultiOutputExactGP":
        X = np.atleast_2d(X)
        Y = np.atleast_2d(Y)
        if Y.shape[1] != self.output_dim:
            if Y.shape[0] == self.output_dim:
                Y = Y.T
            else:
                raise ValueError(f"Y must have {self.output_dim} columns")
        g0 = self.gps[0]
        shared = all(_same_kernel(g0.kernel, g.kernel) and g.noise_variance == g0.noise_variance
                     for g in self.gps)
        if shared:
            for g in self.gps:
                g._check_supported()
            kind, ls, s2 = _spec(g0.kernel)
            h = _Shared(_lib.ExactGPHandle(_lib.default_context(), kind, X, Y, ls, s2, g0.noise_variance))
            for i, g in enumerate(self.gps):
                g._attach(X, Y[:, i], h, i)
        else:
            for i, g in enumerate(self.gps):
                g.fit(X, Y[:, i])
        return self

    def update(self, X_new, Y_new) -> "MultiOutputExactGP":
        """Refit on the concatenated data (MultiOutputSparseGP.update semantics,
        sparse_gp.py:486-504), incrementally on the device (gpmpc_gp_append)
        when every output shares the factor; otherwise a full refit."""
        h = self.device_handle
        g0 = self.gps[0]
        if h is None or g0.X_train is None:
            return self.fit(X_new, Y_new)
        X_new = np.atleast_2d(X_new)
        Y_new = np.atleast_2d(Y_new)
        if Y_new.shape[1] != self.output_dim and Y_new.shape[0] == self.output_dim:
            Y_new = Y_new.T
        X = np.vstack([g0.X_train, X_new])
        Y_old = np.stack([g.y_train * g._y_std + g._y_mean for g in self.gps], axis=1)
        Y = np.vstack([Y_old, Y_new])
        if h.append(X_new, Y):
            shared = self.gps[0]._dev
            shared._cache_key = None
            for i, g in enumerate(self.gps):
                g._attach(X, Y[:, i], shared, i)
            return self
        return self.fit(X, Y)

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
    def log_marginal_likelihood(self) -> float:
        return sum(gp.log_marginal_likelihood for gp in self.gps)

    @property
    def device_handle(self):
        """The shared device GP (or None when outputs were fitted separately)."""
        d = self.gps[0]._dev
        return d.h if d is not None and all(g._dev is d for g in self.gps) else None

    def __repr__(self) -> str:
        return f"MultiOutputExactGP(input_dim={self.input_dim}, output_dim={self.output_dim})"
