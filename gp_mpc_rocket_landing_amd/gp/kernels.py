"""Kernel surfaces of reference src/gp/kernels.py; Gram matrices on the GPU.

Every Gram matrix of SE-ARD / isotropic SE / Matern-3/2 / Matern-5/2 runs
through gpmpc_gram (csrc/gram.hip: expansion-form scaled distance, clamped at
0, kernels.py:205-236).  Hyperparameters are exposed in log space exactly as
get_params/set_params/n_params/param_names define them (kernels.py:320-371).
Sum/product kernels combine device Grams elementwise; WhiteNoise is diagonal.
Every kernel also describes itself as a device program (``device_program``:
the postfix form csrc/gram.hip evaluates), so a GP fitted with a composite
kernel forms its Grams on the device too (gpmpc_gp_fit_exact_prog,
gpmpc_sparse_fit_prog).
``gradients`` (kernels.py:279-318 and the per-kernel variants) returns the
same dictionaries as the reference: SE-ARD / isotropic SE gradient matrices
come from the device (gpmpc_gram_grad), the Matern kernels give only the
log-signal-variance gradient K, as the reference's do.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import List, Optional

import numpy as np

from .. import _lib


def _ctx():
    return _lib.default_context()


class Kernel(ABC):
    """kernels.py:33-127."""

    @abstractmethod
    def __call__(self, X1, X2=None) -> np.ndarray: ...

    @abstractmethod
    def diagonal(self, X) -> np.ndarray: ...

    @property
    @abstractmethod
    def n_params(self) -> int: ...

    @property
    @abstractmethod
    def param_names(self) -> List[str]: ...

    @abstractmethod
    def get_params(self) -> np.ndarray: ...

    @abstractmethod
    def set_params(self, params) -> None: ...

    # device-gram description: (kind, lengthscales, sigma2) or None
    def _device_spec(self):
        return None

    # the kernel as postfix program pairs (code, parameter offset) appended to ops / par
    def _device_prog(self, ops: list, par: list) -> None:
        raise NotImplementedError(f"{type(self).__name__} has no device program")

    def device_program(self) -> "_lib.KernelProgram":
        """This kernel as the device's postfix Gram program (gpmpc.h GPMPC_KP_*)."""
        ops, par = [], []
        self._device_prog(ops, par)
        return _lib.KernelProgram(ops, par)

    def __add__(self, other):
        return SumKernel(self, other)

    def __mul__(self, other):
        return ProductKernel(self, other)


class _StationaryARD(Kernel):
    KIND = _lib.SE_ARD

    def __init__(self, input_dim: int, signal_variance: float = 1.0,
                 lengthscales: Optional[np.ndarray] = None,
                 learn_signal_variance: bool = True, learn_lengthscales: bool = True):
        self.input_dim = int(input_dim)
        self._signal_variance = float(signal_variance)
        if lengthscales is None:
            self._lengthscales = np.ones(self.input_dim)
        else:
            self._lengthscales = np.asarray(lengthscales, float).flatten()
            assert len(self._lengthscales) == self.input_dim
        self.learn_signal_variance = learn_signal_variance
        self.learn_lengthscales = learn_lengthscales

    @property
    def signal_variance(self) -> float:
        return self._signal_variance

    @signal_variance.setter
    def signal_variance(self, value: float) -> None:
        assert value > 0, "Signal variance must be positive"
        self._signal_variance = float(value)

    @property
    def lengthscales(self) -> np.ndarray:
        return self._lengthscales

    @lengthscales.setter
    def lengthscales(self, value) -> None:
        value = np.asarray(value, float).flatten()
        assert len(value) == self.input_dim
        assert np.all(value > 0), "Lengthscales must be positive"
        self._lengthscales = value

    def _device_spec(self):
        return self.KIND, self._lengthscales, self._signal_variance

    def _device_prog(self, ops, par):
        ops.append((self.KIND, len(par)))
        par.extend([self._signal_variance, *self._lengthscales])

    def __call__(self, X1, X2=None) -> np.ndarray:
        return _lib.gram(_ctx(), self.KIND, X1, X2, self._lengthscales, self._signal_variance)

    def diagonal(self, X) -> np.ndarray:
        return np.full(np.atleast_2d(X).shape[0], self._signal_variance)

    def gradients(self, X1, X2=None) -> dict:
        """Matern32/52.gradients (kernels.py:551-558, 644-650): the reference
        returns only d K / d log(sigma2) = K for these kernels."""
        return {"log_signal_variance": self(X1, X2)}

    @property
    def n_params(self) -> int:
        return int(self.learn_signal_variance) + (self.input_dim if self.learn_lengthscales else 0)

    @property
    def param_names(self) -> List[str]:
        names = ["log_signal_variance"] if self.learn_signal_variance else []
        if self.learn_lengthscales:
            names += [f"log_lengthscale_{i}" for i in range(self.input_dim)]
        return names

    def get_params(self) -> np.ndarray:
        p = [np.log(self._signal_variance)] if self.learn_signal_variance else []
        if self.learn_lengthscales:
            p.extend(np.log(self._lengthscales))
        return np.array(p)

    def set_params(self, params) -> None:
        params = np.asarray(params, float).flatten()
        i = 0
        if self.learn_signal_variance:
            self._signal_variance = float(np.exp(params[i])); i += 1
        if self.learn_lengthscales:
            self._lengthscales = np.exp(params[i:i + self.input_dim])

    def __repr__(self) -> str:
        return f"{type(self).__name__}(input_dim={self.input_dim}, σ²={self._signal_variance:.4g})"


class SquaredExponentialARD(_StationaryARD):
    """kernels.py:130-384: sigma2 exp(-r^2/2), r^2 = |x/l - x'/l|^2."""
    KIND = _lib.SE_ARD

    def gradients(self, X1, X2=None) -> dict:
        """kernels.py:279-318: d K / d log(sigma2) = K and, per input dimension,
        d K / d log(l_i) = K (x1_i - x2_i)^2 / l_i^2 (device)."""
        K, G = _lib.gram_grad(_ctx(), _lib.SE_ARD, X1, X2, self._lengthscales, self._signal_variance)
        grads = {}
        if self.learn_signal_variance:
            grads["log_signal_variance"] = K.copy()
        if self.learn_lengthscales:
            for i in range(self.input_dim):
                grads[f"log_lengthscale_{i}"] = G[i]
        return grads


class Matern32(_StationaryARD):
    """kernels.py:482-576: sigma2 (1 + sqrt3 r) exp(-sqrt3 r)."""
    KIND = _lib.MATERN32

    def __init__(self, input_dim: int, signal_variance: float = 1.0, lengthscales=None):
        super().__init__(input_dim, signal_variance, lengthscales)


class Matern52(_StationaryARD):
    """kernels.py:579-673: sigma2 (1 + sqrt5 r + 5 r^2/3) exp(-sqrt5 r)."""
    KIND = _lib.MATERN52

    def __init__(self, input_dim: int, signal_variance: float = 1.0, lengthscales=None):
        super().__init__(input_dim, signal_variance, lengthscales)


class SquaredExponential(Kernel):
    """kernels.py:392-479: isotropic SE (one lengthscale)."""

    def __init__(self, signal_variance: float = 1.0, lengthscale: float = 1.0):
        self._signal_variance = float(signal_variance)
        self._lengthscale = float(lengthscale)

    @property
    def signal_variance(self) -> float:
        return self._signal_variance

    @property
    def lengthscale(self) -> float:
        return self._lengthscale

    def _device_spec(self):
        return _lib.SE_ISO, np.array([self._lengthscale]), self._signal_variance

    def _device_prog(self, ops, par):
        ops.append((_lib.SE_ISO, len(par)))
        par.extend([self._signal_variance, self._lengthscale])

    def __call__(self, X1, X2=None) -> np.ndarray:
        return _lib.gram(_ctx(), _lib.SE_ISO, X1, X2, np.array([self._lengthscale]), self._signal_variance)

    def diagonal(self, X) -> np.ndarray:
        return np.full(np.atleast_2d(X).shape[0], self._signal_variance)

    def gradients(self, X1, X2=None) -> dict:
        """kernels.py:438-456: K and K r^2 / l^2 (device)."""
        K, G = _lib.gram_grad(_ctx(), _lib.SE_ISO, X1, X2, np.array([self._lengthscale]),
                              self._signal_variance)
        return {"log_signal_variance": K, "log_lengthscale": G[0]}

    @property
    def n_params(self) -> int:
        return 2

    @property
    def param_names(self) -> List[str]:
        return ["log_signal_variance", "log_lengthscale"]

    def get_params(self) -> np.ndarray:
        return np.log([self._signal_variance, self._lengthscale])

    def set_params(self, params) -> None:
        self._signal_variance, self._lengthscale = (float(v) for v in np.exp(np.asarray(params)[:2]))


class SumKernel(Kernel):
    """kernels.py:676-726."""

    OP = _lib.KP_SUM

    def __init__(self, k1: Kernel, k2: Kernel):
        self.k1, self.k2 = k1, k2

    def _device_prog(self, ops, par):
        self.k1._device_prog(ops, par)
        self.k2._device_prog(ops, par)
        ops.append((self.OP, 0))

    def __call__(self, X1, X2=None):
        return self.k1(X1, X2) + self.k2(X1, X2)

    def diagonal(self, X):
        return self.k1.diagonal(X) + self.k2.diagonal(X)

    @property
    def n_params(self):
        return self.k1.n_params + self.k2.n_params

    @property
    def param_names(self):
        return [f"k1_{n}" for n in self.k1.param_names] + [f"k2_{n}" for n in self.k2.param_names]

    def get_params(self):
        return np.concatenate([self.k1.get_params(), self.k2.get_params()])

    def set_params(self, params):
        params = np.asarray(params)
        self.k1.set_params(params[:self.k1.n_params])
        self.k2.set_params(params[self.k1.n_params:])

    def gradients(self, X1, X2=None) -> dict:
        """kernels.py:697-707."""
        grads = {f"k1_{n}": g for n, g in self.k1.gradients(X1, X2).items()}
        grads.update({f"k2_{n}": g for n, g in self.k2.gradients(X1, X2).items()})
        return grads


class ProductKernel(SumKernel):
    """kernels.py:729-782."""
    OP = _lib.KP_PROD

    def __call__(self, X1, X2=None):
        return self.k1(X1, X2) * self.k2(X1, X2)

    def gradients(self, X1, X2=None) -> dict:
        """kernels.py:750-763: product rule."""
        K1, K2 = self.k1(X1, X2), self.k2(X1, X2)
        grads = {f"k1_{n}": g * K2 for n, g in self.k1.gradients(X1, X2).items()}
        grads.update({f"k2_{n}": K1 * g for n, g in self.k2.gradients(X1, X2).items()})
        return grads

    def diagonal(self, X):
        return self.k1.diagonal(X) * self.k2.diagonal(X)


class WhiteNoise(Kernel):
    """kernels.py:790-844: sigma2 I on the training set, zero cross-covariance."""

    def __init__(self, noise_variance: float = 1e-6):
        self._noise_variance = float(noise_variance)

    def _device_prog(self, ops, par):
        ops.append((_lib.KP_WHITE, len(par)))
        par.append(self._noise_variance)

    @property
    def noise_variance(self) -> float:
        return self._noise_variance

    def __call__(self, X1, X2=None):
        X1 = np.atleast_2d(X1)
        if X2 is None:
            return self._noise_variance * np.eye(X1.shape[0])
        return np.zeros((X1.shape[0], np.atleast_2d(X2).shape[0]))

    def diagonal(self, X):
        return np.full(np.atleast_2d(X).shape[0], self._noise_variance)

    @property
    def n_params(self):
        return 1

    @property
    def param_names(self):
        return ["log_noise_variance"]

    def get_params(self):
        return np.array([np.log(self._noise_variance)])

    def set_params(self, params):
        self._noise_variance = float(np.exp(np.asarray(params)[0]))

    def gradients(self, X1, X2=None) -> dict:
        """kernels.py:822-827."""
        return {"log_noise_variance": self(X1, X2)}


# aliases (kernels.py:383-384)
RBF = SquaredExponentialARD
SE_ARD = SquaredExponentialARD


def create_matern_kernel(input_dim: int, nu: float = 2.5, **kw) -> Kernel:
    """kernels.py:875-898."""
    if nu == 1.5:
        return Matern32(input_dim, **kw)
    if nu == 2.5:
        return Matern52(input_dim, **kw)
    raise ValueError(f"Unsupported nu={nu}. Use 1.5 or 2.5")
