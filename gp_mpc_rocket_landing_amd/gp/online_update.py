"""Online GP updates (reference src/gp/online_update.py) over the device GPs.

The reference refits its GP from scratch at every update (online_update.py:
361-408).  Here the refit runs on the device, and when the GP is exact and the
buffer only grew since the last fit (no eviction by the ring buffer), the
update appends the new rows to the device factor in O(n^2 k)
(``ExactGP.update`` -> gpmpc_gp_append) -- the same GP as the
refit.  Everything else (buffering, novelty filter, cadence, statistics) is
host plumbing with the reference's names and defaults.
"""
from __future__ import annotations

import time
from collections import deque
from dataclasses import dataclass
from typing import Callable, Deque, List, Optional, Tuple

import numpy as np


@dataclass
class OnlineUpdateConfig:
    """online_update.py:37-62."""
    buffer_size: int = 1000
    min_data_for_fit: int = 20
    use_novelty_filter: bool = True
    novelty_threshold: float = 0.3
    min_distance: float = 0.01
    update_interval: int = 10
    refit_interval: int = 100
    max_update_time_ms: float = 5.0
    add_inducing_on_novel: bool = True
    max_inducing_points: int = 100
    inducing_update_threshold: float = 0.5


@dataclass
class DataPoint:
    """online_update.py:65-73."""
    x: np.ndarray
    u: np.ndarray
    d: np.ndarray
    timestamp: float
    novelty: float = 0.0


class DataBuffer:
    """online_update.py:76-229: ring buffer of (features, targets) with a
    novelty filter.  ``total_added`` counts every accepted point, so
    ``total_added == size`` means nothing was ever evicted."""

    def __init__(self, max_size: int = 1000, feature_dim: int = 10, target_dim: int = 3):
        self.max_size = max_size
        self.feature_dim = feature_dim
        self.target_dim = target_dim
        self._features: Deque[np.ndarray] = deque(maxlen=max_size)
        self._targets: Deque[np.ndarray] = deque(maxlen=max_size)
        self._novelties: Deque[float] = deque(maxlen=max_size)
        self._timestamps: Deque[float] = deque(maxlen=max_size)
        self._total_added = 0
        self._total_rejected = 0

    @property
    def size(self) -> int:
        return len(self._features)

    @property
    def is_empty(self) -> bool:
        return self.size == 0

    @property
    def is_full(self) -> bool:
        return self.size >= self.max_size

    @property
    def total_added(self) -> int:
        return self._total_added

    def add(self, features, targets, novelty: float = 0.0, timestamp: Optional[float] = None) -> bool:
        if timestamp is None:
            timestamp = time.time()
        self._features.append(np.array(features, dtype=float, copy=True))
        self._targets.append(np.array(targets, dtype=float, copy=True))
        self._novelties.append(novelty)
        self._timestamps.append(timestamp)
        self._total_added += 1
        return True

    def add_if_novel(self, features, targets, novelty: float, threshold: float = 0.3,
                     min_distance: Optional[float] = None) -> bool:
        """online_update.py:151-185: reject below the novelty threshold or
        closer than min_distance to a stored point."""
        if novelty < threshold:
            self._total_rejected += 1
            return False
        if min_distance is not None and self.size > 0:
            distances = np.linalg.norm(self.get_features() - features, axis=1)
            if np.min(distances) < min_distance:
                self._total_rejected += 1
                return False
        return self.add(features, targets, novelty)

    def get_features(self) -> np.ndarray:
        if self.is_empty:
            return np.empty((0, self.feature_dim))
        return np.array(list(self._features))

    def get_targets(self) -> np.ndarray:
        if self.is_empty:
            return np.empty((0, self.target_dim))
        return np.array(list(self._targets))

    def get_data(self) -> Tuple[np.ndarray, np.ndarray]:
        return self.get_features(), self.get_targets()

    def get_recent(self, n: int) -> Tuple[np.ndarray, np.ndarray]:
        n = min(n, self.size)
        return np.array(list(self._features)[-n:]), np.array(list(self._targets)[-n:])

    def clear(self) -> None:
        self._features.clear()
        self._targets.clear()
        self._novelties.clear()
        self._timestamps.clear()

    def get_statistics(self) -> dict:
        return {
            "size": self.size,
            "max_size": self.max_size,
            "total_added": self._total_added,
            "total_rejected": self._total_rejected,
            "acceptance_rate": self._total_added / max(1, self._total_added + self._total_rejected),
            "mean_novelty": np.mean(list(self._novelties)) if self.size > 0 else 0.0,
        }


def _targets_for_fit(D: np.ndarray) -> np.ndarray:
    """online_update.py:384-388: one target column (the first, or the mean of several)."""
    if D.ndim == 1:
        return D
    return D[:, 0] if D.shape[1] == 1 else D.mean(axis=1)


def _is_fitted(gp) -> bool:
    return getattr(gp, "_dev", None) is not None or getattr(gp, "_L_B", None) is not None


class OnlineGPUpdater:
    """online_update.py:232-425 for a device GP (SparseGP or ExactGP)."""

    def __init__(self, gp, config: Optional[OnlineUpdateConfig] = None,
                 feature_extractor: Optional[Callable[[np.ndarray, np.ndarray], np.ndarray]] = None):
        self.gp = gp
        self.config = config or OnlineUpdateConfig()
        self.feature_extractor = feature_extractor or (lambda x, u: np.concatenate([x, u]))
        self._feature_dim: Optional[int] = None
        self._target_dim: int = 1
        self._buffer: Optional[DataBuffer] = None
        self._points_since_update = 0
        self._points_since_refit = 0
        self._total_updates = 0
        self._last_update_time = 0.0
        self._update_times: List[float] = []
        self._fitted_rows = 0      # buffer rows the GP was last fitted on (no eviction since)
        self.incremental_updates = 0

    def _ensure_buffer(self, feature_dim: int, target_dim: int = 1) -> None:
        if self._buffer is None:
            self._feature_dim, self._target_dim = feature_dim, target_dim
            self._buffer = DataBuffer(self.config.buffer_size, feature_dim, target_dim)

    def add_observation(self, x, u, d) -> bool:
        """online_update.py:293-345 (novelty = predicted variance / prior variance)."""
        z = self.feature_extractor(x, u)
        d = np.atleast_1d(d)
        self._ensure_buffer(len(z), len(d))
        if self.config.use_novelty_filter and _is_fitted(self.gp):
            try:
                pred = self.gp.predict(z.reshape(1, -1))
                novelty = float(np.mean(pred.variance) / self.gp.kernel.signal_variance)
            except Exception:  # noqa: BLE001  (online_update.py:324-325)
                novelty = 1.0
        else:
            novelty = 1.0
        if self.config.use_novelty_filter:
            added = self._buffer.add_if_novel(z, d, novelty, threshold=self.config.novelty_threshold,
                                              min_distance=self.config.min_distance)
        else:
            added = self._buffer.add(z, d, novelty)
        if added:
            self._points_since_update += 1
            self._points_since_refit += 1
        return added

    def should_update(self) -> bool:
        if self._buffer is None or self._buffer.size < self.config.min_data_for_fit:
            return False
        return self._points_since_update >= self.config.update_interval

    def should_refit(self) -> bool:
        if self._buffer is None:
            return False
        return self._points_since_refit >= self.config.refit_interval

    def update(self, force: bool = False) -> dict:
        """online_update.py:361-408.  Incremental when the GP is exact, was fitted
        on a prefix of the buffer and nothing was evicted since."""
        if self._buffer is None or self._buffer.is_empty:
            return {"status": "no_data"}
        if not force and not self.should_update():
            return {"status": "skipped"}
        start = time.perf_counter()
        Z, D = self._buffer.get_data()
        t = _targets_for_fit(D)
        n_old = self._fitted_rows
        grew_only = (0 < n_old < self._buffer.size and self._buffer.total_added == self._buffer.size)
        try:
            if grew_only and hasattr(self.gp, "update") and getattr(self.gp, "_dev", None) is not None \
                    and type(self.gp).__name__ == "ExactGP":
                self.gp.update(Z[n_old:], t[n_old:])
                self.incremental_updates += 1
            else:
                self.gp.fit(Z, t)
            self._fitted_rows = self._buffer.size
            status = "success"
        except Exception as e:  # noqa: BLE001  (online_update.py:391-392)
            status = f"error: {e}"
        elapsed = (time.perf_counter() - start) * 1000
        self._update_times.append(elapsed)
        self._last_update_time = elapsed
        self._total_updates += 1
        self._points_since_update = 0
        if self.should_refit():
            self._points_since_refit = 0
        return {"status": status, "time_ms": elapsed, "n_data": self._buffer.size,
                "total_updates": self._total_updates}

    def get_statistics(self) -> dict:
        stats = {"total_updates": self._total_updates,
                 "points_since_update": self._points_since_update,
                 "last_update_time_ms": self._last_update_time}
        if self._buffer is not None:
            stats.update(self._buffer.get_statistics())
        if self._update_times:
            stats["mean_update_time_ms"] = np.mean(self._update_times)
            stats["max_update_time_ms"] = np.max(self._update_times)
        return stats


class OnlineStructuredGPUpdater:
    """online_update.py:428-537 for the device StructuredRocketGP."""

    def __init__(self, gp, config: Optional[OnlineUpdateConfig] = None):
        self.gp = gp
        self.config = config or OnlineUpdateConfig()
        self._points_since_update = 0
        self._total_observations = 0
        self._total_updates = 0
        self._update_times: List[float] = []

    def add_observation(self, x, u, d_v, d_omega) -> bool:
        if self.config.use_novelty_filter and self.gp._is_fitted:
            if not self.gp.is_novel(x, u):
                return False
        self.gp.add_data(np.reshape(x, (1, -1)), np.reshape(u, (1, -1)),
                         np.reshape(d_v, (1, -1)), np.reshape(d_omega, (1, -1)))
        self._points_since_update += 1
        self._total_observations += 1
        return True

    def should_update(self) -> bool:
        if self.gp.n_data < self.config.min_data_for_fit:
            return False
        return self._points_since_update >= self.config.update_interval

    def update(self, force: bool = False) -> dict:
        if not force and not self.should_update():
            return {"status": "skipped"}
        start = time.perf_counter()
        try:
            self.gp.fit()
            status = "success"
        except Exception as e:  # noqa: BLE001
            status = f"error: {e}"
        elapsed = (time.perf_counter() - start) * 1000
        self._update_times.append(elapsed)
        self._total_updates += 1
        self._points_since_update = 0
        return {"status": status, "time_ms": elapsed, "n_data": self.gp.n_data,
                "total_updates": self._total_updates}

    def get_statistics(self) -> dict:
        stats = {"total_observations": self._total_observations,
                 "total_updates": self._total_updates,
                 "points_since_update": self._points_since_update,
                 "n_data": self.gp.n_data, "gp_fitted": self.gp._is_fitted}
        if self._update_times:
            stats["mean_update_time_ms"] = np.mean(self._update_times)
            stats["max_update_time_ms"] = np.max(self._update_times)
        return stats


class ResidualCollector:
    """online_update.py:540-677: d = (x_actual - f_nominal(x, u)) / dt on the
    velocity (4:7) and angular-velocity (11:14) blocks of the 14-state."""

    def __init__(self, nominal_dynamics: Callable[[np.ndarray, np.ndarray, float], np.ndarray],
                 max_samples: int = 10000):
        self.nominal_dynamics = nominal_dynamics
        self.max_samples = max_samples
        self.states: List[np.ndarray] = []
        self.controls: List[np.ndarray] = []
        self.residuals_v: List[np.ndarray] = []
        self.residuals_omega: List[np.ndarray] = []

    def record(self, x, u, x_next_actual, dt: float) -> None:
        if len(self.states) >= self.max_samples:
            self.states.pop(0); self.controls.pop(0)
            self.residuals_v.pop(0); self.residuals_omega.pop(0)
        residual = np.asarray(x_next_actual) - self.nominal_dynamics(x, u, dt)
        self.states.append(np.array(x, dtype=float, copy=True))
        self.controls.append(np.array(u, dtype=float, copy=True))
        self.residuals_v.append(residual[4:7] / dt)
        self.residuals_omega.append(residual[11:14] / dt)

    def get_training_data(self):
        if not self.states:
            return np.empty((0, 14)), np.empty((0, 3)), np.empty((0, 3)), np.empty((0, 3))
        return (np.array(self.states), np.array(self.controls), np.array(self.residuals_v),
                np.array(self.residuals_omega))

    @property
    def n_samples(self) -> int:
        return len(self.states)

    def clear(self) -> None:
        self.states.clear(); self.controls.clear()
        self.residuals_v.clear(); self.residuals_omega.clear()

    def get_statistics(self) -> dict:
        if not self.states:
            return {"n_samples": 0}
        D_v = np.array(self.residuals_v); D_w = np.array(self.residuals_omega)
        return {"n_samples": self.n_samples,
                "d_v_mean": np.mean(D_v, axis=0).tolist(), "d_v_std": np.std(D_v, axis=0).tolist(),
                "d_omega_mean": np.mean(D_w, axis=0).tolist(),
                "d_omega_std": np.std(D_w, axis=0).tolist()}
