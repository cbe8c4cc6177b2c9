"""SURVEY 8f-4 -- incremental exact GP on the device (gpmpc_gp_append): k rows
appended to a fitted GP in O(n^2 k) must give the GP a full refit of the
concatenated data gives (the SparseGP.update / online refit semantics,
sparse_gp.py:328-353, online_update.py:361-408), checked against the numpy
oracle's ExactGP.fit on the concatenated set.  Tolerance: SURVEY 8c, 1e-6 of
max(|ref|, y_std) for means and of max(|ref|, sigma2 y_std^2) for variances;
L and the LML to 1e-9 relative."""
import numpy as np
import pytest

from conftest import close

pytestmark = pytest.mark.gpu


def _data(n, seed=0):
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data, query_points
    from oracle import gp_oracle
    X, U, D = synthetic_training_data(n, seed=seed)
    Xq, Uq = query_points(X, U, 25, seed=7)
    return gp_oracle.features_3dof(X, U), D, gp_oracle.features_3dof(Xq, Uq)


def _check(h, Z, D, Zq, gp_oracle):
    st = gp_oracle.exact_fit(Z, D)
    mo, vo = gp_oracle.exact_predict(st, Zq)
    m, v = h.predict(Zq)
    ok_m, em = close(m, mo, st["y_std"][None, :])
    ok_v, ev = close(v, vo, st["y_std"][None, :] ** 2)
    assert ok_m and ok_v, (em, ev)
    np.testing.assert_allclose(h.lml, st["lml"], rtol=1e-9)
    np.testing.assert_allclose(h.y_mean, st["y_mean"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(h.y_std, st["y_std"], rtol=1e-12)
    L, a = h.state()
    np.testing.assert_allclose(np.tril(L), st["L"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(a, st["alpha"], rtol=1e-7, atol=1e-9 * np.abs(st["alpha"]).max())


@pytest.mark.parametrize("k", [1, 7, 64, 300])
def test_append_equals_refit(gpu_ctx, k):
    from gp_mpc_rocket_landing_amd import _lib
    from oracle import gp_oracle
    Z, D, Zq = _data(300 + k)
    h = _lib.ExactGPHandle(gpu_ctx, _lib.SE_ARD, Z[:300], D[:300], np.ones(11), 1.0, 1e-4)
    assert h.append(Z[300:], D)
    assert h.n == 300 + k
    _check(h, Z, D, Zq, gp_oracle)


def test_streaming_appends(gpu_ctx):
    """Five appends of 20 rows after a 200-row fit = one fit on 300 rows."""
    from gp_mpc_rocket_landing_amd import _lib
    from oracle import gp_oracle
    Z, D, Zq = _data(300, seed=4)
    h = _lib.ExactGPHandle(gpu_ctx, _lib.SE_ARD, Z[:200], D[:200], np.ones(11), 1.0, 1e-4)
    for r in range(200, 300, 20):
        assert h.append(Z[r:r + 20], D[:r + 20])
    _check(h, Z, D, Zq, gp_oracle)


def test_append_refused_after_jitter_and_update_falls_back(gpu_ctx):
    """A GP fitted with jitter cannot grow incrementally (the refit reruns the
    ladder on the whole matrix): append returns False, the handle is unchanged,
    and MultiOutputExactGP.update refits."""
    from gp_mpc_rocket_landing_amd import _lib
    from gp_mpc_rocket_landing_amd.gp.exact_gp import MultiOutputExactGP
    from oracle import gp_oracle
    Z, D, Zq = _data(120, seed=5)
    Zd = np.vstack([Z[:40], Z[:40]]); Dd = np.vstack([D[:40], D[:40] + 1e-3])
    h = _lib.ExactGPHandle(gpu_ctx, _lib.SE_ARD, Zd, Dd, np.ones(11), 1.0, -2e-3)
    assert h.jitter_steps == 5
    m0, v0 = h.predict(Zq)
    assert not h.append(Z[40:60], np.vstack([Dd, D[40:60]]))
    assert h.n == 80
    m1, v1 = h.predict(Zq)
    assert np.array_equal(m0, m1) and np.array_equal(v0, v1)
    gp = MultiOutputExactGP(11, 3, noise_variance=-2e-3)
    gp.fit(Zd, Dd)
    h1 = gp.device_handle
    gp.update(Z[40:60], D[40:60])
    assert gp.device_handle is not h1 and gp.device_handle.n == 100   # refitted
    assert gp.device_handle.jitter_steps == 5
    st = gp_oracle.exact_fit(np.vstack([Zd, Z[40:60]]), np.vstack([Dd, D[40:60]]), noise=-2e-3)
    assert st["jitter_steps"] == 5
    mo, vo = gp_oracle.exact_predict(st, Zq)
    m, v = gp.predict(Zq)
    assert close(m, mo, st["y_std"][None, :])[0] and close(v, vo, st["y_std"][None, :] ** 2)[0]


def test_simple3dof_incremental_fit(gpu_ctx):
    """Simple3DoFGP(use_sparse=False): add_data + fit after more data arrived grows
    the device factor in place; predictions equal the oracle's fit on all rows."""
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data, query_points
    from gp_mpc_rocket_landing_amd.gp.structured_gp import Simple3DoFGP
    from oracle import gp_oracle
    X, U, D = synthetic_training_data(340, seed=9)
    Xq, Uq = query_points(X, U, 20, seed=7)
    g = Simple3DoFGP(use_sparse=False)
    g.add_data(X[:300], U[:300], D[:300])
    g.fit()
    h0 = g.gp.device_handle
    g.add_data(X[300:], U[300:], D[300:])
    g.fit()
    assert g.gp.device_handle is h0 and h0.n == 340   # grown, not rebuilt
    st, (mo, vo) = gp_oracle.simple3dof_fit_predict_exact(X, U, D, Xq, Uq)
    m, v = g.predict_batch(Xq, Uq)
    assert close(m, mo, st["y_std"][None, :])[0] and close(v, vo, st["y_std"][None, :] ** 2)[0]


def test_fleet_refuses_grown_gp(gpu_ctx):
    from gp_mpc_rocket_landing_amd import _lib, fleet
    Z, D, _ = _data(260, seed=2)
    h = _lib.ExactGPHandle(gpu_ctx, _lib.SE_ARD, Z[:200], D[:200], np.ones(11), 1.0, 1e-4)
    fl = fleet.Fleet(gpu_ctx, h, 4, horizon=20)
    fl.reset(fleet.initial_conditions(4, seed0=42))
    fl.step(1)
    assert h.append(Z[200:], D)
    with pytest.raises(_lib.HIPError):
        fl.step(1)
    fl.close()


@pytest.mark.parametrize("buffer_size", [1000, 100])
def test_online_updater_exact_gp(gpu_ctx, buffer_size):
    """OnlineGPUpdater (online_update.py:232-425) on the device ExactGP: 150
    streamed observations, an update every 10; with room in the buffer every
    update after the first is an O(n^2 k) append, after evictions (buffer 100)
    a refit; either way the GP equals the oracle's fit on the buffer."""
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.gp.exact_gp import ExactGP
    from gp_mpc_rocket_landing_amd.gp.features import Simple3DoFFeatureExtractor
    from gp_mpc_rocket_landing_amd.gp.kernels import SquaredExponentialARD
    from gp_mpc_rocket_landing_amd.gp.online_update import OnlineGPUpdater, OnlineUpdateConfig
    from oracle import gp_oracle
    X, U, D = synthetic_training_data(150, seed=6)
    fe = Simple3DoFFeatureExtractor()
    gp = ExactGP(SquaredExponentialARD(11), noise_variance=1e-4)
    up = OnlineGPUpdater(gp, OnlineUpdateConfig(buffer_size=buffer_size, use_novelty_filter=False,
                                                update_interval=10), feature_extractor=fe.extract)
    for i in range(150):
        up.add_observation(X[i], U[i], D[i])
        if up.should_update():
            assert up.update()["status"] == "success"
    Z, T = up._buffer.get_data()
    assert Z.shape[0] == min(150, buffer_size) and gp.n_train == Z.shape[0]
    if buffer_size == 1000:
        assert up.incremental_updates == 13   # fits at 20, then appends at 30 .. 150
    else:
        assert up.incremental_updates == 8    # appends 30 .. 100, refits once the ring evicts
    st = gp_oracle.exact_fit(Z, T.mean(axis=1))
    Zq = Z[::7] + 0.01
    mo, vo = gp_oracle.exact_predict(st, Zq)
    p = gp.predict(Zq)
    assert close(p.mean, mo[:, 0], st["y_std"][0])[0]
    assert close(p.variance, vo[:, 0], st["y_std"][0] ** 2)[0]
