"""Host side of the 14-state path (no GPU): the Rocket6DoFDynamics mirror
against the oracle restatement, the GPMPC dispatch and its refusals, and the
C-ABI's 6-DoF default config (read back through ctypes: checks the struct
layout too)."""
import numpy as np
import pytest


def _states(n=6, seed=0):
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFDynamics
    d = Rocket6DoFDynamics()
    rs = np.random.RandomState(seed)
    out = []
    for _ in range(n):
        ax = rs.randn(3)
        x = d.create_initial_state(altitude=10 + 30 * rs.rand(), downrange=rs.randn(), crossrange=rs.randn(),
                                   velocity=rs.randn(3), tilt_angle=0.2 * rs.randn(), tilt_axis=ax,
                                   omega=0.2 * rs.randn(3), mass=1.5 + rs.rand())
        u = rs.randn(3) + np.array([2.0, 0.0, 0.0])
        out.append((x, u))
    return d, out


J_FULL = np.array([[0.02, 0.004, -0.002], [0.004, 1.0, 0.03], [-0.002, 0.03, 0.95]]) * 0.168


def test_rocket6dof_mirror_matches_oracle_bitwise():
    """step (RK4 + normalisation) and linearize(dt) are the oracle's formulas
    (nominal_mpc.py:163-203, rocket_6dof.py:427-459) bit for bit -- for the default
    diagonal J_B and for a full (non-diagonal) tensor (VERDICT r5 missing #1)."""
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFConfig, Rocket6DoFDynamics
    from oracle import sixdof_oracle as so
    _, cases = _states()
    for d, rk in ((Rocket6DoFDynamics(), None),
                  (Rocket6DoFDynamics(Rocket6DoFConfig(J_B=J_FULL)), so.rocket_params(J_FULL))):
        if rk is not None:
            assert "Jf" in rk
        for x, u in cases:
            np.testing.assert_array_equal(d.step(x, u, 0.1), so.step(x, u, 0.1, rk))
            A, B = d.linearize(x, u, 0.1)
            Ao, Bo = so.linearize(x, u, 0.1, rk)
            np.testing.assert_allclose(A, Ao, rtol=0, atol=1e-17)
            np.testing.assert_array_equal(B, Bo)
    # a diagonal tensor given in full is the diagonal model
    assert "Jf" not in so.rocket_params(np.diag([0.1, 0.2, 0.3]))


def test_rocket6dof_jacobians_match_finite_differences():
    """Analytic A_c, B_c against central differences of f, also for a full
    (non-diagonal) inertia tensor (the J^-1([J w]x - [w]x J) form)."""
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFConfig, Rocket6DoFDynamics
    J = np.array([[0.01, 0.001, 0.0], [0.001, 0.2, 0.002], [0.0, 0.002, 0.18]])
    for dyn in (Rocket6DoFDynamics(), Rocket6DoFDynamics(Rocket6DoFConfig(J_B=J))):
        _, cases = _states(3, seed=1)
        for x, u in cases:
            A, B = dyn.jacobian_x(x, u), dyn.jacobian_u(x, u)
            h = 1e-6
            for j in range(14):
                e = np.zeros(14); e[j] = h
                fd = (dyn.dynamics(x + e, u) - dyn.dynamics(x - e, u)) / (2 * h)
                np.testing.assert_allclose(A[:, j], fd, atol=2e-7)
            for j in range(3):
                e = np.zeros(3); e[j] = h
                fd = (dyn.dynamics(x, u + e) - dyn.dynamics(x, u - e)) / (2 * h)
                np.testing.assert_allclose(B[:, j], fd, atol=2e-7)


def test_rocket6dof_api():
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFDynamics, create_rocket_6dof
    d = Rocket6DoFDynamics()
    x = d.create_initial_state(altitude=12.0, mass=1.8)
    assert d.n_state == 14 and d.n_control == 3 and d.params.g0 == 1.0
    assert d.params.alpha == 1.0 / 30.0 and d.matches_device_model()
    np.testing.assert_allclose(d.hover_thrust(x), [1.8, 0, 0])
    assert d.get_altitude(x) == 12.0 and d.get_tilt_angle(x) == 0.0
    assert d.thrust_constraint(np.array([1.0, 0, 0]))[0] == pytest.approx(0.5)
    A_d, B_d, c = d.linearize_discrete(x, np.array([2.0, 0.1, 0.0]), 0.1)
    np.testing.assert_allclose(A_d @ x + B_d @ np.array([2.0, 0.1, 0.0]) + c,
                               d.step(x, np.array([2.0, 0.1, 0.0]), 0.1), atol=1e-14)
    # the device model's rocket parameters are runtime values, the inertia tensor any
    # invertible one (ABI 4)
    assert create_rocket_6dof(I_sp=25.0).matches_device_model()
    J = np.diag([0.02, 1.0, 1.0]) * 0.168; J[0, 1] = J[1, 0] = 0.01
    assert create_rocket_6dof(J_B=J).matches_device_model()


def test_gpmpc_dispatches_on_the_state_dimension():
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFConfig, Rocket6DoFDynamics
    from gp_mpc_rocket_landing_amd.gp.structured_gp import StructuredRocketGP
    from gp_mpc_rocket_landing_amd.mpc import CostWeights, GPMPC, GPMPCConfig
    from gp_mpc_rocket_landing_amd.mpc.gp_mpc import GPMPC6DoF
    gp = StructuredRocketGP()
    m = GPMPC(Rocket6DoFDynamics(), gp)          # GPMPCConfig(): the reference's N = 20
    assert isinstance(m, GPMPC6DoF) and isinstance(m, GPMPC) and m.config.N == 20
    assert m._cfg_kw["fitc_mean_as_written"] == 1 and m._cfg_kw["horizon"] == 20
    assert GPMPC(Rocket6DoFDynamics(), gp, GPMPCConfig(N=30))._cfg_kw["horizon"] == 30
    assert GPMPC(Rocket6DoFDynamics(), gp, GPMPCConfig(N=15))._cfg_kw["horizon"] == 15   # any N in 2..30
    for bad in (1, 31):
        with pytest.raises(NotImplementedError):    # outside the compiled horizons
            GPMPC(Rocket6DoFDynamics(), gp, GPMPCConfig(N=bad))
    # a non-default rocket reaches the device config (rocket_6dof.py:36-84 fields)
    k = GPMPC(Rocket6DoFDynamics(Rocket6DoFConfig(I_sp=20.0, g0=2.0, r_T_B=np.array([-0.3, 0.01, 0.0]))),
              gp)._cfg_kw
    assert k["rocket_alpha"] == 1.0 / 40.0 and k["rocket_g0"] == 2.0
    np.testing.assert_array_equal(k["rocket_r_t"], [-0.3, 0.01, 0.0])
    np.testing.assert_array_equal(k["rocket_j"], np.array([0.02, 1.0, 1.0]) * 0.168)
    assert "rocket_J" not in k                   # diagonal: the diagonal model
    J = np.diag([0.02, 1.0, 1.0]) * 0.168; J[0, 2] = J[2, 0] = 0.01
    k = GPMPC(Rocket6DoFDynamics(Rocket6DoFConfig(J_B=J)), gp)._cfg_kw   # a full tensor goes through
    np.testing.assert_array_equal(k["rocket_J"], J.reshape(9))
    c = __import__("gp_mpc_rocket_landing_amd._lib", fromlist=["x"]).rollout6_default_config(**{
        kk: v for kk, v in k.items() if kk.startswith("rocket_")})
    np.testing.assert_array_equal(np.array(c.rocket_J), J.reshape(9))
    Q = CostWeights().Q.copy(); Q[1, 2] = Q[2, 1] = 0.5
    with pytest.raises(NotImplementedError):
        GPMPC(Rocket6DoFDynamics(), gp, cost_weights=CostWeights(Q=Q))


def test_rollout6_default_config_is_the_reference_problem():
    """gpmpc_rollout6_default_config: CostWeights, ConstraintParams, trust
    radii, the osqp_rti settings; ctypes reads every field where C wrote it."""
    from gp_mpc_rocket_landing_amd import _lib
    from gp_mpc_rocket_landing_amd.mpc import ConstraintParams, CostWeights
    c = _lib.rollout6_default_config()
    cw, cp = CostWeights(), ConstraintParams()
    np.testing.assert_array_equal(np.array(c.q_diag), np.diag(cw.Q))
    np.testing.assert_array_equal(np.array(c.p_diag), np.diag(cw.P))
    np.testing.assert_array_equal(np.array(c.r_diag), np.diag(cw.R))
    assert (c.t_min, c.t_max) == (cp.T_min, cp.T_max)
    assert c.tan_gamma_gs == np.tan(cp.gamma_gs_rad)
    assert (c.trust_x2, c.trust_u2, c.use_gp_mean, c.upright_target) == (10.0, 5.0, 1, 0)
    assert c.horizon == 30 and c.qp.max_iter == 50 and c.qp.eps_abs == 1e-4
    assert c.fitc_mean_as_written == 1   # the reference's arithmetic by default
    # Rocket6DoFConfig defaults (rocket_6dof.py:36-84)
    np.testing.assert_array_equal(np.array(c.rocket_j), np.array([0.02, 1.0, 1.0]) * 0.168)
    assert list(c.rocket_r_t) == [-0.25, 0.0, 0.0] and list(c.rocket_g_i) == [-1.0, 0.0, 0.0]
    assert c.rocket_alpha == 1.0 / 30.0 and c.rocket_g0 == 1.0
    c2 = _lib.rollout6_default_config(q_diag=np.arange(14.0), max_iter=7)
    assert list(c2.q_diag) == list(range(14)) and c2.qp.max_iter == 7
    with pytest.raises(ValueError):
        _lib.rollout6_default_config(r_diag=[1.0, 2.0])


def test_cross3_is_np_cross_bitwise():
    """rocket_6dof._cross3 (the dynamics' 3-vector cross product) forms np.cross's
    products and differences in the same order: identical bits."""
    from gp_mpc_rocket_landing_amd.dynamics.rocket_6dof import _cross3
    rs = np.random.RandomState(0)
    for _ in range(20000):
        a = rs.randn(3) * 10 ** rs.uniform(-6, 6, 3)
        b = rs.randn(3) * 10 ** rs.uniform(-6, 6, 3)
        assert np.array_equal(np.cross(a, b), _cross3(a, b))
