"""The reference's own 14-state GPMPC.solve on the device:
``GPMPC(Rocket6DoFDynamics(), StructuredRocketGP, GPMPCConfig())`` (N = 20, or
N = 30 for BASELINE configs[4]) runs csrc/fleet6.hip at a batch of one
(gpmpc_rollout6_solve_ref) and is checked per
control step against oracle/sixdof_oracle.gpmpc_solve (gp_mpc.py:229-369
restated, the QP made linear as the rollouts, the C OSQP-0.6 restatement),
from the device's own previous controller state (warm-start U, scaled duals,
rho) so that the inputs are identical: QP status, ADMM iterations, SQP passes
and convergence exact; plan X, U within the SURVEY 8c tolerance (1e-6
relative, unit floor).  The closed loop is the Monte-Carlo solve protocol
(monte_carlo.py:495-512: incremental target, u0 into the plant)."""
import numpy as np
import pytest

from conftest import close
from test_gpu_rollouts6 import oracle_gps

pytestmark = pytest.mark.gpu


def _surface(n_train=300, n_inducing=50, use_sparse=True):
    from gp_mpc_rocket_landing_amd.rollouts6 import fit_structured_gp
    return fit_structured_gp(n_train, n_inducing, seed=0, use_sparse=use_sparse)


def _target(x):
    """monte_carlo.py:497-500."""
    t = x.copy()
    t[4:7] = 0.0
    t[1] = max(0.5, x[1] - 2.0)
    return t


def _fly(gp, steps, max_sqp_iter, seed_index=0, tol=1e-6, device_alpha=False, N=30, rocket_cfg=None,
         config=None, refs=False):
    """``rocket_cfg``: a Rocket6DoFConfig for the plant and the oracle; ``config``:
    the GPMPCConfig as given (default GPMPCConfig(N, max_sqp_iter)); ``refs``: a
    reference trajectory X_ref (a straight line from x to the target over the
    horizon) and controls U_ref (hover thrust) in every solve (gp_mpc.py:442-453,
    U_ref also the first guess, :268-269)."""
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFConfig, Rocket6DoFDynamics
    from gp_mpc_rocket_landing_amd.mpc import GPMPC, GPMPCConfig
    from gp_mpc_rocket_landing_amd.rollouts6 import initial_conditions_6dof, qp_rows
    from oracle import sixdof_oracle as so
    ov, ow = oracle_gps(gp)
    if device_alpha:  # the oracle loop on the device fit's coefficients (fit pinned elsewhere)
        ov = dict(ov, alpha=gp.gp_v.device_handle.alpha())
        ow = dict(ow, alpha=gp.gp_omega.device_handle.alpha())
    rc = rocket_cfg or Rocket6DoFConfig()
    dyn = Rocket6DoFDynamics(rc)
    rk = so.rocket_params(np.asarray(rc.J_B, float), rc.r_T_B, rc.g_I, rc.I_sp, rc.g0)
    cfg = config or GPMPCConfig(N=N, max_sqp_iter=max_sqp_iter, use_gp_uncertainty=False)
    N, max_sqp_iter = cfg.N, cfg.max_sqp_iter
    from oracle import admm_ref
    mi, eps = cfg.qp_settings()
    qs = admm_ref.default_settings(max_iter=int(mi), eps_abs=float(eps), eps_rel=float(eps))
    mpc = GPMPC(dyn, gp, cfg)
    assert type(mpc).__name__ == "GPMPC6DoF" and isinstance(mpc, GPMPC)
    x = initial_conditions_6dof(seed_index + 1)[seed_index]
    S = dict(U=so.hover_guess(x, N, rc.g0), y=np.zeros(qp_rows(N)), rho=0.1)
    seen = []
    try:
        for k in range(steps):
            xt = _target(x)
            Xr = Ur = None
            if refs:
                a = (np.arange(N + 1) / N)[:, None]
                Xr = (1 - a) * x + a * xt
                Ur = np.tile([0.0, 0.0, 0.9 * x[0] * rc.g0], (N, 1))
                if k == 0:
                    S["U"] = Ur.copy()   # U_ref as the first guess
            sol = mpc.solve(x, xt, X_ref=Xr, U_ref=Ur)
            want = so.gpmpc_solve(ov, ow, S, x, xt, max_sqp_iter=max_sqp_iter, sqp_tol=cfg.sqp_tol,
                                  corrected=False, rk=rk, X_ref=Xr, U_ref=Ur, qp_settings=qs)
            tag = (k, max_sqp_iter)
            assert mpc.last_status == want["qp_status"], (tag, mpc.last_status, want["qp_status"])
            assert mpc.last_iterations == want["qp_iters"], (tag, mpc.last_iterations, want["qp_iters"])
            assert mpc.last_passes == want["passes"], (tag, mpc.last_passes, want["passes"])
            if max_sqp_iter > 1:
                assert sol.success == want["converged"] and sol.iterations == want["passes"], tag
            else:
                assert sol.success == (want["qp_status"] in (1, 2, -2)), tag
            for key, got in (("X", sol.X_opt), ("U", sol.U_opt)):
                ok, worst = close(got, want[key], 1.0, rtol=tol)
                assert ok, (tag, key, worst)
            if np.isfinite(sol.cost):
                ok, worst = close(sol.cost, so.solution_cost(want["X"], want["U"], xt if Xr is None else Xr,
                                                             U_ref=Ur), 1.0, rtol=tol)
                assert ok, (tag, "cost", worst)
            seen.append((want["qp_status"], want["qp_iters"], want["passes"], want["converged"]))
            st = mpc._ro.state()   # the device's controller state for the next step's oracle
            S = dict(U=st["U"][0], y=st["y"][0], rho=float(st["rho"][0]))
            if not sol.success and max_sqp_iter <= 1:
                break
            x = so.truth_step(x, sol.u0, 0.1, rk)
    finally:
        mpc.close()
    return seen


def test_gpmpc6_reference_defaults_n20():
    """``GPMPC(Rocket6DoFDynamics(), gp, GPMPCConfig())`` -- the
    reference docstring's call (gp_mpc.py:85), N = 20 (gp_mpc.py:110), the
    default uncertainty propagation on -- runs on the device and matches the
    oracle over 10 control steps: status, iterations, passes exact, plans 1e-6."""
    from gp_mpc_rocket_landing_amd.mpc import GPMPCConfig
    seen = _fly(_surface(), 10, 1, config=GPMPCConfig())
    assert len(seen) >= 10, seen


def test_gpmpc6_reference_loop_n20():
    """The reference's 10-pass loop at N = 20 (GPMPCConfig(max_sqp_iter=10))."""
    from gp_mpc_rocket_landing_amd.mpc import GPMPCConfig
    seen = _fly(_surface(), 6, 10, config=GPMPCConfig(max_sqp_iter=10, use_gp_uncertainty=False))
    assert len(seen) == 6, seen


def test_gpmpc6_nondefault_rocket():
    """A Rocket6DoFConfig other than the default (diagonal J_B, r_T_B, g_I,
    I_sp, g0) at N = 20 and N = 30: the device dynamics, Jacobians and hover
    guess take the caller's rocket; 8 steps each vs the oracle with it."""
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFConfig
    rc = Rocket6DoFConfig(J_B=np.diag([0.03, 1.1, 0.9]) * 0.168, r_T_B=np.array([-0.3, 0.0, 0.02]),
                          g_I=np.array([-1.0, 0.01, 0.0]), I_sp=25.0, g0=1.05)
    for N in (20, 30):
        seen = _fly(_surface(), 8, 1, N=N, rocket_cfg=rc)
        assert len(seen) >= 8, (N, seen)


# a full inertia tensor: products of inertia ~10% of the principal moments (and a
# strong one between the two transverse axes), symmetric positive definite
J_FULL = np.array([[0.02, 0.004, -0.002], [0.004, 1.0, 0.03], [-0.002, 0.03, 0.95]]) * 0.168


def test_gpmpc6_full_inertia_tensor():
    """VERDICT r5 missing #1: Rocket6DoFConfig.J_B is any 3 x 3 array
    (rocket_6dof.py:44, 77-78, 147) and the reference's dynamics solve with it
    (nominal_mpc.py:196-199: w' = J^-1 (r_T x u - w x J w)).  A non-diagonal J_B goes
    through GPMPC to the device (rocket_J, ABI 4) and matches the oracle with the
    same tensor per control step at N = 20 and N = 30 (status, iterations, passes
    exact, plans 1e-6), and in the reference's 10-pass loop at N = 20."""
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFConfig
    from gp_mpc_rocket_landing_amd.mpc import GPMPCConfig
    rc = Rocket6DoFConfig(J_B=J_FULL)
    for N in (20, 30):
        seen = _fly(_surface(), 8, 1, N=N, rocket_cfg=rc)
        assert len(seen) >= 8, (N, seen)
    seen = _fly(_surface(), 4, 10, rocket_cfg=rc, config=GPMPCConfig(max_sqp_iter=10, use_gp_uncertainty=False))
    assert len(seen) == 4, seen


def test_gpmpc6_any_horizon():
    """MPCConfig.N is a free integer in the reference
    (nominal_mpc.py:47, gp_mpc.py:253, 392); the device controller is compiled for
    every N from 2 to 30, odd ones included (the twisted factor's bottom end then
    has one block step fewer).  N = 15 (OSQPRTIConfig's default horizon), the odd
    extremes 3 and 29, and 2: RTI steps vs the oracle."""
    for N, steps in ((15, 8), (3, 4), (2, 4), (29, 4)):
        seen = _fly(_surface(), steps, 1, N=N)
        assert len(seen) >= steps, (N, seen)
    seen = _fly(_surface(), 4, 10, N=15)   # the reference's 10-pass loop at N = 15
    assert len(seen) >= 4, seen


def test_gpmpc6_reference_trajectory():
    """X_ref / U_ref in the QP cost (gp_mpc.py:442-453) and U_ref as the first
    guess (:268-269), RTI and the 10-pass loop, N = 20."""
    for passes in (1, 10):
        seen = _fly(_surface(), 8, passes, N=20, refs=True)
        assert len(seen) >= 8, (passes, seen)


def test_gpmpc6_rti_step_matches_oracle():
    """max_sqp_iter = 1 (the RTI control step, D14): 12 closed-loop steps."""
    seen = _fly(_surface(), 12, 1)
    assert len(seen) >= 10, seen


def test_gpmpc6_reference_loop_matches_oracle():
    """The reference's loop: up to 10 linearise -> GP -> QP passes per solve,
    stop at 1e-4 (gp_mpc.py:296-345); passes and convergence exact."""
    seen = _fly(_surface(), 10, 10)
    assert len(seen) == 10 and all(p >= 1 for _, _, p, _ in seen), seen


def test_gpmpc6_exact_structured_gp():
    """StructuredRocketGP(use_sparse=False): the device mean is K* alpha over
    the training rows (gpmpc_rollout6_create_exact)."""
    seen = _fly(_surface(n_train=200, use_sparse=False), 10, 1)
    assert len(seen) >= 10, seen


def test_gpmpc6_config5_gp():
    """BASELINE configs[4]'s GP (M = 2000 kmeans2 inducing points, N = 4000
    rows) through the surface, 6 control steps of the reference loop (10
    passes).  At this size K_uu is badly conditioned: the as-written mean
    K*u alpha of the device fit and of the numpy fit agree only to ~3e-7
    absolute (|mean| ~ 10, measured), and the reference loop does not
    contract (its c_k = GP mean dt has no fixed point with dX = 0, DESIGN.md
    section 9), so passes amplify that fit-level difference.  The fit is
    pinned by the FITC parity tests at this size; here the oracle loop runs on
    the device fit's alpha (gpmpc_fitc_get_state), which isolates the control
    loop: statuses / iterations / passes exact, plans at 1e-6."""
    seen = _fly(_surface(n_train=4000, n_inducing=2000), 6, 10, device_alpha=True)
    assert len(seen) == 6, seen


def test_gpmpc6_warm_start_survives_gp_refit():
    """A refit of the GP rebuilds the device controller and carries the
    warm-start controls, duals and rho (gpmpc_rollout6_set_state)."""
    from gp_mpc_rocket_landing_amd.dynamics import Rocket6DoFDynamics
    from gp_mpc_rocket_landing_amd.mpc import GPMPC, GPMPCConfig
    from gp_mpc_rocket_landing_amd.rollouts6 import initial_conditions_6dof
    gp = _surface()
    mpc = GPMPC(Rocket6DoFDynamics(), gp, GPMPCConfig(N=30, use_gp_uncertainty=False))
    try:
        x = initial_conditions_6dof(1)[0]
        mpc.solve(x, _target(x))
        before = mpc._ro.state()
        gp.fit()
        h0 = mpc._ro
        mpc._rollout()
        assert mpc._ro is not h0
        after = mpc._ro.state()
        for k in ("U", "y", "rho"):
            np.testing.assert_array_equal(after[k], before[k])
    finally:
        mpc.close()


def test_gpmpc6_solved_setting():
    """The 14-state GPMPC with the >= 90%-solved ADMM setting (qp_max_iter 4000,
    GPMPCConfig's QP knobs) at N = 20: 6 RTI steps vs the oracle."""
    import bench
    from gp_mpc_rocket_landing_amd.mpc import GPMPCConfig
    cfg = GPMPCConfig(qp_max_iter=bench.SOLVED_QP6["max_iter"], qp_eps=bench.SOLVED_QP6["eps_abs"],
                      use_gp_uncertainty=False)
    seen = _fly(_surface(), 6, 1, config=cfg)
    assert len(seen) >= 6, seen
