"""The product's Monte-Carlo protocol (gp_mpc_rocket_landing_amd.experiments)
against the reference's own outputs, and the oracle's full-size Monte-Carlo
fixture against the live oracle (CPU).

* sample_initial_condition (monte_carlo.py:368-399) vs F7, both configs;
* LandingConstraints.check_landing (monte_carlo.py:54-104) vs F8, both
  tolerance sets, reason text;
* tests/golden/mc_oracle_1024.npz (gen_mc_oracle.py) re-derived on a sample
  of landings covering every outcome it holds.
"""
import numpy as np
import pytest

from conftest import golden


def test_product_initial_conditions_match_f7():
    from gp_mpc_rocket_landing_amd.experiments.monte_carlo import (SimulationConfig,
                                                                   sample_initial_condition)
    from gp_mpc_rocket_landing_amd.fleet import initial_conditions
    f = golden("f7_mc_initial_conditions.npz")
    cfg = SimulationConfig.run_experiments()
    x0 = np.array([sample_initial_condition(42 + i, cfg) for i in range(1024)])
    np.testing.assert_array_equal(x0, f["x0_run_experiments"])
    np.testing.assert_array_equal(initial_conditions(1024), f["x0_run_experiments"])
    np.testing.assert_array_equal(initial_conditions(24, first=1000), f["x0_run_experiments"][1000:])
    x0d = np.array([sample_initial_condition(42 + i, SimulationConfig()) for i in range(16)])
    np.testing.assert_array_equal(x0d, f["x0_default"])


def test_product_check_landing_matches_f8():
    from gp_mpc_rocket_landing_amd.experiments.monte_carlo import LandingConstraints, SimulationConfig
    f = golden("f8_check_landing.npz")
    for k, lc in enumerate((LandingConstraints(), SimulationConfig.run_experiments().landing_constraints)):
        for s, m, ok, reason in zip(f["states"], f["m0"], f["ok"][k], f["reason"][k]):
            r_ok, r_reason = lc.check_landing(s, m)
            assert int(r_ok) == int(ok), (s, m, k)
            assert r_reason.split(":")[0] == str(reason), (r_reason, reason)


@pytest.fixture(scope="module")
def gp_state():
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from threadpoolctl import threadpool_limits
    from oracle import gp_oracle
    X, U, D = synthetic_training_data(1000, seed=0)
    with threadpool_limits(1):   # the fixture generator's BLAS threading
        return gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)


def test_mc_oracle_fixture_is_the_oracle(gp_state):
    """Rows of the committed full-size fixture re-derived live: a fuel-exhausted,
    a constraint-violation and a successful landing, bit-identical records."""
    from threadpoolctl import threadpool_limits
    from oracle import mc_oracle
    R = golden("mc_oracle_1024.npz")["records"]
    oc = R[:, 0].astype(int)
    assert sorted(set(oc.tolist())) == [1, 3, 4]
    assert (oc == 1).sum() == 838 and (oc == 3).sum() == 2 and (oc == 4).sum() == 184
    for i in (int(np.nonzero(oc == 3)[0][0]), int(np.nonzero(oc == 4)[0][0]), 0):
        with threadpool_limits(1):   # the generator's BLAS threading (summation order)
            rec, x, trace = mc_oracle.closed_loop_landing(gp_state, mc_oracle.sample_initial_condition(42 + i))
        np.testing.assert_array_equal(rec, R[i])
        assert len(trace) == int(rec[1]) and sum(t[0] for t in trace) == rec[11]


def test_landing_step_termination_rules():
    """The termination branch of the oracle's step (monte_carlo.py:455-488 order:
    timeout first once max_steps ran, then crash, fuel, divergence, landing)."""
    from oracle import mc_oracle
    S = mc_oracle.new_landing(mc_oracle.sample_initial_condition(42))
    cases = [  # (state edits, steps so far, expected outcome)
        ({1: -0.1}, 0, mc_oracle.CRASH),
        ({0: 1.01}, 0, mc_oracle.FUEL_EXHAUSTED),
        ({5: 2e6}, 0, mc_oracle.DIVERGENCE),
        ({6: np.nan}, 0, mc_oracle.DIVERGENCE),
        ({1: 0.5, 4: -1.0, 2: 0.0, 3: 0.0, 5: 0.0, 6: 0.0}, 0, mc_oracle.SUCCESS),
        ({1: 0.5, 4: -1.0, 2: 6.0}, 0, mc_oracle.CONSTRAINT_VIOLATION),
        ({1: -0.1}, 300, mc_oracle.TIMEOUT),
    ]
    for edits, steps, want in cases:
        T = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in S.items()}
        for i, v in edits.items():
            T["x"][i] = v
        T["rec"][1] = steps
        out, info = mc_oracle.landing_step(None, T)
        assert info is None and int(out["rec"][0]) == want, (edits, steps, out["rec"][0])
        np.testing.assert_array_equal(out["rec"][4:11], T["x"])
