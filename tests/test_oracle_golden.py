"""The CPU oracle against the reference's own outputs (golden fixtures F1-F12).

These pin the oracle before it is trusted as the parity checker for the HIP path.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import close, golden
from oracle import admm_oracle, admm_ref, gp_oracle, mc_oracle, qp_oracle


def test_f3_kernels():
    f = golden("f3_kernels.npz")
    X1, X2, ls, s2 = f["X1"], f["X2"], f["ls"], float(f["sigma2"])
    np.testing.assert_allclose(gp_oracle.gram("se_ard", X1, X2, s2, ls), f["se_ard"], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(gp_oracle.gram("se_ard", X1, None, s2, ls), f["se_ard_self"], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(gp_oracle.gram("matern32", X1, X2, s2, ls), f["matern32"], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(gp_oracle.gram("matern52", X1, X2, s2, ls), f["matern52"], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(gp_oracle.gram("se_iso", X1, X2, s2, [float(f["iso_l"])]), f["se_iso"], rtol=1e-13, atol=1e-15)
    s = gp_oracle.gram("se_ard", X1, X2, s2, ls) + gp_oracle.gram("matern32", X1, X2, 0.3, ls)
    np.testing.assert_allclose(s, f["sum_se_m32"], rtol=1e-13, atol=1e-15)
    p = gp_oracle.gram("se_ard", X1, X2, s2, ls) * gp_oracle.gram("matern52", X1, X2, 0.5, ls)
    np.testing.assert_allclose(p, f["prod_se_m52"], rtol=1e-13, atol=1e-15)


def test_f1_features_and_exact_gp():
    f = golden("f1_exact_simple3dof.npz")
    Z = gp_oracle.features_3dof(f["X"], f["U"])
    np.testing.assert_allclose(Z, f["Z"], rtol=1e-14, atol=1e-15)
    st = gp_oracle.exact_fit(Z, f["D"])
    assert st["jitter_steps"] == 0
    np.testing.assert_allclose(np.diag(st["L"]), f["diagL"], rtol=1e-10)
    np.testing.assert_allclose(st["y_mean"], f["y_mean"], rtol=1e-14)
    np.testing.assert_allclose(st["y_std"], f["y_std"], rtol=1e-14)
    np.testing.assert_allclose(st["lml"], f["lml"], rtol=1e-8)
    mean, var = gp_oracle.exact_predict(st, gp_oracle.features_3dof(f["Xq"], f["Uq"]))
    ok, e = close(mean, f["mean"], f["y_std"]); assert ok, e
    ok, e = close(var, f["var"], f["y_std"] ** 2); assert ok, e
    m1, v1 = gp_oracle.exact_predict(st, gp_oracle.features_3dof(f["Xq"][:1], f["Uq"][:1]))
    ok, e = close(m1[0], f["single_mean"], f["y_std"]); assert ok, e
    ok, e = close(v1[0], f["single_var"], f["y_std"] ** 2); assert ok, e


def test_f2_small_exact_jitter_and_cov():
    f = golden("f2_exact_small.npz")
    st = gp_oracle.exact_fit(f["X"], f["Y"], noise=1e-3)
    np.testing.assert_allclose(st["L"], f["L"], rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(st["alpha"], f["alpha"], rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(st["lml"], f["lml"], rtol=1e-10)
    mean, var = gp_oracle.exact_predict(st, f["Xq"])
    np.testing.assert_allclose(mean, f["mean"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(var, f["var"], rtol=1e-9, atol=1e-12)
    mc, cov = gp_oracle.exact_predict_cov(st, f["Xq"], out=1)
    np.testing.assert_allclose(mc, f["cov_mean"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(cov, f["cov"], rtol=1e-8, atol=1e-12)
    # jitter ladder (exact_gp.py:163-175)
    sd = gp_oracle.exact_fit(f["Xdup"], f["ydup"], noise=-1e-7)
    assert gp_oracle.jitter_ladder()[sd["jitter_steps"] - 1] == float(f["dup_jitter"])
    np.testing.assert_allclose(sd["L"], f["dup_L"], rtol=1e-9, atol=1e-12)
    with pytest.raises(ValueError, match="not positive definite"):
        gp_oracle.exact_fit(f["X"], f["Y"][:, 0], noise=-5.0)
    assert int(f["neg_noise_raises"]) == 1


def test_jitter_ladder_values():
    lad = gp_oracle.jitter_ladder()
    assert lad[0] == 1e-6 and len(lad) == 6 and lad[-1] < 1.0
    assert lad[1] == 9.999999999999999e-06  # repeated multiplication, not 10**k


def test_f4_fitc():
    f = golden("f4_fitc_simple3dof.npz")
    X = gp_oracle.features_3dof(f["X"], f["U"])
    st = gp_oracle.fitc_fit(f["Zi"], X, f["D"])
    np.testing.assert_allclose(st["lam"], f["lam"], rtol=1e-9, atol=1e-15)
    np.testing.assert_allclose(np.diag(st["Luu"]), f["diagLuu"], rtol=1e-12)
    np.testing.assert_allclose(st["alpha"], f["alpha"], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(st["lml"], f["lml"], rtol=1e-8)
    mean, var = gp_oracle.fitc_predict(st, f["Zq"])
    ok, e = close(mean, f["mean"], f["y_std"]); assert ok, e
    ok, e = close(var, f["var"], f["y_std"] ** 2); assert ok, e


def test_f12_vfe():
    """SparseGP(method="vfe") restated (gp_oracle.vfe_fit) vs the reference's own fit."""
    f = golden("f12_vfe_3dof.npz")
    st = gp_oracle.vfe_fit(f["Zi"], f["Z"], f["Y"], float(f["sigma2"]), f["ls"], float(f["noise"]),
                           float(f["jitter"]))
    mean, var = gp_oracle.fitc_predict(st, f["Zq"])
    for c in range(2):
        np.testing.assert_allclose(np.diag(st["LB"]), f[f"diagLB{c}"], rtol=1e-12)
        np.testing.assert_allclose(st["alpha"][:, c], f[f"alpha{c}"], rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(st["lml"][c], f[f"lml{c}"], rtol=1e-9)
        ok, e = close(mean[:, c], f[f"mean{c}"], st["y_std"][c]); assert ok, e
        ok, e = close(var[:, c], f[f"var{c}"], st["y_std"][c] ** 2); assert ok, e


def test_f5_structured_features():
    f = golden("f5_structured_6dof.npz")
    np.testing.assert_allclose(gp_oracle.features_translational(f["X"], f["U"]), f["Zv"], rtol=1e-13, atol=1e-14)
    np.testing.assert_allclose(gp_oracle.features_rotational(f["X"], f["U"]), f["Zw"], rtol=1e-13, atol=1e-14)
    Zv = gp_oracle.features_translational(f["X"], f["U"])
    Zw = gp_oracle.features_rotational(f["X"], f["U"])
    sv = gp_oracle.exact_fit(Zv, f["Dv"]); sw = gp_oracle.exact_fit(Zw, f["Dw"])
    mv, vv = gp_oracle.exact_predict(sv, gp_oracle.features_translational(f["Xq"], f["Uq"]))
    mw, vw = gp_oracle.exact_predict(sw, gp_oracle.features_rotational(f["Xq"], f["Uq"]))
    for a, b, s in ((mv, f["exact_dv_mean"], sv["y_std"]), (mw, f["exact_dw_mean"], sw["y_std"]),
                    (vv, f["exact_dv_var"], sv["y_std"] ** 2), (vw, f["exact_dw_var"], sw["y_std"] ** 2)):
        ok, e = close(a, b, s); assert ok, e
    fv = gp_oracle.fitc_fit(f["fitc_Zv"], Zv, f["Dv"]); fw = gp_oracle.fitc_fit(f["fitc_Zw"], Zw, f["Dw"])
    mv, vv = gp_oracle.fitc_predict(fv, gp_oracle.features_translational(f["Xq"], f["Uq"]))
    mw, vw = gp_oracle.fitc_predict(fw, gp_oracle.features_rotational(f["Xq"], f["Uq"]))
    for a, b, s in ((mv, f["fitc_dv_mean"], fv["y_std"]), (mw, f["fitc_dw_mean"], fw["y_std"]),
                    (vv, f["fitc_dv_var"], fv["y_std"] ** 2), (vw, f["fitc_dw_var"], fw["y_std"] ** 2)):
        ok, e = close(a, b, s); assert ok, e


def test_f6_qp_assembly():
    f = golden("f6_qp_assembly.npz")
    for i in range(int(f["ncases"])):
        X, U, x0, xt = f[f"c{i}_X"], f[f"c{i}_U"], f[f"c{i}_x0"], f[f"c{i}_xt"]
        P, q = qp_oracle.cost(20, np.tile(xt, (21, 1)))
        A, l, u = qp_oracle.constraints(X, U, x0, 0.1, sign=+1.0)
        Pr = sp.csc_matrix((f[f"c{i}_P_data"], f[f"c{i}_P_indices"], f[f"c{i}_P_indptr"]), shape=P.shape)
        Ar = sp.csc_matrix((f[f"c{i}_A_data"], f[f"c{i}_A_indices"], f[f"c{i}_A_indptr"]), shape=A.shape)
        assert (P != Pr).nnz == 0
        np.testing.assert_array_equal(A.indptr, Ar.indptr)
        np.testing.assert_array_equal(A.indices, Ar.indices)
        np.testing.assert_allclose(A.data, Ar.data, rtol=1e-15, atol=0)
        np.testing.assert_allclose(q, f[f"c{i}_q"], rtol=0, atol=0)
        np.testing.assert_allclose(l, f[f"c{i}_l"], rtol=1e-14, atol=1e-14)
        np.testing.assert_allclose(u, f[f"c{i}_u"], rtol=1e-14, atol=1e-14)
        Ak, Bk = qp_oracle.linearize(X[0], U[0], 0.1)
        np.testing.assert_allclose(Ak, f[f"c{i}_A0"], rtol=1e-15)
        np.testing.assert_allclose(Bk, f[f"c{i}_B0"], rtol=1e-15)
        np.testing.assert_array_equal(qp_oracle.to_vector(X, U), f[f"c{i}_zvec"])
    # pattern depends on values
    assert len(f["c0_A_data"]) == 654 and len(f["c1_A_data"]) == 734


def test_f7_initial_conditions():
    f = golden("f7_mc_initial_conditions.npz")
    x0 = np.array([mc_oracle.sample_initial_condition(42 + i) for i in range(1024)])
    np.testing.assert_array_equal(x0, f["x0_run_experiments"])
    x0d = np.array([mc_oracle.sample_initial_condition(42 + i, mc_oracle.DEFAULT_CFG) for i in range(16)])
    np.testing.assert_array_equal(x0d, f["x0_default"])


def test_f8_check_landing():
    f = golden("f8_check_landing.npz")
    for k, cfg in enumerate((mc_oracle.DEFAULT_CFG, mc_oracle.RUN_EXPERIMENTS_CFG)):
        for s, m, ok, reason in zip(f["states"], f["m0"], f["ok"][k], f["reason"][k]):
            r = mc_oracle.check_landing(s, m, cfg)
            assert int(r[0]) == int(ok) and r[1] == str(reason)


def _qp_case(seed, N=20):
    rs = np.random.RandomState(seed)
    x0 = np.array([2.0, 30, 1, -1, -3, 0.2, 0.1]) + rs.randn(7) * [0.1, 3, 1, 1, 0.5, 0.2, 0.2]
    xt = mc_oracle.incremental_target(x0)
    X, U = qp_oracle.initial_guess(x0, xt, N)
    P, q = qp_oracle.cost(N, np.tile(xt, (N + 1, 1)))
    A, l, u = qp_oracle.constraints(X, U, x0, 0.1, gp_dv=rs.randn(N, 3) * 0.01, sign=-1.0)
    return P, q, A, l, u, qp_oracle.to_vector(X, U)


@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4, 5])
def test_admm_c_port_matches_numpy_kkt_oracle(seed):
    """The fast C restatement (reduced banded KKT) vs the numpy KKT-LU restatement:
    identical status / iteration counts / adaptive-rho decisions, x within 1e-6 rel."""
    P, q, A, l, u, xw = _qp_case(seed)
    a = admm_oracle.OSQPOracle(P, q, A, l, u); a.warm_start_x(xw)
    b = admm_ref.RefQP(A.shape[0])
    for rep in range(2):
        ra = a.solve(); rb = b.solve(P.diagonal(), q, A, l, u, xw)
        assert ra["status"] == rb["status"] and ra["iter"] == rb["iter"]
        assert abs(ra["rho"] - rb["rho"]) <= 1e-6 * ra["rho"]
        ok, e = close(rb["x"], ra["x"], np.max(np.abs(ra["x"]))); assert ok, e
        a.update(P, q, A, l, u); a.warm_start_x(ra["x"]); xw = rb["x"]


def test_admm_kkt_optimality():
    """Solved QPs satisfy the OSQP termination criteria in unscaled terms."""
    P, q, A, l, u, xw = _qp_case(11)
    r = admm_ref.RefQP(A.shape[0])
    for _ in range(3):
        res = r.solve(P.diagonal(), q, A, l, u, xw)
        xw = res["x"]
    assert res["status"] in (1, 2)
    Ax = A @ res["x"]
    assert np.all(Ax >= l - 1e-2) and np.all(Ax <= u + 1e-2)


def test_f9_linear_propagation_oracle():
    """The numpy restatement of _propagate_linear against the reference's own
    output (exact StructuredRocketGP on F5, toy 14-state plant)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from toy_dynamics import ToyRocket14
    from oracle import uprop_oracle
    f5 = golden("f5_structured_6dof.npz"); f9 = golden("f9_uncertainty_prop.npz")
    gp = uprop_oracle.structured_exact_predictor(f5["X"], f5["U"], f5["Dv"], f5["Dw"])
    means, covs = uprop_oracle.propagate_linear(ToyRocket14(), gp, f9["x0"], f9["U"], None, 0.1)
    np.testing.assert_allclose(means, f9["linear_means"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(covs, f9["linear_covs"], rtol=1e-7, atol=1e-14)


def test_oracle_lml_and_optimiser_vs_f10():
    """SURVEY 8f-3 oracle pinned to F10: the LML objective at 16 parameter sets
    (exact), the 5-step jitter case, and the optimiser's converged refinement
    (exact_gp.py:357-421) from the reference optimum."""
    from oracle import gp_oracle
    f = golden("f10_hyperparameters.npz")
    Z, y = f["Z"], f["y"]
    lml = [gp_oracle.lml_at(Z, y, np.exp(p[0]), np.exp(p[1:-1]), np.exp(p[-1]))[0] for p in f["grid"]]
    np.testing.assert_allclose(lml, f["lml"], rtol=1e-12)
    lj, sj = gp_oracle.lml_at(f["Zd"], f["yd"], 1.0, np.ones(11), -2e-3)
    assert sj == 5 and np.isclose(lj, float(f["lml_jitter"]), rtol=1e-12)
    assert gp_oracle.lml_at(f["Zd"], f["yd"], 1.0, np.ones(11), -10.0) == (-np.inf, -1)
    np.random.seed(5)
    r, p, nz = gp_oracle.optimize_hyperparameters(Z, y, f["ref_start_params"],
                                                  float(f["ref_start_noise"]), n_restarts=1)
    assert r["success"] and bool(f["ref_success"])
    assert abs(r["log_marginal_likelihood"] - float(f["ref_lml"])) < 1e-8 * abs(float(f["ref_lml"]))
    assert np.max(np.abs(p - f["ref_params"])) < 1e-2


def test_f11_kernel_gradients():
    """Oracle gradient restatement vs the reference's gradients (F11)."""
    f = golden("f11_kernel_gradients.npz")
    X1, X2, ls, s2 = f["X1"], f["X2"], f["ls"], float(f["sigma2"])
    for name, kind, l in (("se_ard", "se_ard", ls), ("se_iso", "se_iso", f["iso_l"]),
                          ("matern32", "matern32", ls), ("matern52", "matern52", ls)):
        g = gp_oracle.gram_gradients(kind, X1, X2, s2, l)
        assert len(g) == len(f[f"{name}_x12_names"])
        for j, gj in enumerate(g):
            np.testing.assert_allclose(gj, f[f"{name}_x12_{j}"], rtol=1e-12, atol=1e-14)
    g = gp_oracle.gram_gradients("se_ard", X1, None, s2, ls)
    for j, gj in enumerate(g):
        np.testing.assert_allclose(gj, f[f"se_ard_x11_{j}"], rtol=1e-12, atol=1e-14)


def f13_specs(g):
    """The F13 kernels as gp_oracle composite specs (gen_golden.f13)."""
    ls1, ls2 = g["ls1"], g["ls2"]
    return {"sumwhite": (("sum", ("se_ard", 1.3, ls1), ("white", 2e-3)), 1e-3),
            "prod": (("prod", ("se_ard", 1.1, ls1), ("matern52", 0.9, ls2)), 1e-3),
            "nested": (("sum", ("prod", ("se_iso", 1.2, np.array([2.5])), ("matern32", 0.8, ls2)),
                        ("white", 5e-3)), 1e-3)}


F13_SPARSE = lambda g: ("sum", ("matern52", 1.4, g["ls2"]), ("white", 1e-3))  # noqa: E731


def test_f13_composite_kernels():
    """F13: the reference's ExactGP / SparseGP (FITC, VFE) fitted with composite
    kernels (kernels.py:676-844) -- the oracle's composite specs reproduce alpha,
    LML, diag L, predictions and the full covariance."""
    g = golden("f13_composite_kernels.npz")
    Z, Y, Zq = g["Z"], g["Y"], g["Zq"]
    for name, (spec, noise) in f13_specs(g).items():
        st = gp_oracle.exact_fit(Z, Y[:, :2], kind=spec, noise=noise)
        m, v = gp_oracle.exact_predict(st, Zq)
        for c in range(2):
            ys = st["y_std"][c]
            ok, w = close(st["alpha"][:, c], g[f"{name}_alpha{c}"], np.abs(g[f"{name}_alpha{c}"]).max(), 1e-8)
            assert ok, (name, "alpha", w)
            assert abs(st["lml"][c] - g[f"{name}_lml{c}"]) <= 1e-8 * abs(g[f"{name}_lml{c}"])
            ok, w = close(np.diag(st["L"]), g[f"{name}_diagL{c}"], 1.0, 1e-10); assert ok, (name, "L", w)
            ok, w = close(m[:, c], g[f"{name}_mean{c}"], ys, 1e-8); assert ok, (name, "mean", w)
            ok, w = close(v[:, c], g[f"{name}_var{c}"], st["sigma2"] * ys ** 2, 1e-8); assert ok, (name, "var", w)
    st = gp_oracle.exact_fit(Z, Y[:, :1], kind=f13_specs(g)["sumwhite"][0], noise=1e-3)
    mc, cov = gp_oracle.exact_predict_cov(st, Zq)
    ok, w = close(cov, g["sumwhite_cov0"], 1.0, 1e-8); assert ok, ("cov", w)
    ok, w = close(mc, g["sumwhite_covmean0"], st["y_std"][0], 1e-8); assert ok, ("covmean", w)
    for method, fit in (("fitc", gp_oracle.fitc_fit), ("vfe", gp_oracle.vfe_fit)):
        st = fit(g["Zi"], Z, Y[:, :2], noise=2e-2, kind=F13_SPARSE(g))
        m, v = gp_oracle.fitc_predict(st, Zq)
        for c in range(2):
            ys = st["y_std"][c]
            ok, w = close(st["alpha"][:, c], g[f"{method}_alpha{c}"], np.abs(g[f"{method}_alpha{c}"]).max(), 1e-8)
            assert ok, (method, "alpha", w)
            assert abs(st["lml"][c] - g[f"{method}_lml{c}"]) <= 1e-8 * abs(g[f"{method}_lml{c}"]), method
            ok, w = close(m[:, c], g[f"{method}_mean{c}"], ys, 1e-8); assert ok, (method, "mean", w)
            ok, w = close(v[:, c], g[f"{method}_var{c}"], st["sigma2"] * ys ** 2, 1e-8); assert ok, (method, "var", w)
