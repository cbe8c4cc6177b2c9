"""Generate the golden fixtures F1-F13 (plus F9-F13 of later rounds) from the reference itself.

Container-only: it imports /root/reference/src/{gp,mpc,experiments} through a
namespace shim that bypasses src/__init__.py (which needs the absent simdyn /
casadi).  The reference never travels to the GPU box -- only the small .npz
outputs written next to this script do.  Run:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
"""
from __future__ import annotations

import importlib
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src"
sys.path.insert(0, REPO)

from gp_mpc_rocket_landing_amd.data import (synthetic_training_data,  # noqa: E402
                                            synthetic_6dof_training_data, query_points)


def shim(name, sub):
    pkg = types.ModuleType(name)
    pkg.__path__ = [os.path.join(REF, sub)]
    sys.modules[name] = pkg


shim("refgp", "gp")
shim("refmpc", "mpc")
shim("refexp", "experiments")
kernels = importlib.import_module("refgp.kernels")
exact_gp = importlib.import_module("refgp.exact_gp")
sparse_gp = importlib.import_module("refgp.sparse_gp")
features = importlib.import_module("refgp.features")
structured_gp = importlib.import_module("refgp.structured_gp")
osqp_rti = importlib.import_module("refmpc.osqp_rti")
uncertainty_prop = importlib.import_module("refmpc.uncertainty_prop")
monte_carlo = importlib.import_module("refexp.monte_carlo")


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrs)
    print("wrote", path, os.path.getsize(path), "bytes")


# ---------------------------------------------------------------- F1
def f1():
    X, U, D = synthetic_training_data(1000, seed=0)
    gp = structured_gp.Simple3DoFGP(use_sparse=False)
    gp.add_data(X, U, D)
    gp.fit()
    Z = gp.feature_extractor.extract_batch(X, U)
    Xq, Uq = query_points(X, U, 20, seed=7)
    Xq = Xq + np.random.RandomState(11).normal(0, 0.05, Xq.shape)
    Zq = gp.feature_extractor.extract_batch(Xq, Uq)
    mq, vq = gp.gp.predict(Zq)
    m1, v1 = gp.predict(Xq[0], Uq[0])
    gps = gp.gp.gps
    save("f1_exact_simple3dof.npz", X=X, U=U, D=D, Z=Z, Xq=Xq, Uq=Uq, Zq=Zq, mean=mq, var=vq,
         single_mean=m1, single_var=v1,
         y_mean=np.array([g._y_mean for g in gps]), y_std=np.array([g._y_std for g in gps]),
         alpha=np.stack([g._alpha for g in gps], axis=1),
         diagL=np.diag(gps[0]._L).copy(), lml=np.array([g.log_marginal_likelihood for g in gps]))


# ---------------------------------------------------------------- F2
def f2():
    rs = np.random.RandomState(5)
    X = rs.normal(0, 1, (64, 11))
    Y = np.stack([np.sin(X[:, 0]) + 0.1 * X[:, 1], np.cos(X[:, 2]), X[:, 3] ** 2], axis=1)
    g = exact_gp.MultiOutputExactGP(11, 3, noise_variance=1e-3)
    g.fit(X, Y)
    Xq = rs.normal(0, 1, (7, 11))
    mq, vq = g.predict(Xq)
    mu_c, cov_c = g.gps[1].predict(Xq, return_cov=True)
    K = g.gps[0].kernel(X)
    # singular: duplicated rows with a slightly negative noise (set on the private
    # field, the setter asserts > 0) -> plain Cholesky fails, the jitter ladder recovers
    Xd = np.concatenate([X[:32], X[:32]], axis=0)
    gd = exact_gp.ExactGP(kernels.SquaredExponentialARD(11), noise_variance=1e-3)
    gd._noise_variance = -1e-7
    gd.fit(Xd, Y[:, 0])
    Kd = gd.kernel(Xd) + (-1e-7) * np.eye(64)
    jit_used = -1.0
    try:
        np.linalg.cholesky(Kd)
        jit_used = 0.0
    except np.linalg.LinAlgError:
        j = 1e-6
        while j < 1.0:
            try:
                Lj = np.linalg.cholesky(Kd + j * np.eye(64))
                if np.array_equal(Lj, gd._L):
                    jit_used = j
                    break
            except np.linalg.LinAlgError:
                pass
            j *= 10
    md, vd = gd.predict(Xq).mean, gd.predict(Xq).variance
    # exhausted ladder -> ValueError
    ge = exact_gp.ExactGP(kernels.SquaredExponentialARD(11), noise_variance=1e-3)
    raised = 0
    try:
        ge.noise_variance = 1e-3
        ge._noise_variance = -5.0   # K - 5 I is indefinite for every jitter < 1
        ge.fit(X, Y[:, 0])
    except ValueError as e:
        raised = int("not positive definite" in str(e))
    save("f2_exact_small.npz", X=X, Y=Y, Xq=Xq, K=K, L=g.gps[0]._L,
         alpha=np.stack([gg._alpha for gg in g.gps], axis=1), mean=mq, var=vq,
         cov_mean=mu_c, cov=cov_c, lml=np.array([gg.log_marginal_likelihood for gg in g.gps]),
         Xdup=Xd, ydup=Y[:, 0], dup_mean=md, dup_var=vd, dup_jitter=jit_used, dup_L=gd._L,
         neg_noise_raises=raised)


# ---------------------------------------------------------------- F3
def f3():
    rs = np.random.RandomState(9)
    X1 = rs.normal(0, 1, (32, 11)); X2 = rs.normal(0, 1, (48, 11))
    ls = rs.uniform(0.5, 2.0, 11); s2 = 0.7
    out = dict(X1=X1, X2=X2, ls=ls, sigma2=s2)
    out["se_ard"] = kernels.SquaredExponentialARD(11, s2, ls)(X1, X2)
    out["se_ard_self"] = kernels.SquaredExponentialARD(11, s2, ls)(X1)
    out["matern32"] = kernels.Matern32(11, s2, ls)(X1, X2)
    out["matern52"] = kernels.Matern52(11, s2, ls)(X1, X2)
    out["se_iso"] = kernels.SquaredExponential(s2, 1.3)(X1, X2)
    out["iso_l"] = 1.3
    out["matern52_diag"] = kernels.Matern52(11, s2, ls).diagonal(X1)
    # composite kernels (kernels.py:676-782)
    k = kernels.SquaredExponentialARD(11, s2, ls) + kernels.Matern32(11, 0.3, ls)
    out["sum_se_m32"] = k(X1, X2)
    k = kernels.SquaredExponentialARD(11, s2, ls) * kernels.Matern52(11, 0.5, ls)
    out["prod_se_m52"] = k(X1, X2)
    save("f3_kernels.npz", **out)


# ---------------------------------------------------------------- F11
def f11():
    """Kernel hyperparameter gradients (kernels.py:279-318, 438-456, 551-558,
    644-650, 697-707, 750-763, WhiteNoise), same inputs as F3."""
    rs = np.random.RandomState(9)
    X1 = rs.normal(0, 1, (32, 11)); X2 = rs.normal(0, 1, (48, 11))
    ls = rs.uniform(0.5, 2.0, 11); s2 = 0.7
    X1, X2 = X1[:16], X2[:24]
    out = dict(X1=X1, X2=X2, ls=ls, sigma2=s2, iso_l=1.3)
    cases = {
        "se_ard": kernels.SquaredExponentialARD(11, s2, ls),
        "se_iso": kernels.SquaredExponential(s2, 1.3),
        "matern32": kernels.Matern32(11, s2, ls),
        "matern52": kernels.Matern52(11, s2, ls),
        "white": kernels.WhiteNoise(0.05),
        "sum_se_m32": kernels.SquaredExponentialARD(11, s2, ls) + kernels.Matern32(11, 0.3, ls),
        "prod_se_m52": kernels.SquaredExponentialARD(11, s2, ls) * kernels.Matern52(11, 0.5, ls),
    }
    for name, k in cases.items():
        for tag, args in (("x12", (X1, X2)),) + ((("x11", (X1,)),) if name == "se_ard" else ()):
            g = k.gradients(*args)
            out[f"{name}_{tag}_names"] = np.array(list(g.keys()))
            for j, v in enumerate(g.values()):
                out[f"{name}_{tag}_{j}"] = v
    save("f11_kernel_gradients.npz", **out)


# ---------------------------------------------------------------- F4
def f4():
    X, U, D = synthetic_training_data(1000, seed=0)
    np.random.seed(1234)
    gp = structured_gp.Simple3DoFGP(n_inducing=50, use_sparse=True)
    gp.add_data(X, U, D)
    gp.fit()
    gps = gp.gp.gps
    Xq, Uq = query_points(X, U, 20, seed=7)
    Zq = gp.feature_extractor.extract_batch(Xq, Uq)
    mq, vq = gp.gp.predict(Zq)
    save("f4_fitc_simple3dof.npz", X=X, U=U, D=D, Zi=gps[0]._Z, Zq=Zq, mean=mq, var=vq,
         lam=gps[0]._Lambda_diag, alpha=np.stack([g._alpha for g in gps], axis=1),
         diagLuu=np.diag(gps[0]._L_uu).copy(), diagLB=np.stack([np.diag(g._L_B) for g in gps], 1),
         y_mean=np.array([g._y_mean for g in gps]), y_std=np.array([g._y_std for g in gps]),
         lml=np.array([g.log_marginal_likelihood for g in gps]))


# ---------------------------------------------------------------- F5
def f5():
    X, U, Dv, Dw = synthetic_6dof_training_data(300, seed=2)
    out = dict(X=X, U=U, Dv=Dv, Dw=Dw)
    fe = features.CombinedFeatureExtractor()
    out["Zv"] = fe.extract_batch_translational(X, U)
    out["Zw"] = fe.extract_batch_rotational(X, U)
    Xq = X[:12] + np.random.RandomState(3).normal(0, 0.02, (12, 14)); Uq = U[:12]
    out["Xq"] = Xq; out["Uq"] = Uq
    for tag, sparse in (("exact", False), ("fitc", True)):
        np.random.seed(77)
        cfg = structured_gp.StructuredGPConfig(n_inducing=50, use_sparse=sparse)
        g = structured_gp.StructuredRocketGP(cfg)
        g.add_data(X, U, Dv, Dw)
        g.fit()
        r = g.predict_batch(Xq, Uq)
        for i, nm in enumerate(("dv_mean", "dw_mean", "dv_var", "dw_var")):
            out[f"{tag}_{nm}"] = r[i]
        one = g.predict(Xq[0], Uq[0])
        out[f"{tag}_single"] = np.stack(one)
        if sparse:
            out["fitc_Zv"] = g.gp_v.gps[0]._Z
            out["fitc_Zw"] = g.gp_omega.gps[0]._Z
    save("f5_structured_6dof.npz", **out)


# ---------------------------------------------------------------- F6
class _Params:
    g0 = 1.0
    alpha = 1.0 / 30.0
    g_vec = np.array([-1.0, 0.0, 0.0])


class _Plant:
    """Euler 3-DoF restatement (nominal_mpc.py:585-605); simdyn is absent."""
    params = _Params()

    def step(self, x, u, dt):
        x = np.asarray(x, float); u = np.asarray(u, float)
        out = np.empty(7)
        out[0] = x[0] - dt * self.params.alpha * np.sqrt(u @ u)
        out[1:4] = x[1:4] + dt * x[4:7]
        out[4:7] = x[4:7] + dt * (u / x[0] + self.params.g_vec)
        return out


def f6():
    osqp_rti.HAS_OSQP = True
    cfg = osqp_rti.OSQPRTIConfig(N=20, dt=0.1)
    mpc = osqp_rti.FastRTI3DoF(_Plant(), cfg)
    rs = np.random.RandomState(21)
    out = {}
    cases = []
    x0 = np.array([2.0, 30.0, 1.0, -1.0, -3.0, 0.2, 0.1])
    xt = np.zeros(7); xt[0] = 2.0
    cases.append((x0, xt, None, None))
    # pattern-change case (D3): lateral thrust makes T_y, T_z != 0
    U = np.tile([2.0, 0.4, -0.3], (20, 1))
    cases.append((x0, xt, None, U))
    for _ in range(2):
        x0r = x0 + rs.normal(0, 1, 7) * [0.1, 5, 2, 2, 0.5, 0.3, 0.3]
        Xr = np.linspace(x0r, xt, 21) + rs.normal(0, 0.1, (21, 7))
        Ur = np.stack([rs.uniform(0.5, 4.5, 20), rs.normal(0, 0.5, 20), rs.normal(0, 0.5, 20)], 1)
        cases.append((x0r, xt, Xr, Ur))
    for i, (x0c, xtc, Xi, Ui) in enumerate(cases):
        mpc._x_ref = np.tile(xtc, (cfg.N + 1, 1))
        mpc._u_ref = np.zeros((cfg.N, 3)); mpc._u_ref[:, 0] = x0c[0] * 1.0
        Xl = Xi if Xi is not None else np.array([(1 - k / 20) * x0c + (k / 20) * xtc for k in range(21)])
        Ul = Ui if Ui is not None else mpc._u_ref.copy()
        P, q = mpc._build_cost_matrix()
        A, l, u = mpc._build_constraint_matrix(Xl, Ul, x0c)
        Ak, Bk = mpc._linearize(Xl[0], Ul[0])
        out.update({f"c{i}_x0": x0c, f"c{i}_xt": xtc, f"c{i}_X": Xl, f"c{i}_U": Ul,
                    f"c{i}_P_data": P.data, f"c{i}_P_indices": P.indices, f"c{i}_P_indptr": P.indptr,
                    f"c{i}_q": q, f"c{i}_A_data": A.data, f"c{i}_A_indices": A.indices,
                    f"c{i}_A_indptr": A.indptr, f"c{i}_l": l, f"c{i}_u": u, f"c{i}_A0": Ak,
                    f"c{i}_B0": Bk, f"c{i}_zvec": mpc._solution_to_vector(Xl, Ul)})
    out["ncases"] = len(cases)
    save("f6_qp_assembly.npz", **out)


# ---------------------------------------------------------------- F6b
def f6b():
    """The caller's-plant hooks of the RTI QP: reference OSQPRTIMPC (forward-
    difference Jacobians through dynamics.step, osqp_rti.py:374-401) and
    FastRTI3DoF (analytic Jacobians, c_k from dynamics.step, :339) driven by a
    plant with drag (toy_dynamics.DragRocket3DoF)."""
    from toy_dynamics import DragRocket3DoF
    osqp_rti.HAS_OSQP = True
    rs = np.random.RandomState(23)
    out = {}
    for name, cls in (("fd", osqp_rti.OSQPRTIMPC), ("fast", osqp_rti.FastRTI3DoF)):
        cfg = osqp_rti.OSQPRTIConfig(N=20, dt=0.1)
        mpc = cls(DragRocket3DoF(), cfg)
        for i in range(2):
            x0 = np.array([2.0, 30.0, 1.0, -1.0, -3.0, 0.2, 0.1]) + rs.normal(0, 1, 7) * [0.1, 5, 2, 2, 0.5, 0.3, 0.3]
            xt = np.zeros(7); xt[0] = x0[0]
            X = np.linspace(x0, xt, 21) + rs.normal(0, 0.1, (21, 7))
            U = np.stack([rs.uniform(0.5, 4.5, 20), rs.normal(0, 0.5, 20), rs.normal(0, 0.5, 20)], 1)
            A, l, u = mpc._build_constraint_matrix(X, U, x0)
            Ak, Bk = mpc._linearize(X[3], U[3])
            out.update({f"{name}{i}_x0": x0, f"{name}{i}_X": X, f"{name}{i}_U": U,
                        f"{name}{i}_A_data": A.data, f"{name}{i}_A_indices": A.indices,
                        f"{name}{i}_A_indptr": A.indptr, f"{name}{i}_l": l, f"{name}{i}_u": u,
                        f"{name}{i}_A3": Ak, f"{name}{i}_B3": Bk})
    save("f6b_rti_plant_hooks.npz", **out)


# ---------------------------------------------------------------- F7 / F8
def f7_f8():
    cfg = monte_carlo.SimulationConfig(
        dt=0.1, max_time=30.0, altitude_mean=30.0, altitude_std=5.0, horizontal_std=3.0,
        velocity_mean=np.array([-3, 0, 0]), velocity_std=np.array([1, 0.5, 0.5]),
        landing_constraints=monte_carlo.LandingConstraints(pos_tol_xy=5.0, vel_tol_z=3.0))
    sim = monte_carlo.MonteCarloSimulator(_Plant(), controller=None, config=cfg)
    x0s = np.array([sim.sample_initial_condition(42 + i) for i in range(1024)])
    sim_d = monte_carlo.MonteCarloSimulator(_Plant(), controller=None)
    x0d = np.array([sim_d.sample_initial_condition(42 + i) for i in range(16)])
    save("f7_mc_initial_conditions.npz", x0_run_experiments=x0s, x0_default=x0d,
         seeds=np.arange(42, 42 + 1024))
    rs = np.random.RandomState(8)
    states = []
    for _ in range(200):
        s = np.array([rs.uniform(0.9, 2.1), rs.uniform(-0.5, 2.0), rs.normal(0, 4), rs.normal(0, 4),
                      rs.normal(0, 2.5), rs.normal(0, 1.2), rs.normal(0, 1.2)])
        states.append(s)
    states = np.array(states)
    m0 = rs.uniform(1.5, 2.5, len(states))
    ok, reason = [], []
    for lc_name, lc in (("default", monte_carlo.LandingConstraints()), ("run_exp", cfg.landing_constraints)):
        r = [lc.check_landing(s, m) for s, m in zip(states, m0)]
        ok.append([int(a) for a, _ in r])
        reason.append([b.split(":")[0] for _, b in r])
    save("f8_check_landing.npz", states=states, m0=m0, ok=np.array(ok), reason=np.array(reason))


# ---------------------------------------------------------------- F9
def f9():
    """Reference UncertaintyPropagator (linear / unscented / Monte Carlo,
    uncertainty_prop.py:117-315) with the exact 6-DoF StructuredRocketGP on the
    F5 training set and the toy 14-state plant of toy_dynamics.py."""
    sys.path.insert(0, HERE)
    from toy_dynamics import ToyRocket14, toy_case
    f5 = np.load(os.path.join(HERE, "f5_structured_6dof.npz"))
    g = structured_gp.StructuredRocketGP(structured_gp.StructuredGPConfig(use_sparse=False))
    g.add_data(f5["X"], f5["U"], f5["Dv"], f5["Dw"])
    g.fit()
    dyn = ToyRocket14()
    x0, U = toy_case()
    out = dict(x0=x0, U=U)
    S0 = np.diag(np.linspace(1e-6, 1e-4, 14))
    for method in ("linear", "unscented", "monte_carlo"):
        np.random.seed(123)
        p = uncertainty_prop.UncertaintyPropagator(dyn, g, method=method)
        r = p.propagate(x0, U, Sigma_0=None if method != "unscented" else S0, dt=0.1)
        out[f"{method}_means"] = r.means
        out[f"{method}_covs"] = r.covariances
    out["S0_unscented"] = S0
    save("f9_uncertainty_prop.npz", **out)


# ---------------------------------------------------------------- F10
def f10():
    """Reference ExactGP (SE-ARD, D = 11 3-DoF features) log marginal likelihood
    at a grid of hyperparameter vectors (exact_gp.py:118-204 via the objective
    of :375-386), one vector whose K needs the jitter ladder (duplicated rows,
    noise 1e-14), and ExactGP.optimize_hyperparameters (:357-421, L-BFGS-B with
    scipy's finite differences, 2 restarts under np.random.seed(5))."""
    X, U, D = synthetic_training_data(120, seed=3)
    Z = features.Simple3DoFFeatureExtractor().extract_batch(X, U)
    y = D[:, 0].copy()
    rs = np.random.RandomState(11)
    p0 = np.concatenate([np.zeros(12), [np.log(1e-4)]])   # [log s2, log l (11), log noise]
    grid = p0 + 0.4 * rs.normal(size=(15, 13))
    grid = np.vstack([p0, grid])
    lml = []
    for p in grid:
        gp = exact_gp.ExactGP(kernels.SquaredExponentialARD(11), noise_variance=np.exp(p[-1]))
        gp.kernel.set_params(p[:-1])
        gp.fit(Z, y)
        lml.append(gp.log_marginal_likelihood)
    # jitter ladder: duplicated rows make K singular, a negative "noise" of -2e-3
    # makes K + s_n^2 I clearly indefinite; jitters 1e-6 .. 1e-3 still fail and
    # 1e-2 succeeds with margins far above rounding (a robust 5-step case)
    Zd = np.vstack([Z[:40], Z[:40]]); yd = np.concatenate([y[:40], y[:40] + 1e-3])
    gpj = exact_gp.ExactGP(kernels.SquaredExponentialARD(11), noise_variance=-2e-3)
    gpj.fit(Zd, yd)
    gpo = exact_gp.ExactGP(kernels.SquaredExponentialARD(11), noise_variance=1e-4)
    gpo.fit(Z, y)
    lml_init = gpo.log_marginal_likelihood
    np.random.seed(5)
    res = gpo.optimize_hyperparameters(n_restarts=2)
    # refinement from the optimum found: converges (success) in a few iterations
    p_opt, n_opt = gpo.kernel.get_params(), gpo.noise_variance
    gpr = exact_gp.ExactGP(kernels.SquaredExponentialARD(11), noise_variance=n_opt)
    gpr.kernel.set_params(p_opt)
    gpr.fit(Z, y)
    np.random.seed(5)
    rr = gpr.optimize_hyperparameters(n_restarts=1)
    save("f10_hyperparameters.npz", Z=Z, y=y, grid=grid, lml=np.array(lml), Zd=Zd, yd=yd,
         ref_start_params=p_opt, ref_start_noise=n_opt, ref_params=gpr.kernel.get_params(),
         ref_noise=gpr.noise_variance, ref_lml=rr["log_marginal_likelihood"],
         ref_nit=rr["n_iterations"], ref_success=rr["success"],
         lml_jitter=gpj.log_marginal_likelihood, L_jitter_diag=np.diag(gpj._L),
         lml_init=lml_init, opt_params=gpo.kernel.get_params(), opt_noise=gpo.noise_variance,
         opt_lml=res["log_marginal_likelihood"], opt_nit=res["n_iterations"],
         opt_success=res["success"])


# ---------------------------------------------------------------- F12
def f12():
    """Reference SparseGP(method="vfe") (sparse_gp.py:150-188, 221-249; predict
    :255-305) on the 3-DoF features, two outputs over caller-set inducing points
    (a random subset, so no kmeans2 draw is involved), non-unit hyperparameters."""
    X, U, D = synthetic_training_data(600, seed=5)
    fe = features.Simple3DoFFeatureExtractor()
    Z = fe.extract_batch(X, U)
    rs = np.random.RandomState(12)
    Zi = Z[rs.choice(Z.shape[0], 40, replace=False)].copy()
    sd = Z.std(0)
    sd[sd < 1e-6] = 1.0
    ls = 3.0 * sd * (0.8 + 0.4 * rs.rand(Z.shape[1]))  # well-conditioned B (cond ~1e5)
    Xq, Uq = query_points(X, U, 25, seed=13)
    Zq = fe.extract_batch(Xq, Uq)
    out = dict(Z=Z, Y=D[:, :2], Zi=Zi, ls=ls, Zq=Zq, sigma2=np.array(1.7), noise=np.array(5e-2),
               jitter=np.array(1e-6))
    for c in range(2):
        k = kernels.SquaredExponentialARD(Z.shape[1], signal_variance=1.7, lengthscales=ls.copy())
        g = sparse_gp.SparseGP(k, n_inducing=40, noise_variance=5e-2, method="vfe",
                               inducing_points=Zi.copy())
        g.fit(Z, D[:, c])
        pr = g.predict(Zq)
        out[f"mean{c}"] = pr.mean; out[f"var{c}"] = pr.variance
        out[f"alpha{c}"] = g._alpha; out[f"lml{c}"] = np.array(g.log_marginal_likelihood)
        out[f"diagLB{c}"] = np.diag(g._L_B).copy()
    save("f12_vfe_3dof.npz", **out)


# ---------------------------------------------------------------- F13
def f13():
    """Composite kernels in fitted GPs (kernels.py:676-844 through exact_gp.py:157,
    237-266 and sparse_gp.py:182-183, 193-199, 277-301): the reference's own ExactGP
    with SumKernel(SE-ARD, WhiteNoise), ProductKernel(SE-ARD, Matern52) and
    SumKernel(ProductKernel(SE iso, Matern32), WhiteNoise), and its FITC and VFE
    SparseGP with SumKernel(Matern52, WhiteNoise) -- fit (alpha, LML, diag L) and
    predict (mean, variance; return_cov for the first) on the 3-DoF features."""
    X, U, D = synthetic_training_data(300, seed=21)
    fe = features.Simple3DoFFeatureExtractor()
    Z = fe.extract_batch(X, U)
    d = Z.shape[1]
    rs = np.random.RandomState(13)
    sd = Z.std(0)
    sd[sd < 1e-6] = 1.0
    ls1 = 2.0 * sd * (0.8 + 0.4 * rs.rand(d))
    ls2 = 3.0 * sd * (0.8 + 0.4 * rs.rand(d))
    Xq, Uq = query_points(X, U, 17, seed=14)
    Zq = fe.extract_batch(Xq, Uq)
    out = dict(Z=Z, Y=D, Zq=Zq, ls1=ls1, ls2=ls2)

    def k_sum_white():
        return kernels.SumKernel(kernels.SquaredExponentialARD(d, 1.3, ls1.copy()), kernels.WhiteNoise(2e-3))

    def k_prod():
        return kernels.ProductKernel(kernels.SquaredExponentialARD(d, 1.1, ls1.copy()),
                                     kernels.Matern52(d, 0.9, ls2.copy()))

    def k_nested():
        return kernels.SumKernel(kernels.ProductKernel(kernels.SquaredExponential(1.2, 2.5),
                                                       kernels.Matern32(d, 0.8, ls2.copy())),
                                 kernels.WhiteNoise(5e-3))

    for name, make in (("sumwhite", k_sum_white), ("prod", k_prod), ("nested", k_nested)):
        for c in range(2):
            g = exact_gp.ExactGP(make(), noise_variance=1e-3)
            g.fit(Z, D[:, c])
            pr = g.predict(Zq)
            out[f"{name}_mean{c}"] = pr.mean; out[f"{name}_var{c}"] = pr.variance
            out[f"{name}_alpha{c}"] = g._alpha; out[f"{name}_lml{c}"] = np.array(g.log_marginal_likelihood)
            out[f"{name}_diagL{c}"] = np.diag(g._L).copy()
            if name == "sumwhite" and c == 0:
                m, cov = g.predict(Zq, return_cov=True)
                out["sumwhite_covmean0"] = m; out["sumwhite_cov0"] = cov
    Zi = Z[rs.choice(Z.shape[0], 40, replace=False)].copy()
    out["Zi"] = Zi
    for method in ("fitc", "vfe"):
        for c in range(2):
            k = kernels.SumKernel(kernels.Matern52(d, 1.4, ls2.copy()), kernels.WhiteNoise(1e-3))
            g = sparse_gp.SparseGP(k, n_inducing=40, noise_variance=2e-2, method=method, inducing_points=Zi.copy())
            g.fit(Z, D[:, c])
            pr = g.predict(Zq)
            out[f"{method}_mean{c}"] = pr.mean; out[f"{method}_var{c}"] = pr.variance
            out[f"{method}_alpha{c}"] = g._alpha; out[f"{method}_lml{c}"] = np.array(g.log_marginal_likelihood)
    save("f13_composite_kernels.npz", **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["f1", "f2", "f3", "f4", "f5", "f6", "f6b", "f7_f8", "f9", "f10", "f11", "f12",
                             "f13"]
    for w in which:
        globals()[w]()
