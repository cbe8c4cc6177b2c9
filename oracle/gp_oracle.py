"""numpy restatement of the reference GP hot path (TEST INFRASTRUCTURE ONLY).

Every function cites the reference file:line it restates.  The restatement is
functional (plain arrays in, plain arrays out) so that tests can compare the
HIP product path against it on identical inputs.  It is pinned against golden
vectors produced by the reference itself (tests/golden/gen_golden.py).
"""
from __future__ import annotations

import numpy as np
from scipy.linalg import cho_solve, solve_triangular

RHO0 = 1.225          # features.py:55  AtmosphereModel.rho_0
SCALE_HEIGHT = 8500.  # features.py:56  AtmosphereModel.scale_height
V_REF = 10.0          # features.py:85  reference_velocity default


# --------------------------------------------------------------------------
# kernels (src/gp/kernels.py)
# --------------------------------------------------------------------------
def scaled_sqdist(X1, X2, ls):
    """kernels.py:205-236 -- expansion form ||a||^2 + ||b||^2 - 2 a.b, clamped at 0."""
    a = X1 / ls
    b = a if X2 is None else X2 / ls
    na = np.sum(a ** 2, axis=1, keepdims=True)
    nb = np.sum(b ** 2, axis=1, keepdims=True)
    d = na + nb.T - 2 * a @ b.T
    return np.maximum(d, 0.0)


def composite_diag(spec):
    """k(x, x) of a composite spec (kernels.py diagonal methods, :694-695, :747-748,
    :817-819): every leaf's diagonal is its sigma2, so the composite's is a constant."""
    if spec[0] == "sum":
        return composite_diag(spec[1]) + composite_diag(spec[2])
    if spec[0] == "prod":
        return composite_diag(spec[1]) * composite_diag(spec[2])
    return float(spec[1])


def gram(kind, X1, X2, sigma2, ls):
    """K(X1, X2) for kind in {se_ard, se_iso, matern32, matern52}, or a composite
    spec (kernels.py:676-844): ("sum", a, b), ("prod", a, b), ("white", s2) or a
    leaf (kind, sigma2, ls); sigma2 / ls are then ignored.  WhiteNoise is s2 I on a
    Gram of one set (X2 None) and zero across sets (kernels.py:805-815).

    se_ard   kernels.py:238-262   sigma2*exp(-0.5 r^2)
    se_iso   kernels.py:417-432   sigma2*exp(-r^2/(2 l^2)), distance on raw inputs
    matern32 kernels.py:516-545   sigma2*(1+sqrt3 r) exp(-sqrt3 r)
    matern52 kernels.py:610-637   sigma2*(1+sqrt5 r+5r^2/3) exp(-sqrt5 r)
    """
    X1 = np.atleast_2d(X1)
    X2 = None if X2 is None else np.atleast_2d(X2)
    if isinstance(kind, tuple):
        if kind[0] == "sum":
            return gram(kind[1], X1, X2, None, None) + gram(kind[2], X1, X2, None, None)
        if kind[0] == "prod":
            return gram(kind[1], X1, X2, None, None) * gram(kind[2], X1, X2, None, None)
        if kind[0] == "white":
            return kind[1] * np.eye(X1.shape[0]) if X2 is None else np.zeros((X1.shape[0], X2.shape[0]))
        return gram(kind[0], X1, X2, kind[1], kind[2])
    if kind == "se_ard":
        return sigma2 * np.exp(-0.5 * scaled_sqdist(X1, X2, np.asarray(ls, float)))
    if kind == "se_iso":
        l = float(np.asarray(ls).ravel()[0])
        d = scaled_sqdist(X1, X2, 1.0)
        return sigma2 * np.exp(-d / (2 * l ** 2))
    r = np.sqrt(scaled_sqdist(X1, X2, np.asarray(ls, float)))
    if kind == "matern32":
        s = np.sqrt(3) * r
        return sigma2 * (1 + s) * np.exp(-s)
    if kind == "matern52":
        s = np.sqrt(5) * r
        return sigma2 * (1 + s + 5 * r ** 2 / 3) * np.exp(-s)
    raise ValueError(kind)


def gram_gradients(kind, X1, X2, sigma2, ls):
    """Hyperparameter gradients d K / d log(theta) as ordered lists.

    se_ard   kernels.py:279-318   [K, K (x1_i - x2_i)^2 / l_i^2 for each i]
    se_iso   kernels.py:438-456   [K, K r^2 / l^2]  (r^2 on raw inputs, clamped)
    matern*  kernels.py:551-558, 644-650   [K]
    """
    X1 = np.atleast_2d(X1)
    X2 = X1 if X2 is None else np.atleast_2d(X2)
    K = gram(kind, X1, X2, sigma2, ls)
    if kind == "se_ard":
        ls = np.asarray(ls, float)
        return [K] + [K * ((X1[:, i:i + 1] - X2[:, i:i + 1].T) ** 2 / ls[i] ** 2) for i in range(X1.shape[1])]
    if kind == "se_iso":
        l = float(np.asarray(ls).ravel()[0])
        return [K, K * scaled_sqdist(X1, X2, 1.0) / l ** 2]
    return [K]


# --------------------------------------------------------------------------
# features (src/gp/features.py)
# --------------------------------------------------------------------------
def density(alt):
    """features.py:57-63 -- rho0*exp(-h/H)."""
    return RHO0 * np.exp(-alt / SCALE_HEIGHT)


def features_3dof(X, U):
    """Simple3DoFFeatureExtractor.extract (features.py:403-444), batched.

    z = [v/10 (3), |v|/10, q_dyn/(0.5 rho0 100), u/10 (3), |u|/10, alt/100, rho/rho0]
    """
    X = np.atleast_2d(X); U = np.atleast_2d(U)
    v = X[:, 4:7]; alt = X[:, 1]
    speed = np.sqrt(np.sum(v * v, axis=1))
    rho = density(alt)
    qd = 0.5 * rho * speed ** 2
    tm = np.sqrt(np.sum(U * U, axis=1))
    cols = [v[:, 0] / V_REF, v[:, 1] / V_REF, v[:, 2] / V_REF, speed / V_REF,
            qd / (0.5 * RHO0 * V_REF ** 2), U[:, 0] / 10.0, U[:, 1] / 10.0, U[:, 2] / 10.0,
            tm / 10.0, alt / 100.0, rho / RHO0]
    return np.stack(cols, axis=1)


def _dcm(q):
    """features.py:265-270 -- body-from-inertial DCM of quaternion [w,x,y,z]."""
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    C = np.empty((q.shape[0], 3, 3))
    C[:, 0, 0] = 1 - 2 * (y ** 2 + z ** 2); C[:, 0, 1] = 2 * (x * y + w * z); C[:, 0, 2] = 2 * (x * z - w * y)
    C[:, 1, 0] = 2 * (x * y - w * z); C[:, 1, 1] = 1 - 2 * (x ** 2 + z ** 2); C[:, 1, 2] = 2 * (y * z + w * x)
    C[:, 2, 0] = 2 * (x * z + w * y); C[:, 2, 1] = 2 * (y * z - w * x); C[:, 2, 2] = 1 - 2 * (x ** 2 + y ** 2)
    return C


def features_translational(X, U):
    """TranslationalFeatureExtractor.extract (features.py:196-263): 13 features."""
    X = np.atleast_2d(X); U = np.atleast_2d(U)
    alt = X[:, 1]; v = X[:, 4:7]
    speed = np.sqrt(np.sum(v * v, axis=1))
    rho = density(alt); qd = 0.5 * rho * speed ** 2
    vB = np.einsum("nij,nj->ni", _dcm(X[:, 7:11]), v)
    moving = speed > 1e-3
    safe = np.where(moving, speed, 1.0)
    aoa = np.where(moving, np.arctan2(-vB[:, 2], vB[:, 0]), 0.0)
    beta = np.where(moving, np.arcsin(np.clip(vB[:, 1] / safe, -1, 1)), 0.0)
    tm = np.sqrt(np.sum(U * U, axis=1))
    cols = [v[:, 0] / V_REF, v[:, 1] / V_REF, v[:, 2] / V_REF, speed / V_REF,
            qd / (0.5 * RHO0 * V_REF ** 2), aoa, beta, U[:, 0] / 10.0, U[:, 1] / 10.0,
            U[:, 2] / 10.0, tm / 10.0, alt / 100.0, rho / RHO0]
    return np.stack(cols, axis=1)


def features_rotational(X, U):
    """RotationalFeatureExtractor.extract (features.py:304-356): 12 features."""
    X = np.atleast_2d(X); U = np.atleast_2d(U)
    alt = X[:, 1]; v = X[:, 4:7]; w = X[:, 11:14]
    speed = np.sqrt(np.sum(v * v, axis=1)); wm = np.sqrt(np.sum(w * w, axis=1))
    rho = density(alt); qd = 0.5 * rho * speed ** 2
    vB = np.einsum("nij,nj->ni", _dcm(X[:, 7:11]), v)
    cols = [w[:, 0], w[:, 1], w[:, 2], wm, U[:, 0] / 10.0, U[:, 1] / 10.0, U[:, 2] / 10.0,
            vB[:, 0] / V_REF, vB[:, 1] / V_REF, vB[:, 2] / V_REF, speed / V_REF,
            qd / (0.5 * RHO0 * V_REF ** 2)]
    return np.stack(cols, axis=1)


# --------------------------------------------------------------------------
# exact GP (src/gp/exact_gp.py)
# --------------------------------------------------------------------------
def normalise(y):
    """exact_gp.py:141-150 -- population std; std < 1e-10 -> 1."""
    m = np.mean(y); s = np.std(y)
    if s < 1e-10:
        s = 1.0
    return (y - m) / s, m, s


def jitter_ladder():
    """exact_gp.py:167-173 -- 1e-6 then repeated *=10 while < 1 (fp64 values kept)."""
    out = []; j = 1e-6
    while j < 1.0:
        out.append(j); j *= 10
    return out


def chol_with_jitter(Kn):
    """exact_gp.py:163-175 -- plain Cholesky, then the jitter ladder, then ValueError.

    Returns (L, jitter_steps) where jitter_steps = 0 means no jitter was needed."""
    n = Kn.shape[0]
    try:
        return np.linalg.cholesky(Kn), 0
    except np.linalg.LinAlgError:
        for i, j in enumerate(jitter_ladder()):
            try:
                return np.linalg.cholesky(Kn + j * np.eye(n)), i + 1
            except np.linalg.LinAlgError:
                pass
    raise ValueError("Kernel matrix is not positive definite even with jitter")


def exact_fit(Z, Y, kind="se_ard", sigma2=1.0, ls=None, noise=1e-4):
    """ExactGP.fit for every column of Y (exact_gp.py:118-184, 186-204; MultiOutput 476-499).

    The three outputs of MultiOutputExactGP share one kernel and one X, so K and
    L are identical across outputs; alpha / y_mean / y_std / lml differ.
    """
    Z = np.atleast_2d(Z); Y = np.asarray(Y, float)
    if Y.ndim == 1:
        Y = Y[:, None]
    n = Z.shape[0]
    if ls is None:
        ls = np.ones(Z.shape[1])
    if isinstance(kind, tuple):   # composite: the prior variance is its diagonal constant
        sigma2 = composite_diag(kind)
    K = gram(kind, Z, None, sigma2, ls)
    L, jit = chol_with_jitter(K + noise * np.eye(n))
    out = dict(L=L, jitter_steps=jit, Z=Z, kind=kind, sigma2=sigma2, ls=np.asarray(ls, float),
               noise=noise, alpha=[], y_mean=[], y_std=[], lml=[])
    for c in range(Y.shape[1]):
        yn, m, s = normalise(Y[:, c])
        a = cho_solve((L, True), yn)
        lml = -0.5 * np.dot(yn, a) - np.sum(np.log(np.diag(L))) - 0.5 * n * np.log(2 * np.pi)
        out["alpha"].append(a); out["y_mean"].append(m); out["y_std"].append(s); out["lml"].append(lml)
    out["alpha"] = np.stack(out["alpha"], axis=1)
    out["y_mean"] = np.array(out["y_mean"]); out["y_std"] = np.array(out["y_std"])
    out["lml"] = np.array(out["lml"])
    return out


def exact_predict(st, Zq):
    """ExactGP.predict (exact_gp.py:213-268) for all outputs: (means (P,o), variances (P,o))."""
    Zq = np.atleast_2d(Zq)
    Ks = gram(st["kind"], Zq, st["Z"], st["sigma2"], st["ls"])
    mean = (Ks @ st["alpha"]) * st["y_std"] + st["y_mean"]
    v = solve_triangular(st["L"], Ks.T, lower=True)
    lat = np.maximum(st["sigma2"] - np.sum(v ** 2, axis=0), 1e-10)
    var = lat[:, None] * st["y_std"] ** 2
    return mean, var


def exact_predict_cov(st, Zq, out=0):
    """ExactGP.predict(return_cov=True) (exact_gp.py:247-254) for one output."""
    Zq = np.atleast_2d(Zq)
    Ks = gram(st["kind"], Zq, st["Z"], st["sigma2"], st["ls"])
    Kss = gram(st["kind"], Zq, None, st["sigma2"], st["ls"])
    mean = (Ks @ st["alpha"][:, out]) * st["y_std"][out] + st["y_mean"][out]
    v = solve_triangular(st["L"], Ks.T, lower=True)
    return mean, (Kss - v.T @ v) * st["y_std"][out] ** 2


# --------------------------------------------------------------------------
# sparse FITC GP (src/gp/sparse_gp.py)
# --------------------------------------------------------------------------
def fitc_fit(Zi, X, Y, sigma2=1.0, ls=None, noise=1e-4, jitter=1e-6, kind="se_ard"):
    """SparseGP.fit, FITC branch (sparse_gp.py:150-219), for every column of Y with a
    shared inducing set Zi (MultiOutputSparseGP.fit sparse_gp.py:430-456).  kind: a
    kernel kind or a composite spec (gram); k_ff_diag = its diagonal constant."""
    X = np.atleast_2d(X); Y = np.asarray(Y, float)
    if Y.ndim == 1:
        Y = Y[:, None]
    if ls is None:
        ls = np.ones(X.shape[1])
    if isinstance(kind, tuple):
        sigma2 = composite_diag(kind)
    M = Zi.shape[0]; N = X.shape[0]
    Kuu = gram(kind, Zi, None, sigma2, ls)
    Kuf = gram(kind, Zi, X, sigma2, ls)
    Luu = np.linalg.cholesky(Kuu + jitter * np.eye(M))
    A = solve_triangular(Luu, Kuf, lower=True)
    lam = np.maximum(np.full(N, sigma2) - np.sum(A ** 2, axis=0) + noise, 1e-10)
    As = A * (1.0 / np.sqrt(lam))
    LB = np.linalg.cholesky(np.eye(M) + As @ As.T)
    st = dict(Zi=Zi, Luu=Luu, LB=LB, lam=lam, sigma2=sigma2, ls=np.asarray(ls, float), kind=kind,
              alpha=[], y_mean=[], y_std=[], lml=[])
    for c in range(Y.shape[1]):
        yn, m, s = normalise(Y[:, c])
        cv = A @ (yn / lam)
        a = cho_solve((LB, True), cv)
        fit = -0.5 * (np.sum(yn ** 2 / lam) - np.dot(cv, cho_solve((LB, True), cv)))
        cplx = -np.sum(np.log(np.diag(LB))) - 0.5 * np.sum(np.log(lam))
        st["alpha"].append(a); st["y_mean"].append(m); st["y_std"].append(s)
        st["lml"].append(fit + cplx - 0.5 * N * np.log(2 * np.pi))
    for k in ("alpha",):
        st[k] = np.stack(st[k], axis=1)
    for k in ("y_mean", "y_std", "lml"):
        st[k] = np.array(st[k])
    return st


def vfe_fit(Zi, X, Y, sigma2=1.0, ls=None, noise=1e-4, jitter=1e-6, kind="se_ard"):
    """SparseGP.fit, VFE branch (sparse_gp.py:221-249 after the shared :181-188), every
    column of Y over one inducing set.  Returns the fitc_fit state layout, so
    fitc_predict evaluates it (the reference's predict has one body for both)."""
    X = np.atleast_2d(X); Y = np.asarray(Y, float)
    if Y.ndim == 1:
        Y = Y[:, None]
    if ls is None:
        ls = np.ones(X.shape[1])
    if isinstance(kind, tuple):
        sigma2 = composite_diag(kind)
    M = Zi.shape[0]; N = X.shape[0]
    Kuu = gram(kind, Zi, None, sigma2, ls)
    Kuf = gram(kind, Zi, X, sigma2, ls)
    Luu = np.linalg.cholesky(Kuu + jitter * np.eye(M))
    A = solve_triangular(Luu, Kuf, lower=True)
    B = Kuu + (1.0 / noise) * Kuf @ Kuf.T + jitter * np.eye(M)
    LB = np.linalg.cholesky(B)
    trace_term = (N * sigma2 - np.sum(A ** 2)) / noise
    st = dict(Zi=Zi, Luu=Luu, LB=LB, lam=None, sigma2=sigma2, ls=np.asarray(ls, float), kind=kind,
              alpha=[], y_mean=[], y_std=[], lml=[])
    for c in range(Y.shape[1]):
        yn, m, s = normalise(Y[:, c])
        cv = Kuf @ yn / noise
        a = cho_solve((LB, True), cv)
        fit = -0.5 / noise * np.dot(yn, yn) + np.dot(cv, a) - 0.5 * np.dot(a, Kuu @ a)
        cplx = -np.sum(np.log(np.diag(LB))) + np.sum(np.log(np.diag(Luu))) - 0.5 * N * np.log(noise)
        st["alpha"].append(a); st["y_mean"].append(m); st["y_std"].append(s)
        st["lml"].append(fit - 0.5 * trace_term + cplx - 0.5 * N * np.log(2 * np.pi))
    st["alpha"] = np.stack(st["alpha"], axis=1)
    for k in ("y_mean", "y_std", "lml"):
        st[k] = np.array(st[k])
    return st


def fitc_predict(st, Xq):
    """SparseGP.predict (sparse_gp.py:255-305); the mean is K*u @ alpha as written (D1)."""
    Xq = np.atleast_2d(Xq)
    Ksu = gram(st.get("kind", "se_ard"), Xq, st["Zi"], st["sigma2"], st["ls"])
    mean = (Ksu @ st["alpha"]) * st["y_std"] + st["y_mean"]
    v = solve_triangular(st["Luu"], Ksu.T, lower=True)
    w = solve_triangular(st["LB"], v, lower=True)
    lat = np.maximum(st["sigma2"] - np.sum(v ** 2, axis=0) + np.sum(w ** 2, axis=0), 1e-10)
    return mean, lat[:, None] * st["y_std"] ** 2


def predict(st, Xq):
    """The predict of whichever GP ``st`` holds: a sparse fit (fitc_fit: "Luu") through
    SparseGP.predict (sparse_gp.py:255-305, mean as written), else ExactGP.predict."""
    return fitc_predict(st, Xq) if "Luu" in st else exact_predict(st, Xq)


# --------------------------------------------------------------------------
# surfaces
# --------------------------------------------------------------------------
def simple3dof_fit_predict_exact(X, U, D, Xq, Uq, noise=1e-4):
    """Simple3DoFGP(use_sparse=False).fit / predict (structured_gp.py:470-493)."""
    st = exact_fit(features_3dof(X, U), D, noise=noise)
    return st, exact_predict(st, features_3dof(Xq, Uq))


# --------------------------------------------------------------------------
# hyperparameter search
# --------------------------------------------------------------------------
def lml_at(Z, y, sigma2, ls, noise, kind="se_ard"):
    """The objective of ExactGP.optimize_hyperparameters (exact_gp.py:375-386):
    a full ExactGP.fit (exact_gp.py:118-204) at one parameter set; returns
    (lml, jitter_steps), (-inf, -1) where the fit raises ValueError."""
    try:
        st = exact_fit(Z, y, kind=kind, sigma2=sigma2, ls=ls, noise=noise)
    except ValueError:
        return -np.inf, -1
    return float(st["lml"][0]), st["jitter_steps"]


def optimize_hyperparameters(Z, y, params0, noise0, n_restarts=5, kind="se_ard"):
    """ExactGP.optimize_hyperparameters (exact_gp.py:357-421) for SE-ARD:
    params = [log sigma2, log l_0..l_{D-1}] (kernels.py:320-371 order) + log
    noise; L-BFGS-B (maxiter 100) with scipy's own finite-difference gradient;
    restarts perturb with 0.5 * np.random.randn (global RNG, as the reference).
    Returns (result dict, best params (kernel), best noise)."""
    from scipy.optimize import minimize
    y = np.asarray(y, float).reshape(-1)

    def objective(p):
        lml, _ = lml_at(Z, y, float(np.exp(p[0])), np.exp(p[1:-1]), float(np.exp(p[-1])), kind)
        return -lml

    initial = np.concatenate([np.asarray(params0, float), [np.log(noise0)]])
    best, best_nll = None, np.inf
    for r in range(n_restarts):
        p0 = initial if r == 0 else initial + 0.5 * np.random.randn(len(initial))
        try:
            res = minimize(objective, p0, method="L-BFGS-B", options={"maxiter": 100, "disp": False})
            if res.fun < best_nll:
                best_nll, best = res.fun, res
        except Exception:  # noqa: BLE001  (the reference swallows restart failures)
            pass
    out = {"success": best is not None and best.success,
           "log_marginal_likelihood": -best_nll if best else None,
           "n_iterations": best.nit if best else 0}
    if best is None:
        return out, np.asarray(params0, float), noise0
    return out, best.x[:-1].copy(), float(np.exp(best.x[-1]))
