"""ctypes binding of libgpmpc_hip.so (include/gpmpc.h).

The product path has no CPU fallback: importing this module without the built
HIP library raises, and every call goes through the C-ABI.  Build with
``python -c "import __graft_entry__ as g; g.build()"`` (hipcc, gfx950).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPMPC_LIB") or os.path.join(_HERE, "libgpmpc_hip.so")  # GPMPC_LIB: A/B builds

SE_ARD, SE_ISO, MATERN32, MATERN52 = 0, 1, 2, 3
ERR_NOT_PD = -100
REC_LEN = 16
COMM_ID_BYTES = 128   # GPMPC_COMM_ID_BYTES (sizeof ncclUniqueId)
# caps of the generic device QP (csrc/qp.h QP_NMAX, QP_MMAX, QP_NNZMAX)
QP_NMAX, QP_MMAX, QP_NNZMAX = 216, 360, 896

QP_STATUS = {1: "solved", 2: "solved inaccurate", -2: "maximum iterations reached",
             -3: "primal infeasible", 3: "primal infeasible inaccurate", -4: "dual infeasible",
             4: "dual infeasible inaccurate", -7: "problem non convex", -10: "unsolved"}

if not os.path.exists(LIB_PATH):
    raise ImportError(f"HIP library missing: {LIB_PATH} (build it with __graft_entry__.build(); "
                      "there is no CPU fallback)")


def _share_torch_hip_runtime():
    """Make this process use ONE HIP runtime.  torch bundles its own
    libamdhip64 (SONAME libamdhip64.so.7, loaded by the unversioned name from
    torch/lib).  If our library pulled /opt/rocm's copy in first, torch would
    later load a second runtime, and whichever initialises second sees no
    device.  Preloading torch's copy globally lets our NEEDED libamdhip64.so.7
    resolve to it (GPMPC_HIP_RUNTIME=system keeps /opt/rocm's instead)."""
    if os.environ.get("GPMPC_HIP_RUNTIME", "") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    tlib = os.path.join(os.path.dirname(spec.origin), "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        p = os.path.join(tlib, name)
        if os.path.exists(p):
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)


_share_torch_hip_runtime()
_L = ctypes.CDLL(LIB_PATH)
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
_vp = ctypes.c_void_p


class QPSettings(ctypes.Structure):
    _fields_ = [("rho", ctypes.c_double), ("sigma", ctypes.c_double), ("alpha", ctypes.c_double),
                ("eps_abs", ctypes.c_double), ("eps_rel", ctypes.c_double),
                ("eps_prim_inf", ctypes.c_double), ("eps_dual_inf", ctypes.c_double),
                ("max_iter", ctypes.c_int), ("check_termination", ctypes.c_int),
                ("adaptive_rho", ctypes.c_int), ("adaptive_rho_interval", ctypes.c_int),
                ("adaptive_rho_tolerance", ctypes.c_double), ("scaling", ctypes.c_int),
                ("warm_start", ctypes.c_int)]


class Rollout6Config(ctypes.Structure):
    _fields_ = [("horizon", ctypes.c_int), ("dt", ctypes.c_double), ("max_steps", ctypes.c_int),
                ("qp", QPSettings), ("fitc_mean_as_written", ctypes.c_int),
                ("q_diag", ctypes.c_double * 14), ("p_diag", ctypes.c_double * 14),
                ("r_diag", ctypes.c_double * 3), ("t_min", ctypes.c_double), ("t_max", ctypes.c_double),
                ("tan_gamma_gs", ctypes.c_double), ("trust_x2", ctypes.c_double),
                ("trust_u2", ctypes.c_double), ("use_gp_mean", ctypes.c_int), ("upright_target", ctypes.c_int),
                ("rocket_j", ctypes.c_double * 3), ("rocket_r_t", ctypes.c_double * 3),
                ("rocket_g_i", ctypes.c_double * 3), ("rocket_alpha", ctypes.c_double),
                ("rocket_g0", ctypes.c_double), ("rocket_J", ctypes.c_double * 9)]


class FleetConfig(ctypes.Structure):
    _fields_ = [("horizon", ctypes.c_int), ("dt", ctypes.c_double), ("target_mode", ctypes.c_int),
                ("use_gp", ctypes.c_int), ("residual_model", ctypes.c_int),
                ("max_steps", ctypes.c_int), ("qp", QPSettings),
                ("sqp_iters", ctypes.c_int), ("sqp_tol", ctypes.c_double), ("sqp_qp", QPSettings)]


def _sig(name, res, *args):
    f = getattr(_L, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_c = ctypes.c_int
_sig("gpmpc_abi_version", _c)
ABI_VERSION = 4   # include/gpmpc.h GPMPC_ABI_VERSION this binding's structures follow
if _L.gpmpc_abi_version() != ABI_VERSION:
    raise ImportError(f"{LIB_PATH} has C-ABI {_L.gpmpc_abi_version()}, this binding needs {ABI_VERSION}: "
                      "rebuild it (__graft_entry__.build())")
_sig("gpmpc_last_error", ctypes.c_char_p)
_sig("gpmpc_ctx_create", _c, _c, ctypes.POINTER(_vp))
_sig("gpmpc_ctx_destroy", _c, _vp)
_sig("gpmpc_ctx_sync", _c, _vp)
_sig("gpmpc_ctx_stream", _vp, _vp)
_sig("gpmpc_gram", _c, _vp, _c, _dp, _c, _dp, _c, _c, _dp, ctypes.c_double, _dp, _c)
_sig("gpmpc_potrf", _c, _vp, _c, _dp, _c, _ip)
_sig("gpmpc_potrf_batched_dev", _c, _vp, _c, _c, _vp, _c, ctypes.c_int64, _vp)
_sig("gpmpc_trsm_lower", _c, _vp, _c, _c, _dp, _c, _dp, _c)
_sig("gpmpc_potrs", _c, _vp, _c, _c, _dp, _c, _dp, _c)
_sig("gpmpc_gp_fit_exact", _c, _vp, _c, _dp, _c, _c, _dp, _c, _dp, ctypes.c_double,
     ctypes.c_double, ctypes.POINTER(_vp), _dp, _dp, _dp, _ip)
_sig("gpmpc_gp_fit_exact_prog", _c, _vp, _ip, _c, _dp, _c, _dp, _c, _c, _dp, _c, ctypes.c_double,
     ctypes.POINTER(_vp), _dp, _dp, _dp, _ip)
_sig("gpmpc_sparse_fit_prog", _c, _vp, _c, _ip, _c, _dp, _c, _dp, _c, _dp, _c, _c, _dp, _c, ctypes.c_double,
     ctypes.c_double, ctypes.POINTER(_vp), _dp, _dp, _dp, _dp)
_sig("gpmpc_gp_predict", _c, _vp, _vp, _dp, _c, _dp, _dp)
_sig("gpmpc_gp_predict_cov", _c, _vp, _vp, _dp, _c, _dp, _dp)
_sig("gpmpc_gp_get_state", _c, _vp, _vp, _dp, _dp)
_sig("gpmpc_gp_destroy", _c, _vp)
_sig("gpmpc_gp_append", _c, _vp, _vp, _dp, _c, _dp, _dp, _dp, _dp)
_sig("gpmpc_gp_lml_batched", _c, _vp, _c, _dp, _c, _c, _dp, _c, _dp, _dp, _dp, _dp, _ip)
_sig("gpmpc_fitc_fit", _c, _vp, _dp, _c, _dp, _c, _c, _dp, _c, _dp, ctypes.c_double,
     ctypes.c_double, ctypes.c_double, ctypes.POINTER(_vp), _dp, _dp, _dp, _dp)
_sig("gpmpc_vfe_fit", _c, _vp, _dp, _c, _dp, _c, _c, _dp, _c, _dp, ctypes.c_double,
     ctypes.c_double, ctypes.c_double, ctypes.POINTER(_vp), _dp, _dp, _dp)
_sig("gpmpc_fitc_predict", _c, _vp, _vp, _dp, _c, _dp, _dp)
_sig("gpmpc_fitc_destroy", _c, _vp)
_sig("gpmpc_fitc_get_state", _c, _vp, _vp, _dp)
_sig("gpmpc_qp_default_settings", None, ctypes.POINTER(QPSettings))
_sig("gpmpc_qp_solve_batched", _c, _vp, _c, _c, _c, _c, _ip, _ip, _dp, _dp, _dp, _dp, _dp,
     ctypes.POINTER(QPSettings), _dp, _dp, _dp, _dp, _dp, _ip, _ip, _dp)
_sig("gpmpc_fleet_default_config", None, ctypes.POINTER(FleetConfig))
_sig("gpmpc_fleet_create", _c, _vp, _vp, ctypes.POINTER(FleetConfig), _c, ctypes.POINTER(_vp))
_sig("gpmpc_fleet_create_shard", _c, _vp, _vp, ctypes.POINTER(FleetConfig), _c, _c, ctypes.POINTER(_vp))
_sig("gpmpc_fleet_create_fitc", _c, _vp, _vp, ctypes.POINTER(FleetConfig), _c, _c, ctypes.POINTER(_vp))
_sig("gpmpc_fleet_reset", _c, _vp, _c, _c, _dp)
_sig("gpmpc_fleet_step", _c, _vp, _c)
_sig("gpmpc_fleet_step_phases", _c, _vp, _c)
_sig("gpmpc_fleet_set_stamps", _c, _vp, _vp)
_sig("gpmpc_fleet_set_trace", _c, _vp, _vp)
_sig("gpmpc_syrk_batched_dev", _c, _vp, _c, _c, _c, _vp, _c, ctypes.c_int64, _vp, _c, ctypes.c_int64,
     ctypes.c_double, ctypes.c_double)
_sig("gpmpc_cov_propagate", _c, _vp, _c, _c, _c, _dp, _dp, _vp, ctypes.c_double, _dp)
_sig("gpmpc_cov_propagate_dev", _c, _vp, _c, _c, _c, _vp, _vp, _vp, ctypes.c_double, _vp)
_sig("gpmpc_uprop3_linear", _c, _vp, _vp, _c, _c, ctypes.c_double, ctypes.c_double, _dp, _dp, _dp, _vp,
     ctypes.c_double, _dp, _dp)
_sig("gpmpc_uprop6_linear", _c, _vp, _vp, _vp, _c, _dp, _c, _c, ctypes.c_double, _dp, _dp, _vp,
     ctypes.c_double, _dp, _dp)
_sig("gpmpc_fleet_read", _c, _vp, _dp, _dp)
_sig("gpmpc_gram_grad", _c, _vp, _c, _dp, _c, _dp, _c, _c, _dp, ctypes.c_double, _dp, _dp)
_sig("gpmpc_fleet_get_state", _c, _vp, _dp, _dp, _dp, _dp)
_sig("gpmpc_fleet_get_posterior", _c, _vp, _dp, _dp)
_sig("gpmpc_fleet_records_dev", _vp, _vp)
_sig("gpmpc_fleet_destroy", _c, _vp)
_sig("gpmpc_rollout6_default_config", None, ctypes.POINTER(Rollout6Config))
_sig("gpmpc_rollout6_create", _c, _vp, _vp, _vp, ctypes.POINTER(Rollout6Config), _c, ctypes.POINTER(_vp))
_sig("gpmpc_rollout6_create_exact", _c, _vp, _vp, _vp, ctypes.POINTER(Rollout6Config), _c, ctypes.POINTER(_vp))
_sig("gpmpc_rollout6_solve", _c, _vp, _dp, _dp, _c, _c, ctypes.c_double, _dp, _dp, _ip, _ip, _ip, _ip)
_sig("gpmpc_rollout6_solve_ref", _c, _vp, _dp, _dp, _dp, _dp, _c, _c, ctypes.c_double, _dp, _dp, _ip, _ip, _ip,
     _ip)
_sig("gpmpc_rollout6_set_state", _c, _vp, _dp, _dp, _dp)
_sig("gpmpc_rollout6_records_dev", _vp, _vp)
_sig("gpmpc_comm_unique_id", _c, ctypes.c_char_p)
_sig("gpmpc_comm_init", _c, _vp, ctypes.c_char_p, _c, _c, ctypes.POINTER(_vp))
_sig("gpmpc_comm_destroy", _c, _vp)
_sig("gpmpc_comm_count", _c, _vp, _ip)
_sig("gpmpc_gather_results", _c, _vp, _vp, _vp, _ip, _c, _dp)
_sig("gpmpc_gather_prepare", _c, _vp, _vp, _vp, _ip, _c)
_sig("gpmpc_gather_collective", _c, _vp, _vp, _ip, _c, _dp)
_sig("gpmpc_rollout6_reset", _c, _vp, _c, _c, _dp)
_sig("gpmpc_rollout6_step", _c, _vp, _c)
_sig("gpmpc_rollout6_step_phases", _c, _vp, _c)
_sig("gpmpc_rollout6_read", _c, _vp, _dp, _dp)
_sig("gpmpc_rollout6_get_state", _c, _vp, _dp, _dp, _dp, _dp, _dp, _dp)
_sig("gpmpc_rollout6_destroy", _c, _vp)

EXPORTED = ["gpmpc_abi_version", "gpmpc_last_error", "gpmpc_ctx_create", "gpmpc_ctx_destroy",
            "gpmpc_ctx_sync", "gpmpc_ctx_stream", "gpmpc_gram", "gpmpc_gram_grad", "gpmpc_potrf",
            "gpmpc_potrf_batched_dev", "gpmpc_trsm_lower", "gpmpc_potrs", "gpmpc_gp_fit_exact",
            "gpmpc_gp_predict", "gpmpc_gp_predict_cov", "gpmpc_gp_fit_exact_prog", "gpmpc_sparse_fit_prog", "gpmpc_gp_get_state", "gpmpc_gp_destroy",
            "gpmpc_gp_lml_batched", "gpmpc_gp_append",
            "gpmpc_fitc_fit", "gpmpc_fitc_predict", "gpmpc_fitc_destroy",
            "gpmpc_qp_default_settings", "gpmpc_qp_solve_batched", "gpmpc_fleet_default_config",
            "gpmpc_fleet_create", "gpmpc_fleet_create_shard", "gpmpc_fleet_create_fitc", "gpmpc_fleet_reset", "gpmpc_fleet_step", "gpmpc_fleet_read",
            "gpmpc_fleet_step_phases", "gpmpc_fleet_get_state", "gpmpc_fleet_get_posterior", "gpmpc_fleet_set_stamps", "gpmpc_fleet_set_trace",
            "gpmpc_syrk_batched_dev", "gpmpc_cov_propagate", "gpmpc_cov_propagate_dev", "gpmpc_uprop3_linear", "gpmpc_uprop6_linear",
            "gpmpc_fleet_records_dev", "gpmpc_fleet_destroy", "gpmpc_rollout6_default_config",
            "gpmpc_rollout6_create", "gpmpc_rollout6_reset", "gpmpc_rollout6_step", "gpmpc_rollout6_read",
            "gpmpc_rollout6_get_state", "gpmpc_rollout6_destroy", "gpmpc_rollout6_create_exact",
            "gpmpc_rollout6_solve", "gpmpc_rollout6_solve_ref", "gpmpc_rollout6_set_state", "gpmpc_fitc_get_state",
            "gpmpc_rollout6_records_dev", "gpmpc_comm_unique_id", "gpmpc_comm_init", "gpmpc_comm_destroy",
            "gpmpc_comm_count", "gpmpc_gather_results", "gpmpc_gather_prepare", "gpmpc_gather_collective", "gpmpc_rollout6_step_phases", "gpmpc_vfe_fit"]


class HIPError(RuntimeError):
    """A C-ABI call returned non-zero; ``rc`` is its return code (-2: the arguments
    were refused, e.g. a malformed composite-kernel program)."""

    def __init__(self, msg, rc=None):
        super().__init__(msg)
        self.rc = rc


def _err(rc, what):
    msg = _L.gpmpc_last_error().decode(errors="replace")
    raise HIPError(f"{what} failed ({rc}): {msg}", rc)


def _chk(rc, what):
    if rc != 0:
        _err(rc, what)


def _d(a):
    return a.ctypes.data_as(_dp)


def _i(a):
    return a.ctypes.data_as(_ip)


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def abi_version():
    return _L.gpmpc_abi_version()


class Context:
    """One HIP device + stream (gpmpc_ctx)."""

    def __init__(self, device=0):
        h = _vp()
        _chk(_L.gpmpc_ctx_create(int(device), ctypes.byref(h)), "gpmpc_ctx_create")
        self.h = h
        self.device = device

    @property
    def stream(self):
        return _L.gpmpc_ctx_stream(self.h)

    def sync(self):
        _chk(_L.gpmpc_ctx_sync(self.h), "gpmpc_ctx_sync")

    def close(self):
        if self.h:
            _L.gpmpc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(int(os.environ.get("GPMPC_DEVICE", "0")))
    return _default_ctx


# ---- thin wrappers -----------------------------------------------------------
def gram(ctx, kind, X1, X2, ls, sigma2):
    X1 = f64(np.atleast_2d(X1)); n1, d = X1.shape
    ls = f64(np.atleast_1d(ls))
    if ls.size == 1 and kind != SE_ISO:
        ls = np.full(d, float(ls[0]))
    if X2 is None:
        K = np.empty((n1, n1))
        _chk(_L.gpmpc_gram(ctx.h, kind, _d(X1), n1, None, n1, d, _d(ls), float(sigma2), _d(K), n1), "gram")
        return K
    X2 = f64(np.atleast_2d(X2)); n2 = X2.shape[0]
    K = np.empty((n1, n2))
    _chk(_L.gpmpc_gram(ctx.h, kind, _d(X1), n1, _d(X2), n2, d, _d(ls), float(sigma2), _d(K), n2), "gram")
    return K


def gram_grad(ctx, kind, X1, X2, ls, sigma2):
    """(K, G): the Gram and its log-hyperparameter gradients (gpmpc_gram_grad):
    G (d, n1, n2) for SE_ARD, (1, n1, n2) for SE_ISO."""
    X1 = f64(np.atleast_2d(X1)); n1, d = X1.shape
    ls = f64(np.atleast_1d(ls))
    if ls.size == 1 and kind != SE_ISO:
        ls = np.full(d, float(ls[0]))
    X2a = None if X2 is None else f64(np.atleast_2d(X2))
    n2 = n1 if X2a is None else X2a.shape[0]
    K = np.empty((n1, n2)); G = np.empty((1 if kind == SE_ISO else d, n1, n2))
    _chk(_L.gpmpc_gram_grad(ctx.h, kind, _d(X1), n1, None if X2a is None else _d(X2a), n2, d, _d(ls),
                            float(sigma2), _d(K), _d(G)), "gram_grad")
    return K, G


def potrf(ctx, A):
    """Lower Cholesky of A (returns L with a zero upper triangle) and LAPACK info."""
    A = f64(A).copy(); n = A.shape[0]
    info = np.zeros(1, np.int32)
    rc = _L.gpmpc_potrf(ctx.h, n, _d(A), n, _i(info))
    if rc < 0:
        _err(rc, "potrf")
    return np.tril(A), int(info[0])


def trsm_lower(ctx, L, B):
    L = f64(L); B = f64(B).copy()
    vec = B.ndim == 1
    if vec:
        B = B[:, None].copy()
    _chk(_L.gpmpc_trsm_lower(ctx.h, L.shape[0], B.shape[1], _d(L), L.shape[0], _d(B), B.shape[1]), "trsm")
    return B[:, 0] if vec else B


def potrs(ctx, L, B):
    L = f64(L); B = f64(B).copy()
    vec = B.ndim == 1
    if vec:
        B = B[:, None].copy()
    _chk(_L.gpmpc_potrs(ctx.h, L.shape[0], B.shape[1], _d(L), L.shape[0], _d(B), B.shape[1]), "potrs")
    return B[:, 0] if vec else B


def gp_lml_batched(ctx, kind, X, y, ls, sigma2, noise):
    """Log marginal likelihood of the exact GP at B parameter sets (rows of ls
    (B x d; SE_ISO: B x 1), sigma2 (B,), noise (B,)): returns (lml (B,),
    jitter_steps (B,)); -inf / -1 where the jitter ladder is exhausted."""
    X = f64(np.atleast_2d(X)); n, d = X.shape
    y = f64(np.asarray(y).reshape(-1))
    assert y.size == n, "X and y must have same number of samples"
    sigma2 = f64(np.atleast_1d(sigma2)); B = sigma2.size
    noise = f64(np.broadcast_to(np.atleast_1d(noise), (B,)))
    ls = np.atleast_2d(np.asarray(ls, dtype=np.float64))
    L = np.empty((B, d))
    L[:] = ls[:, :1] if ls.shape[1] == 1 else ls
    L = f64(L)
    lml = np.empty(B); steps = np.empty(B, np.int32)
    _chk(_L.gpmpc_gp_lml_batched(ctx.h, kind, _d(X), n, d, _d(y), B, _d(L), _d(sigma2), _d(noise),
                                 _d(lml), _i(steps)), "gp_lml_batched")
    return lml, steps


KP_WHITE, KP_SUM, KP_PROD = 4, 10, 11   # gpmpc.h GPMPC_KP_*


class KernelProgram:
    """A composite kernel (SumKernel / ProductKernel / WhiteNoise over the stationary
    kernels, kernels.py:676-844) as the device's postfix program: ``ops`` (code,
    parameter offset) pairs and ``par`` (gpmpc.h GPMPC_KP_*).  Passed as ``kind`` to
    ExactGPHandle / FITCHandle, which then ignore ``ls`` / ``sigma2``."""

    def __init__(self, ops, par):
        self.ops = np.ascontiguousarray(np.asarray(ops, np.int32).reshape(-1, 2))
        self.par = f64(np.asarray(par, float).reshape(-1))

    def __eq__(self, other):
        return (isinstance(other, KernelProgram) and np.array_equal(self.ops, other.ops)
                and np.array_equal(self.par, other.par))

    def __repr__(self):
        return f"KernelProgram(ops={self.ops.tolist()}, par={self.par.tolist()})"


class ExactGPHandle:
    """Device-resident exact GP (shared factor across outputs).  ``kind``: one of the
    four kernel kinds, or a KernelProgram (a composite kernel)."""

    def __init__(self, ctx, kind, X, Y, ls, sigma2, noise):
        X = f64(np.atleast_2d(X)); Y = f64(Y)
        if Y.ndim == 1:
            Y = Y[:, None]
        n, d = X.shape; no = Y.shape[1]
        self.ctx = ctx; self.n = n; self.d = d; self.n_out = no
        self.y_mean = np.empty(no); self.y_std = np.empty(no); self.lml = np.empty(no)
        js = np.zeros(1, np.int32)
        h = _vp()
        if isinstance(kind, KernelProgram):
            rc = _L.gpmpc_gp_fit_exact_prog(ctx.h, _i(kind.ops), kind.ops.shape[0], _d(kind.par), kind.par.size,
                                            _d(X), n, d, _d(Y), no, float(noise), ctypes.byref(h),
                                            _d(self.y_mean), _d(self.y_std), _d(self.lml), _i(js))
        else:
            ls = f64(np.atleast_1d(ls))
            if ls.size == 1 and kind != SE_ISO:
                ls = np.full(d, float(ls[0]))
            rc = _L.gpmpc_gp_fit_exact(ctx.h, kind, _d(X), n, d, _d(Y), no, _d(ls), float(sigma2),
                                       float(noise), ctypes.byref(h), _d(self.y_mean), _d(self.y_std),
                                       _d(self.lml), _i(js))
        if rc == ERR_NOT_PD:
            raise ValueError("Kernel matrix is not positive definite even with jitter")
        _chk(rc, "gp_fit_exact")
        self.h = h
        self.jitter_steps = int(js[0])

    def append(self, Xnew, Yall):
        """Grow the GP by the rows Xnew (k x d) in O(n^2 k) (gpmpc_gp_append);
        Yall = the targets of all n + k rows.  False (handle unchanged) when the
        caller must refit instead (jitter-fitted GP / indefinite Schur complement)."""
        Xnew = f64(np.atleast_2d(Xnew)); k = Xnew.shape[0]
        Yall = f64(Yall)
        if Yall.ndim == 1:
            Yall = Yall[:, None]
        assert Xnew.shape[1] == self.d and Yall.shape == (self.n + k, self.n_out)
        ym = np.empty(self.n_out); ys = np.empty(self.n_out); lml = np.empty(self.n_out)
        rc = _L.gpmpc_gp_append(self.ctx.h, self.h, _d(Xnew), k, _d(Yall), _d(ym), _d(ys), _d(lml))
        if rc == ERR_NOT_PD:
            return False
        _chk(rc, "gp_append")
        self.n += k
        self.y_mean, self.y_std, self.lml = ym, ys, lml
        return True

    def predict(self, Xq):
        Xq = f64(np.atleast_2d(Xq)); p = Xq.shape[0]
        mean = np.empty((p, self.n_out)); var = np.empty((p, self.n_out))
        _chk(_L.gpmpc_gp_predict(self.ctx.h, self.h, _d(Xq), p, _d(mean), _d(var)), "gp_predict")
        return mean, var

    def predict_cov(self, Xq):
        Xq = f64(np.atleast_2d(Xq)); p = Xq.shape[0]
        mean = np.empty((p, self.n_out)); cov = np.empty((p, p))
        _chk(_L.gpmpc_gp_predict_cov(self.ctx.h, self.h, _d(Xq), p, _d(mean), _d(cov)), "gp_predict_cov")
        return mean, cov

    def state(self):
        L = np.empty((self.n, self.n)); a = np.empty((self.n, self.n_out))
        _chk(_L.gpmpc_gp_get_state(self.ctx.h, self.h, _d(L), _d(a)), "gp_get_state")
        return L, a

    def __del__(self):
        try:
            if getattr(self, "h", None):
                _L.gpmpc_gp_destroy(self.h)
                self.h = None
        except Exception:
            pass


class FITCHandle:
    """A fitted sparse GP on the device: FITC (gpmpc_fitc_fit) or, with
    ``method="vfe"``, VFE (gpmpc_vfe_fit; ``lam`` is then None)."""

    def __init__(self, ctx, Z, X, Y, ls, sigma2, noise, jitter=1e-6, method="fitc"):
        Z = f64(np.atleast_2d(Z)); X = f64(np.atleast_2d(X)); Y = f64(Y)
        if Y.ndim == 1:
            Y = Y[:, None]
        m, d = Z.shape; n = X.shape[0]; no = Y.shape[1]
        self.ctx = ctx; self.n_out = no; self.m = m
        self.y_mean = np.empty(no); self.y_std = np.empty(no); self.lml = np.empty(no)
        h = _vp()
        prog = ls if isinstance(ls, KernelProgram) else None
        if prog is None:
            ls = f64(np.atleast_1d(ls))
            if ls.size == 1:
                ls = np.full(d, float(ls[0]))
        if prog is not None and method in ("fitc", "vfe"):
            # a composite kernel (``ls`` is its KernelProgram): gpmpc_sparse_fit_prog
            self.lam = np.empty(n) if method == "fitc" else None
            rc = _L.gpmpc_sparse_fit_prog(ctx.h, 0 if method == "fitc" else 1, _i(prog.ops), prog.ops.shape[0],
                                          _d(prog.par), prog.par.size, _d(Z), m, _d(X), n, d, _d(Y), no,
                                          float(noise), float(jitter), ctypes.byref(h), _d(self.y_mean),
                                          _d(self.y_std), _d(self.lml),
                                          _d(self.lam) if self.lam is not None else None)
        elif method == "vfe":
            self.lam = None
            rc = _L.gpmpc_vfe_fit(ctx.h, _d(Z), m, _d(X), n, d, _d(Y), no, _d(ls), float(sigma2),
                                  float(noise), float(jitter), ctypes.byref(h), _d(self.y_mean),
                                  _d(self.y_std), _d(self.lml))
        elif method == "fitc":
            self.lam = np.empty(n)
            rc = _L.gpmpc_fitc_fit(ctx.h, _d(Z), m, _d(X), n, d, _d(Y), no, _d(ls), float(sigma2),
                                   float(noise), float(jitter), ctypes.byref(h), _d(self.y_mean),
                                   _d(self.y_std), _d(self.lml), _d(self.lam))
        else:
            raise ValueError(f"method must be 'fitc' or 'vfe', got {method!r}")
        if rc > 0:
            raise np.linalg.LinAlgError(_L.gpmpc_last_error().decode())
        _chk(rc, "fitc_fit")
        self.h = h

    def predict(self, Xq):
        Xq = f64(np.atleast_2d(Xq)); p = Xq.shape[0]
        mean = np.empty((p, self.n_out)); var = np.empty((p, self.n_out))
        _chk(_L.gpmpc_fitc_predict(self.ctx.h, self.h, _d(Xq), p, _d(mean), _d(var)), "fitc_predict")
        return mean, var

    def alpha(self):
        """The fitted alpha (m x n_out), gpmpc_fitc_get_state."""
        a = np.empty((self.m, self.n_out))
        _chk(_L.gpmpc_fitc_get_state(self.ctx.h, self.h, _d(a)), "fitc_get_state")
        return a

    def __del__(self):
        try:
            if getattr(self, "h", None):
                _L.gpmpc_fitc_destroy(self.h)
                self.h = None
        except Exception:
            pass


def _field_names(struct):
    return {f[0] for f in struct._fields_}


def set_fields(struct, kw, nested=None):
    """Assign keyword settings to a ctypes struct, refusing names it does not
    have (ctypes would silently accept a typo such as ``max_iters``).  Keys
    unknown to ``struct`` go to the ``nested`` member struct when given."""
    own = _field_names(type(struct))
    sub = getattr(struct, nested) if nested else None
    subn = _field_names(type(sub)) if sub is not None else set()
    for k, v in kw.items():
        if k in own and k != nested:
            cur = getattr(struct, k)
            if isinstance(cur, ctypes.Structure) and isinstance(v, dict):  # a nested settings struct
                set_fields(cur, v)
                continue
            if isinstance(cur, ctypes.Array):  # fixed-size array fields take a sequence
                v = np.ravel(np.asarray(v, dtype=np.float64))
                if v.size != len(cur):
                    raise ValueError(f"{k} needs {len(cur)} values, got {v.size}")
                v = type(cur)(*v.tolist())
            setattr(struct, k, v)
        elif k in subn:
            setattr(sub, k, v)
        else:
            raise TypeError(f"unknown setting {k!r} for {type(struct).__name__}")
    return struct


def qp_default_settings(**kw):
    s = QPSettings()
    _L.gpmpc_qp_default_settings(ctypes.byref(s))
    return set_fields(s, kw)


def rollout6_default_config(**kw):
    """6-DoF rollout config; QP settings may be given flat (``max_iter=...``)."""
    c = Rollout6Config()
    _L.gpmpc_rollout6_default_config(ctypes.byref(c))
    return set_fields(c, kw, nested="qp")


def fleet_default_config(**kw):
    """Fleet config; QP settings may be given flat (``max_iter=...``); the SQP
    passes' settings as ``sqp_qp=dict(...)`` on top of the (final) ``qp``."""
    c = FleetConfig()
    _L.gpmpc_fleet_default_config(ctypes.byref(c))
    sq = kw.pop("sqp_qp", None)
    set_fields(c, kw, nested="qp")
    if sq:   # explicit pass settings on top of qp; otherwise max_iter 0 = "the same as qp"
        c.sqp_qp = c.qp
        set_fields(c.sqp_qp, sq)
    return c


class QPWorkspace:
    """OSQP-workspace equivalent over gpmpc_qp_solve_batched: a fixed CSR
    pattern of A shared by ``batch`` problems, diagonal P, and the state OSQP
    keeps between solves (rho, scaled y).  Mirrors osqp.OSQP().setup/update/
    warm_start/solve as osqp_rti.py:454-567 drives it."""

    def __init__(self, ctx, n, m, rowptr, colidx, batch=1, settings=None):
        self.ctx = ctx; self.n = int(n); self.m = int(m); self.batch = int(batch)
        self.rowptr = np.ascontiguousarray(rowptr, np.int32)
        self.colidx = np.ascontiguousarray(colidx, np.int32)
        self.nnz = int(self.rowptr[-1])
        self.settings = settings if settings is not None else qp_default_settings()
        self.reset()

    def reset(self):
        """Fresh workspace: rho back to settings.rho, y = 0 (osqp.OSQP().setup)."""
        self.rho = np.full(self.batch, float(self.settings.rho))
        self.y_scaled = np.zeros((self.batch, self.m))

    def solve(self, Aval, Pdiag, q, l, u, x_ws=None, pattern=None):
        """``pattern`` = (rowptr, colidx) replaces the workspace's pattern for this
        solve (a value-filtered A whose non-zeros move); the rows, and
        with them OSQP's persistent y, stay the same."""
        B, n, m = self.batch, self.n, self.m
        rowptr, colidx = self.rowptr, self.colidx
        if pattern is not None:
            rowptr = np.ascontiguousarray(pattern[0], np.int32)
            colidx = np.ascontiguousarray(pattern[1], np.int32)
            assert rowptr.size == m + 1
        nnz = int(rowptr[-1])
        Av = f64(np.reshape(Aval, (B, nnz))); Pd = f64(np.reshape(Pdiag, (B, n)))
        qv = f64(np.reshape(q, (B, n))); lv = f64(np.reshape(l, (B, m))); uv = f64(np.reshape(u, (B, m)))
        xw = None if x_ws is None else f64(np.reshape(x_ws, (B, n)))
        x = np.empty((B, n)); y = np.empty((B, m)); obj = np.empty(B)
        it = np.zeros(B, np.int32); st = np.zeros(B, np.int32)
        rc = _L.gpmpc_qp_solve_batched(self.ctx.h, B, n, m, nnz, _i(rowptr), _i(colidx),
                                       _d(Av), _d(Pd), _d(qv), _d(lv), _d(uv), ctypes.byref(self.settings),
                                       None if xw is None else _d(xw), _d(self.rho), _d(self.y_scaled),
                                       _d(x), _d(y), _i(it), _i(st), _d(obj))
        _chk(rc, "qp_solve_batched")
        return dict(x=x, y=y, iter=it, status=st, obj_val=obj, rho=self.rho.copy())


QP_STATUS_TEXT = {1: "solved", 2: "solved_inaccurate", -2: "maximum iterations reached",
                  -3: "primal infeasible", 3: "primal infeasible inaccurate",
                  -4: "dual infeasible", 4: "dual infeasible inaccurate", -7: "problem non convex",
                  -10: "unsolved", -100: "kkt factorisation failed"}


def uprop3_linear(ctx, gp, X0, U, S0=None, dt=0.1, alpha=1.0 / 30.0, g=(-1.0, 0.0, 0.0), s0_diag=1e-6):
    """gpmpc_uprop3_linear: the 3-DoF linear uncertainty propagation of B trajectories on the
    device.  gp: an ExactGPHandle of the 3-DoF GP; X0 (B, 7), U (B, N, 3), S0 None or
    (B, 7, 7) -> means (B, N+1, 7), covariances (B, N+1, 7, 7)."""
    X0 = f64(np.atleast_2d(X0)); U = f64(U)
    B, N = U.shape[0], U.shape[1]
    if X0.shape != (B, 7) or U.shape != (B, N, 3):
        raise ValueError(f"uprop3_linear: shapes X0 {X0.shape}, U {U.shape}")
    g3 = f64(np.asarray(g, float).reshape(3))
    means = np.empty((B, N + 1, 7)); covs = np.empty((B, N + 1, 7, 7))
    s0 = None
    if S0 is not None:
        S0 = f64(S0)
        if S0.shape != (B, 7, 7):
            raise ValueError(f"uprop3_linear: S0 shape {S0.shape}")
        s0 = S0.ctypes.data_as(_vp)
    _chk(_L.gpmpc_uprop3_linear(ctx.h, gp.h, B, N, float(dt), float(alpha), _d(g3), _d(X0), _d(U), s0,
                                float(s0_diag), _d(means), _d(covs)), "uprop3_linear")
    return means, covs


def uprop6_linear(ctx, hv, hw, exact, rocket, X0, U, S0=None, dt=0.1, s0_diag=1e-6):
    """gpmpc_uprop6_linear: the 14-state linear uncertainty propagation of B trajectories on
    the device.  hv, hw: the StructuredRocketGP's device pair (ExactGPHandle with exact=True,
    else FITCHandle); rocket: 17 doubles (J_B row-major, r_T_B, g_I, alpha, g0); X0 (B, 14),
    U (B, N, 3), S0 None or (B, 14, 14) -> means (B, N+1, 14), covariances (B, N+1, 14, 14)."""
    X0 = f64(np.atleast_2d(X0)); U = f64(U)
    B, N = U.shape[0], U.shape[1]
    if X0.shape != (B, 14) or U.shape != (B, N, 3):
        raise ValueError(f"uprop6_linear: shapes X0 {X0.shape}, U {U.shape}")
    rk = f64(np.asarray(rocket, float).reshape(17))
    means = np.empty((B, N + 1, 14)); covs = np.empty((B, N + 1, 14, 14))
    s0 = None
    if S0 is not None:
        S0 = f64(S0)
        if S0.shape != (B, 14, 14):
            raise ValueError(f"uprop6_linear: S0 shape {S0.shape}")
        s0 = S0.ctypes.data_as(_vp)
    _chk(_L.gpmpc_uprop6_linear(ctx.h, hv.h, hw.h, int(bool(exact)), _d(rk), B, N, float(dt), _d(X0), _d(U), s0,
                                float(s0_diag), _d(means), _d(covs)), "uprop6_linear")
    return means, covs


def cov_propagate(ctx, A, q, S0=None, s0_diag=1e-6):
    """Batched Sigma_{k+1} = A_k Sigma_k A_k^T + diag(q_k) on the device.
    A (B, N, nx, nx), q (B, N, nx), S0 (B, nx, nx) or None -> (B, N+1, nx, nx)."""
    A = f64(A); q = f64(q)
    B, N, nx = A.shape[0], A.shape[1], A.shape[-1]
    if A.shape != (B, N, nx, nx) or q.shape != (B, N, nx):
        raise ValueError(f"cov_propagate: shapes A {A.shape}, q {q.shape}")
    out = np.empty((B, N + 1, nx, nx))
    s0 = None
    if S0 is not None:
        S0 = f64(S0)
        if S0.shape != (B, nx, nx):
            raise ValueError(f"cov_propagate: S0 shape {S0.shape}")
        s0 = S0.ctypes.data_as(_vp)
    _chk(_L.gpmpc_cov_propagate(ctx.h, B, N, nx, _d(A), _d(q), s0, float(s0_diag), _d(out)),
         "cov_propagate")
    return out
