"""ctypes binding of oracle/admm_ref.c (TEST INFRASTRUCTURE / CPU BASELINE ONLY).

Builds ``oracle/_build/libadmm_ref.so`` with gcc on first use if it is missing.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import scipy.sparse as sp

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libadmm_ref.so")


class RefSettings(ctypes.Structure):
    _fields_ = [("rho", ctypes.c_double), ("sigma", ctypes.c_double), ("alpha", ctypes.c_double),
                ("eps_abs", ctypes.c_double), ("eps_rel", ctypes.c_double),
                ("eps_prim_inf", ctypes.c_double), ("eps_dual_inf", ctypes.c_double),
                ("max_iter", ctypes.c_int), ("check_termination", ctypes.c_int),
                ("adaptive_rho", ctypes.c_int), ("adaptive_rho_interval", ctypes.c_int),
                ("adaptive_rho_tolerance", ctypes.c_double), ("scaling", ctypes.c_int),
                ("warm_start", ctypes.c_int)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double); ip = ctypes.POINTER(ctypes.c_int)
        L.ref_qp_solve.argtypes = [ctypes.c_int, ctypes.c_int, ip, ip, dp, dp, dp, dp, dp,
                                   ctypes.POINTER(RefSettings), dp, dp, dp, dp, dp, ip, ip, dp, dp]
        L.ref_qp_solve.restype = ctypes.c_int
        L.ref_qp_default_settings.argtypes = [ctypes.POINTER(RefSettings)]
        _lib = L
    return _lib


def default_settings(**kw):
    s = RefSettings()
    lib().ref_qp_default_settings(ctypes.byref(s))
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def _d(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _i(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


class RefQP:
    """Persistent OSQP-like state (rho, scaled y) over successive solves."""

    def __init__(self, m, settings=None):
        self.s = settings or default_settings()
        self.rho = np.array([self.s.rho])
        self.y = np.zeros(m)

    def solve(self, Pdiag, q, A, l, u, x_ws):
        A = sp.csr_matrix(A)
        A.sort_indices()
        n, m = A.shape[1], A.shape[0]
        rp = np.ascontiguousarray(A.indptr, dtype=np.int32)
        ci = np.ascontiguousarray(A.indices, dtype=np.int32)
        av = np.ascontiguousarray(A.data, dtype=np.float64)
        P = np.ascontiguousarray(Pdiag, dtype=np.float64)
        q = np.ascontiguousarray(q, dtype=np.float64)
        l = np.ascontiguousarray(l, dtype=np.float64); u = np.ascontiguousarray(u, dtype=np.float64)
        xw = np.ascontiguousarray(x_ws, dtype=np.float64)
        x = np.empty(n); y = np.empty(m); obj = np.empty(1); res = np.empty(2)
        it = np.zeros(1, np.int32); st = np.zeros(1, np.int32)
        rc = lib().ref_qp_solve(n, m, _i(rp), _i(ci), _d(av), _d(P), _d(q), _d(l), _d(u),
                                ctypes.byref(self.s), _d(xw), _d(self.rho), _d(self.y), _d(x), _d(y),
                                _i(it), _i(st), _d(obj), _d(res))
        if rc != 0:
            raise RuntimeError("reduced KKT matrix not positive definite")
        return dict(x=x, y=y, iter=int(it[0]), status=int(st[0]), obj_val=float(obj[0]),
                    rho=float(self.rho[0]), pri_res=float(res[0]), dua_res=float(res[1]))
