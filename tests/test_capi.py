"""The C-ABI library loads and exports every symbol include/gpmpc.h declares
(no compute call: runs without a GPU)."""
import ctypes
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(REPO, "include", "gpmpc.h")).read()
    return sorted(set(re.findall(r"\b(gpmpc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from gp_mpc_rocket_landing_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(header_symbols()) <= set(_lib.EXPORTED) | {"gpmpc_abi_version"}


def test_abi_version_and_error_string():
    from gp_mpc_rocket_landing_amd import _lib
    assert _lib.abi_version() == 4 == _lib.ABI_VERSION
    assert isinstance(_lib._L.gpmpc_last_error(), bytes)


def test_default_settings_pin_reference_osqp_config():
    """osqp_rti.py:54-60 + OSQP 0.6 defaults."""
    from gp_mpc_rocket_landing_amd import _lib
    s = _lib.qp_default_settings()
    assert (s.max_iter, s.check_termination, s.scaling, s.warm_start) == (50, 25, 3, 1)
    assert (s.rho, s.sigma, s.alpha, s.eps_abs, s.eps_rel) == (0.1, 1e-6, 1.6, 1e-4, 1e-4)
    assert (s.adaptive_rho, s.adaptive_rho_interval, s.adaptive_rho_tolerance) == (1, 25, 5.0)
    c = _lib.fleet_default_config()
    assert (c.horizon, c.dt, c.max_steps) == (20, 0.1, 300)


def test_settings_reject_unknown_keys():
    """ctypes structs accept any attribute name; the settings helpers must not
    (a typo such as max_iters=100 was silently ignored)."""
    import pytest
    from gp_mpc_rocket_landing_amd import _lib
    s = _lib.qp_default_settings(max_iter=7, eps_abs=1e-5)
    assert s.max_iter == 7 and s.eps_abs == 1e-5
    with pytest.raises(TypeError):
        _lib.qp_default_settings(max_iters=100)
    c = _lib.fleet_default_config(max_steps=12, max_iter=9)
    assert c.max_steps == 12 and c.qp.max_iter == 9
    with pytest.raises(TypeError):
        _lib.fleet_default_config(eps=1e-5)
    with pytest.raises(TypeError):
        _lib.fleet_default_config(qp=None)


def test_qp_caps_match_the_header():
    """_lib's QP caps (used for the OSQPRTIMPC pattern check) are csrc/qp.h's."""
    from gp_mpc_rocket_landing_amd import _lib
    src = open(os.path.join(REPO, "gp_mpc_rocket_landing_amd", "csrc", "qp.h")).read()
    caps = {k: int(v) for k, v in re.findall(r"#define (QP_NMAX|QP_MMAX|QP_NNZMAX) (\d+)", src)}
    assert caps == {"QP_NMAX": _lib.QP_NMAX, "QP_MMAX": _lib.QP_MMAX, "QP_NNZMAX": _lib.QP_NNZMAX}


def test_sqp_settings_default_to_qp_at_launch():
    """the SQP passes' settings default to "the same as qp" by a
    max_iter = 0 sentinel resolved at launch (csrc/fleet.hip fleet_args), so a
    C caller that edits only cfg.qp after gpmpc_fleet_default_config changes
    the passes as well; explicit sqp_qp settings start from the final qp."""
    from gp_mpc_rocket_landing_amd import _lib
    c = _lib.fleet_default_config()
    assert c.sqp_qp.max_iter == 0
    c = _lib.fleet_default_config(max_iter=80, sqp_qp=dict(eps_abs=1e-7))
    assert c.sqp_qp.max_iter == 80 and c.sqp_qp.eps_abs == 1e-7 and c.qp.eps_abs == 1e-4
