"""The driver's entry points: build() compiles the library and the oracle and checks the
loaded library's ABI against the Python mirror's (a stale constant there once failed the
driver's build check); smoke() is importable (it needs a GPU to run)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def test_build_checks_the_mirrored_abi():
    import __graft_entry__ as g
    g.build()
    from gp_mpc_rocket_landing_amd import _lib
    assert _lib.abi_version() == _lib.ABI_VERSION
    assert callable(g.smoke)
