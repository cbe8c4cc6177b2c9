"""The C-ABI gather (gpmpc_comm_* / gpmpc_gather_results) on
the GPU box's one device: a world of one exercises the RCCL bootstrap
(unique id, ncclCommInitRank), the device-side padding of a ragged shard and
the ncclGather itself; the ragged multi-rank compaction is the same code as
the gloo-tested Python path (tests/test_sharding.py) and runs at N > 1 in
the driver's multi-GPU bench."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_gather_fleet_records_world1(gpu_ctx):
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    from gp_mpc_rocket_landing_amd.sharding import RCCLRecordGather
    gp = fit_gp(gpu_ctx, n_train=200)
    fl = Fleet(gpu_ctx, gp, 37)
    g = RCCLRecordGather(gpu_ctx)
    try:
        fl.reset(initial_conditions(37))
        fl.step(5)
        rec, _ = fl.read()
        out = g.gather(fl.records_dev, 37)
        np.testing.assert_array_equal(out, rec)
        assert (g.world, g.rank, g.nranks) == (1, 0, 1)
    finally:
        g.close()
        fl.close()


def test_rccl_gather_rollout6_records_world1(gpu_ctx):
    from gp_mpc_rocket_landing_amd.rollouts6 import Rollouts6, fit_structured_fitc, initial_conditions_6dof
    from gp_mpc_rocket_landing_amd.sharding import RCCLRecordGather
    gv, gw = fit_structured_fitc(gpu_ctx, n_train=300, n_inducing=50)
    ro = Rollouts6(gpu_ctx, gv, gw, 5)
    g = RCCLRecordGather(gpu_ctx)
    try:
        ro.reset(initial_conditions_6dof(5))
        ro.step(3)
        rec, _ = ro.read()
        np.testing.assert_array_equal(g.gather(ro.records_dev, 5), rec)
    finally:
        g.close()
        ro.close()


def test_gather_shard_records_world1_reports_rccl(gpu_ctx):
    """The bench's gather helper on the GPU: the RCCL path runs
    (no fallback), its info names it, the ranks RCCL's communicator spans
    (ncclCommCount) and the rows gathered; the records equal the fleet's."""
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    from gp_mpc_rocket_landing_amd.sharding import gather_shard_records
    gp = fit_gp(gpu_ctx, n_train=200)
    fl = Fleet(gpu_ctx, gp, 21)
    try:
        fl.reset(initial_conditions(21))
        fl.step(3)
        rec, _ = fl.read()
        out, info = gather_shard_records(gpu_ctx, fl.records_dev, rec, 21)
        np.testing.assert_array_equal(out, rec)
        assert info == {"path": "rccl", "nranks": 1, "records": 21, "requested": "rccl", "fallback": None}
    finally:
        fl.close()


def test_gather_collective_refuses_counts_other_than_prepared(gpu_ctx):
    """gpmpc_gather_collective with counts or a root other than those its prepare
    sized and padded the buffers for returns -2 instead of gathering a block of
    another size; the prepared block stays valid for the right call."""
    from gp_mpc_rocket_landing_amd import _lib
    from gp_mpc_rocket_landing_amd.fleet import Fleet, fit_gp, initial_conditions
    from gp_mpc_rocket_landing_amd.sharding import RCCLRecordGather
    gp = fit_gp(gpu_ctx, n_train=200)
    fl = Fleet(gpu_ctx, gp, 9)
    g = RCCLRecordGather(gpu_ctx)
    try:
        fl.reset(initial_conditions(9))
        fl.step(2)
        rec, _ = fl.read()
        g.prepare(fl.records_dev, 9)
        out = np.empty((40, _lib.REC_LEN))
        rc = _lib._L.gpmpc_gather_collective(gpu_ctx.h, g.h, _lib._i(np.array([40], np.int32)), 0, _lib._d(out))
        assert rc == -2 and "differ" in _lib._L.gpmpc_last_error().decode()
        np.testing.assert_array_equal(g.collective(9), rec)
    finally:
        g.close()
        fl.close()
