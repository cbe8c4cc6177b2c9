"""The N>1 path on CPU: contiguous (ragged) landing shards and the single
record gather, world_size 2 over gloo (the GPU run uses the same code over
RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from gp_mpc_rocket_landing_amd.sharding import shard_range


def test_shard_range_covers_total_contiguously():
    for total in (0, 1, 7, 1024, 1023):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            pos = 0
            for first, count in spans:
                assert first == pos and count >= 0
                pos += count
            assert pos == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _records_for(first, count):
    # a deterministic stand-in for a shard's fleet records: global index in col 0
    r = np.zeros((count, 16))
    r[:, 0] = np.arange(first, first + count)
    r[:, 1] = np.sqrt(np.arange(first, first + count))
    return r


def _worker(rank, world, total, port, q):
    import torch.distributed as dist
    from gp_mpc_rocket_landing_amd.sharding import gather_records
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = shard_range(total, rank, world)
    out = gather_records(_records_for(first, count), total)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [10, 11])
def test_gather_records_world2_gloo(total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, total, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    np.testing.assert_array_equal(out, _records_for(0, total))


def _fleet_records_worker(rank, world, total, port, q):
    """A rank's shard of real landings, flown by the CPU closed loop (the fleet's
    oracle, monte_carlo.py:401-583 restated), then the one gather."""
    import torch.distributed as dist
    from threadpoolctl import threadpool_limits
    from gp_mpc_rocket_landing_amd.data import synthetic_training_data
    from gp_mpc_rocket_landing_amd.fleet import initial_conditions
    from gp_mpc_rocket_landing_amd.sharding import gather_records
    from oracle import gp_oracle, mc_oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = shard_range(total, rank, world)
    with threadpool_limits(1):
        X, U, D = synthetic_training_data(1000, seed=0)
        st = gp_oracle.exact_fit(gp_oracle.features_3dof(X, U), D)
        x0 = initial_conditions(count, first=first)
        rec = np.array([mc_oracle.closed_loop_landing(st, x)[0] for x in x0]).reshape(count, 16)
    out = gather_records(rec, total)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_gather_real_landing_records_world2_gloo():
    """Two ranks each fly their contiguous (ragged: 4 + 3) shard of BASELINE
    configs[3] landings to termination and gather the records: rank 0 holds
    exactly the single-process Monte-Carlo's records (mc_oracle_1024.npz)."""
    from conftest import golden
    total = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fleet_records_worker, args=(r, 2, total, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    np.testing.assert_array_equal(out, golden("mc_oracle_1024.npz")["records"][:total])


def _agreed_gather_worker(rank, world, total, port, q):
    """gather_shard_records on a gloo group with no device context on any rank:
    the RCCL set-up fails everywhere, every rank learns that from the agreed
    readiness count, and all fall back to torch.distributed.gather together."""
    import torch.distributed as dist
    from gp_mpc_rocket_landing_amd.sharding import gather_shard_records
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = shard_range(total, rank, world)
    out, info = gather_shard_records(None, None, _records_for(first, count), total)
    q.put((rank, out, info))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_shard_records_agreed_fallback_world2_gloo():
    """The bench's / run_monte_carlo's gather: a failed RCCL set-up
    never leaves one rank in a collective the others skipped -- both ranks
    return, rank 0 holds the ragged records in global order, and the info
    records the path that ran, the ranks it spanned and the fallback reason."""
    total = 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agreed_gather_worker, args=(r, 2, total, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (o, i)) for r, o, i in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    out0, info0 = res[0]
    out1, info1 = res[1]
    np.testing.assert_array_equal(out0, _records_for(0, total))
    assert out1 is None
    for info in (info0, info1):
        assert info["path"] == "torch" and info["nranks"] == 2 and info["requested"] == "rccl"
        assert "2 of 2 ranks not ready" in info["fallback"], info
    assert info0["records"] == total and info1["records"] == 0


def test_gather_shard_records_world1_without_group():
    """No process group, no context: a world of one falls back to the host
    records themselves and says so."""
    from gp_mpc_rocket_landing_amd.sharding import gather_shard_records
    rec = _records_for(0, 5)
    out, info = gather_shard_records(None, None, rec, 5)
    np.testing.assert_array_equal(out, rec)
    assert info["path"] == "torch" and info["nranks"] == 1 and info["records"] == 5
    out, info = gather_shard_records(None, None, rec, 5, path="torch")
    assert info["fallback"] is None and info["path"] == "torch"
    import pytest
    with pytest.raises(ValueError):
        gather_shard_records(None, None, rec, 5, path="mpi")


class _FakeGather:
    """Stands in for RCCLRecordGather on a gloo group (no GPU): set-up succeeds,
    prepare fails on the ranks listed in FAIL_PREPARE, and a collective entered
    by any rank is recorded (it must never be entered when a prepare failed)."""
    FAIL_PREPARE = (1,)

    def __init__(self, ctx, _fail_local=False):
        from gp_mpc_rocket_landing_amd.sharding import _world
        self.world, self.rank, _ = _world()
        self.nranks = self.world
        self.closed = False
        self.entered = False

    def prepare(self, d_records, total):
        if self.rank in self.FAIL_PREPARE:
            raise RuntimeError("gather_prepare failed (-1): hipMalloc out of memory (injected)")

    def collective(self, total):
        self.entered = True
        raise AssertionError("collective entered although a peer's prepare failed")

    def close(self):
        self.closed = True


def _prepare_failure_worker(rank, world, total, port, q):
    import torch.distributed as dist
    from gp_mpc_rocket_landing_amd.sharding import gather_shard_records
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = shard_range(total, rank, world)
    made = []

    def factory(ctx, _fail_local=False):
        made.append(_FakeGather(ctx))
        return made[-1]
    out, info = gather_shard_records(None, None, _records_for(first, count), total, _gather=factory)
    q.put((rank, out, info, made[0].entered, made[0].closed))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_prepare_failure_on_one_rank_is_agreed_world2_gloo():
    """a failure in the local half of the gather (buffers, padding --
    gpmpc_gather_prepare) on ONE rank is agreed before anyone enters the
    collective: no rank calls it, both fall back to torch.distributed.gather
    together, and the communicator is closed only after the agreement."""
    total = 9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_prepare_failure_worker, args=(r, 2, total, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (out0, info0, ent0, cl0), (out1, info1, ent1, cl1) = res[0], res[1]
    np.testing.assert_array_equal(out0, _records_for(0, total))
    assert out1 is None
    assert not ent0 and not ent1 and cl0 and cl1
    for info in (info0, info1):
        assert info["path"] == "torch" and info["nranks"] == 2
        assert info["fallback"].startswith("gather prepare failed on 1 of 2 ranks"), info
    assert "injected" in info1["fallback"] and "injected" not in info0["fallback"]
