"""Landing shards across ranks and the one collective of the path.

Monte-Carlo landings are independent (monte_carlo.py:401-583 depends only on
x0 and the seed), so rank r of G owns the contiguous block
[r*B/G, (r+1)*B/G) and runs it on its own GPU with no data-path
communication.  At the end the fixed-size per-landing records
(GPMPC_REC_LEN doubles) are gathered to rank 0 with ONE gather -- RCCL over
xGMI on GPUs (backend "nccl"), gloo in the CPU tests.  Shards may be ragged
(B not divisible by G): records are padded to the largest shard for the
gather and trimmed on rank 0.
"""
from __future__ import annotations

import os

import numpy as np


def shard_range(total: int, rank: int, world: int):
    """Contiguous [first, first+count) of ``total`` items for ``rank`` of ``world``."""
    base, extra = divmod(int(total), int(world))
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def gather_records(records: np.ndarray, total: int, device=None):
    """Gather every rank's (count, L) record block to rank 0 in global order.

    Returns the (total, L) array on rank 0 and None elsewhere.  One collective
    (torch.distributed.gather) of max-shard-sized padded blocks."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    L = records.shape[1]
    cmax = shard_range(total, 0, world)[1]
    buf = torch.zeros((cmax, L), dtype=torch.float64, device=device)
    if records.shape[0]:
        buf[:records.shape[0]] = torch.from_numpy(np.ascontiguousarray(records)).to(buf.device)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    if rank != 0:
        return None
    out = [parts[r][:shard_range(total, r, world)[1]].cpu().numpy() for r in range(world)]
    return np.concatenate(out, axis=0)


def _world():
    """(world, rank, dist-or-None) of the default torch.distributed group; a
    process without one is a world of one."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(), dist.get_rank(), dist
    except ImportError:
        pass
    return 1, 0, None


def _count_ready(flag: bool) -> int:
    """How many ranks of the default group set ``flag`` (one all_reduce of a
    scalar; 0/1 without a group).  Every rank calls it at the same point, so
    every rank learns the same count and takes the same branch after it."""
    world, _, dist = _world()
    if dist is None:
        return int(bool(flag))
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(t)
    return int(t.item())


class GatherSetupError(RuntimeError):
    """The RCCL gather could not be set up on every rank; every rank raises it
    at the same point (the readiness counts are agreed), so no rank is left
    inside a collective its peers never enter."""


class RCCLRecordGather:
    """The gather as the C-ABI's RCCL collective (gpmpc_comm_* /
    gpmpc_gather_results): one ncclGather over xGMI straight from
    the device record arrays (Fleet.records_dev, Rollouts6.records_dev).

    The communicator spans the ranks of the default torch.distributed group
    (one process per GPU); rank 0's ncclUniqueId reaches the others through
    that group.  Without a process group it is a world of one.

    Set-up is agreed before and after ncclCommInitRank: a rank whose local
    preparation failed (no context, RCCL not loadable, no unique id on rank 0)
    still takes part in the id broadcast and the readiness count, so every rank
    raises GatherSetupError together instead of some blocking in the
    communicator's bootstrap.  ``nranks`` is what RCCL's communicator reports
    (gpmpc_comm_count), not what was asked for."""

    def __init__(self, ctx, _fail_local=False):
        import ctypes

        from . import _lib
        self._lib, self.ctx, self.h = _lib, ctx, None
        world, rank, dist = _world()
        self.world, self.rank = world, rank
        err = None
        if ctx is None or getattr(ctx, "h", None) is None:
            err = "no device context on this rank"
        elif _fail_local:
            err = "local set-up failure (injected)"
        uid = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
        raw = uid.raw
        if rank == 0 and err is None:
            try:
                _lib._chk(_lib._L.gpmpc_comm_unique_id(uid), "comm_unique_id")
                raw = uid.raw
            except Exception as e:  # noqa: BLE001  (reported to every rank below)
                err = str(e)
        if world > 1:
            box = [(raw, err if rank == 0 else None)]
            dist.broadcast_object_list(box, src=0)   # every rank, even after a failure
            raw, root_err = box[0]
            if root_err and err is None:
                err = f"rank 0: {root_err}"
        ready = _count_ready(err is None)
        if ready < world:
            raise GatherSetupError(f"RCCL gather not set up: {world - ready} of {world} ranks not ready"
                                   + (f" (this rank: {err})" if err else ""))
        h = _lib._vp()
        rc = _lib._L.gpmpc_comm_init(ctx.h, raw, world, rank, ctypes.byref(h))
        init_err = None if rc == 0 else _lib._L.gpmpc_last_error().decode(errors="replace")
        ready = _count_ready(init_err is None)
        if init_err is None:
            self.h = h
        if ready < world:
            self.close()
            raise GatherSetupError(f"ncclCommInitRank failed on {world - ready} of {world} ranks"
                                   + (f" (this rank: {init_err})" if init_err else ""))
        n = ctypes.c_int(0)
        _lib._chk(_lib._L.gpmpc_comm_count(self.h, ctypes.byref(n)), "comm_count")
        self.nranks = int(n.value)

    def _counts(self, total):
        return np.array([shard_range(total, r, self.world)[1] for r in range(self.world)], np.int32)

    def prepare(self, d_records, total: int, root: int = 0):
        """The local half (gpmpc_gather_prepare): argument checks, buffers, the
        device padding of this rank's block.  Raises on this rank's failure."""
        lib = self._lib
        self._root = int(root)
        lib._chk(lib._L.gpmpc_gather_prepare(self.ctx.h, self.h, d_records, lib._i(self._counts(total)),
                                             int(root)), "gather_prepare")

    def collective(self, total: int, root: int = 0):
        """The ncclGather itself (gpmpc_gather_collective), after every rank's prepare
        succeeded.  Returns the (total, REC_LEN) records on the root, None elsewhere."""
        lib = self._lib
        out = np.empty((int(total), lib.REC_LEN)) if self.rank == root else None
        lib._chk(lib._L.gpmpc_gather_collective(self.ctx.h, self.h, lib._i(self._counts(total)), int(root),
                                                lib._d(out) if out is not None else None), "gather_collective")
        return out

    def gather(self, d_records, total: int, root: int = 0):
        """prepare + collective without an agreement in between (a world of one,
        or a caller that has agreed by other means)."""
        self.prepare(d_records, total, root)
        return self.collective(total, root)

    def close(self):
        if getattr(self, "h", None):
            self._lib._L.gpmpc_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GatherCollectiveError(RuntimeError):
    """The ncclGather failed after every rank had prepared its block.  Peers may
    be inside the collective or past it, so there is no agreed way back: the
    caller must treat this as fatal (exit non-zero)."""


def gather_shard_records(ctx, d_records, host_records, total: int, path: str | None = None,
                         device=None, _fail_local=False, _gather=None):
    """The one collective of the path, with a record of what ran.

    path "rccl" (default, or GPMPC_GATHER): the C-ABI's ncclGather of the device
    record arrays, in three agreed stages.  (1) Set-up (communicator): if it
    fails on any rank every rank knows it (RCCLRecordGather's readiness counts).
    (2) prepare (gpmpc_gather_prepare: buffers, padding -- everything a rank can
    fail alone): one readiness count after it on every rank.  If either stage
    failed anywhere, all ranks fall back together to torch.distributed.gather of
    the host records, and only then destroy the communicator.  (3) The collective
    itself: a failure there is fatal (GatherCollectiveError), because a peer may
    already be inside it or past it.  path "torch": torch.distributed.gather
    directly.

    Returns (records on rank 0 / None elsewhere, info) with info =
    {"path": "rccl" | "torch", "nranks": ranks the collective spanned (RCCL's
    communicator count, or the process group's size), "records": rows gathered
    on rank 0 (0 elsewhere), "requested": path, "fallback": reason or None}.
    ``_gather``: a factory standing in for RCCLRecordGather (tests)."""
    path = path or os.environ.get("GPMPC_GATHER", "rccl")
    world, rank, dist = _world()
    info = {"path": None, "nranks": None, "records": 0, "requested": path, "fallback": None}
    if path == "rccl":
        g = None
        try:
            g = (_gather or RCCLRecordGather)(ctx, _fail_local=_fail_local)
        except GatherSetupError as e:
            info["fallback"] = str(e)
        if g is not None:
            err = None
            try:
                g.prepare(d_records, total)
            except Exception as e:  # noqa: BLE001  (agreed below)
                err = str(e)
            ready = _count_ready(err is None)
            if ready == world:
                try:
                    out = g.collective(total)
                except Exception as e:  # noqa: BLE001
                    raise GatherCollectiveError(f"ncclGather failed on rank {rank}: {e}") from e
                nr = g.nranks
                g.close()
                info.update(path="rccl", nranks=nr, records=0 if out is None else int(out.shape[0]))
                return out, info
            g.close()   # every rank skips the collective: the communicator is idle everywhere
            info["fallback"] = (f"gather prepare failed on {world - ready} of {world} ranks"
                                + (f" (this rank: {err})" if err else ""))
    elif path != "torch":
        raise ValueError(f"unknown gather path {path!r} (rccl or torch)")
    if dist is None:
        out = np.ascontiguousarray(host_records)
    else:
        out = gather_records(host_records, total, device=device)
    info.update(path="torch", nranks=world, records=0 if out is None else int(out.shape[0]))
    return out, info
