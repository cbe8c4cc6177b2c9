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


class RCCLRecordGather:
    """The gather as the C-ABI's RCCL collective (gpmpc_comm_* /
    gpmpc_gather_results): one ncclGather over xGMI straight from
    the device record arrays (Fleet.records_dev, Rollouts6.records_dev).

    The communicator spans the ranks of the default torch.distributed group
    (one process per GPU); rank 0's ncclUniqueId reaches the others through
    that group.  Without a process group it is a world of one."""

    def __init__(self, ctx):
        import ctypes

        from . import _lib
        self._lib, self.ctx = _lib, ctx
        world, rank = 1, 0
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                world, rank = dist.get_world_size(), dist.get_rank()
        except ImportError:
            dist = None
        self.world, self.rank = world, rank
        uid = ctypes.create_string_buffer(128)
        if rank == 0:
            _lib._chk(_lib._L.gpmpc_comm_unique_id(uid), "comm_unique_id")
        raw = uid.raw
        if world > 1:
            box = [raw]
            dist.broadcast_object_list(box, src=0)
            raw = box[0]
        h = _lib._vp()
        _lib._chk(_lib._L.gpmpc_comm_init(ctx.h, raw, world, rank, ctypes.byref(h)), "comm_init")
        self.h = h

    def gather(self, d_records, total: int, root: int = 0):
        """d_records: this rank's device record pointer (shard_range(total, rank, world)
        rows).  Returns the (total, REC_LEN) records on the root, None elsewhere."""
        lib = self._lib
        counts = np.array([shard_range(total, r, self.world)[1] for r in range(self.world)], np.int32)
        out = np.empty((int(total), lib.REC_LEN)) if self.rank == root else None
        lib._chk(lib._L.gpmpc_gather_results(self.ctx.h, self.h, d_records, lib._i(counts), int(root),
                                             lib._d(out) if out is not None else None), "gather_results")
        return out

    def close(self):
        if getattr(self, "h", None):
            self._lib._L.gpmpc_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
