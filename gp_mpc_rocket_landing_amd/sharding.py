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
