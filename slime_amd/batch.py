"""Object partitioning across GPUs.

Objects are independent, so a batch is split into contiguous per-rank ranges
and every rank runs the hot path on its own GPU with no data exchange.  The
only cross-rank traffic is the control plane (barrier, max-over-ranks time),
carried by torch.distributed on the CPU (gloo).
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.distributed as dist


def partition(nobj: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, start+count) share of nobj objects for `rank`.

    The first nobj % world ranks get one extra object (C5: 64 objects over 8
    GPUs -> 8 each)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(nobj, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def max_over_ranks(values: Sequence[float]) -> list[float]:
    """Element-wise max across ranks (identity when not distributed)."""
    t = torch.tensor(list(values), dtype=torch.float64)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def barrier() -> None:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def gather_strings(s: str) -> list[str]:
    """One string from every rank, in rank order ([s] when not distributed)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        out: list = [None] * dist.get_world_size()
        dist.all_gather_object(out, s)
        return [str(x) for x in out]
    return [s]
