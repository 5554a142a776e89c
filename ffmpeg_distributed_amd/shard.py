"""Segment sharding across GPUs: segments share no state, so N ranks split
the segment list with no data-path collective.  The reference hands segments out by
dynamic pull from one queue (ffmpeg_distributed.py:127,185-192); the dispatcher keeps
that for `-H gpu:N` workers, while the benchmark uses this fixed round-robin split so
every rank's work is known up front (weak scaling: equal segments per rank).

The process group is used only for bookkeeping: a barrier around the timed region and
a MAX reduction of the elapsed time (the slowest rank defines the job time).
"""
from __future__ import annotations

import time
from typing import Callable, List, Optional


def segments_for_rank(n_segments: int, rank: int, world: int) -> List[int]:
    """Round-robin: segment g goes to rank g % world."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} of {world}")
    return list(range(rank, n_segments, world))


def timed_region(step: Callable[[int], None], warmup: int, steps: int,
                 barrier: Callable[[], None], sync: Callable[[], None],
                 before_timing: Optional[Callable[[], None]] = None) -> float:
    """W untimed steps, then exactly K steps bracketed by barrier + device sync on both
    sides; returns this rank's wall time of the K steps in seconds."""
    for s in range(warmup):
        step(s)
    if before_timing:
        before_timing()
    barrier()
    sync()
    t0 = time.perf_counter()
    for s in range(steps):
        step(warmup + s)
    sync()
    barrier()
    return time.perf_counter() - t0


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """MAX of a per-rank float over the default process group (identity when single)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
