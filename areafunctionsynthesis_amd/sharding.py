"""Utterance sharding for one process per GPU (bench.py, batch jobs).

Utterances are independent, so the batch is split into contiguous per-rank blocks with no
data-path collective; each rank builds exactly the rows the full batch would give it
(workloads.* take ``first_utterance``; seeds are u + 1 for the global index u, so audio is
independent of the GPU count).  The only collective is the gather of the audio to rank 0
(RCCL ``gather`` on the GPU, gloo in the CPU tests).
"""
from __future__ import annotations

from typing import List, Optional, Tuple


def shard_range(rank: int, world: int, per_rank: int) -> Tuple[int, int]:
    """First global utterance index and count of ``rank``'s block (weak scaling)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    return rank * per_rank, per_rank


def gather_to_rank0(t, world: int, rank: int, dist) -> Optional[List]:
    """Gather equally shaped per-rank tensors to rank 0 (rank order); None elsewhere."""
    if world == 1:
        return [t]
    bufs = [t.new_empty(t.shape) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gather_list=bufs, dst=0)
    return bufs
