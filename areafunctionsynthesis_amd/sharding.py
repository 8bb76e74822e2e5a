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


class PcmGather:
    """int16 audio of each step gathered to rank 0 while the next step synthesizes.

    ``submit(samples)`` converts the step's float audio to the reference's int16 format
    (``convert(samples, out)``, i.e. ``Context.to_int16`` on the synthesis stream) into one
    of ``depth`` rotating buffers and starts an asynchronous gather of it; the collective runs
    on the process group's own stream, so the next step's kernels are not queued behind it.
    A buffer is reused only after its previous gather completed.  int16 quarters the bytes
    that cross xGMI compared with gathering the float64 output.
    """

    def __init__(self, convert, shape, world: int, rank: int, dist, device=None, depth: int = 2):
        import torch
        self.convert, self.world, self.rank, self.dist = convert, world, rank, dist
        self.bufs = [torch.empty(tuple(shape), dtype=torch.int16, device=device) for _ in range(depth)]
        # the collective moves raw bytes (gloo has no int16 collectives; RCCL does not care)
        self.recv = [[torch.empty_like(b) for _ in range(world)] if (rank == 0 and world > 1) else None
                     for b in self.bufs]
        self.work = [None] * depth
        self.k = 0

    def submit(self, samples):
        import torch
        slot = self.k % len(self.bufs)
        self.k += 1
        if self.work[slot] is not None:
            self.work[slot].wait()
            self.work[slot] = None
        self.convert(samples, self.bufs[slot])
        if self.world > 1:
            recv = [r.view(-1).view(torch.uint8) for r in self.recv[slot]] if self.recv[slot] else None
            self.work[slot] = self.dist.gather(self.bufs[slot].view(-1).view(torch.uint8), gather_list=recv,
                                               dst=0, async_op=True)
        return slot

    def result(self, slot):
        """Rank 0: the gathered [world] list of int16 shards of ``slot`` (after :meth:`drain`)."""
        return self.recv[slot] if self.world > 1 else [self.bufs[slot]]

    def drain(self):
        for i, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[i] = None
