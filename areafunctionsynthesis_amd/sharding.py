"""Utterance sharding for one process per GPU (bench.py, batch jobs).

Utterances are independent, so the batch is split into contiguous per-rank blocks with no
data-path collective; each rank builds exactly the rows the full batch would give it
(workloads.* take ``first_utterance``; seeds are u + 1 for the global index u, so audio is
independent of the GPU count).  The only collective is the gather of the audio to rank 0:
on GPUs the library's own RCCL gather (``afs_gather_pcm`` through :class:`CommTransport`), in
the CPU tests torch's gloo gather (:class:`TorchTransport`) -- :class:`PcmGather` is the same
code over either.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple


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


class CommTransport:
    """The library's RCCL gather (afs_gather_pcm): runs on the comm's own stream behind the
    conversion, so the next synthesis overlaps it; ``fence`` orders later writes of the
    buffers after it on the synthesis stream (no host wait)."""

    def __init__(self, comm):
        self.comm = comm

    def gather(self, slot, local, root):
        self.comm.gather_pcm(local.view(-1), root.view(-1) if root is not None else None)

    def fence(self, slot):
        self.comm.fence()

    def drain(self):
        self.comm.synchronize()


class TorchTransport:
    """torch.distributed gather into rank 0's root buffer (gloo in the CPU tests; the
    collective moves raw bytes, gloo has no int16 collectives)."""

    def __init__(self, dist, world: int, rank: int):
        self.dist, self.world, self.rank = dist, world, rank
        self.work = {}

    def gather(self, slot, local, root):
        import torch
        recv = None
        if self.rank == 0:
            recv = [r.view(-1).view(torch.uint8) for r in root.view(self.world, -1)]
        self.work[slot] = self.dist.gather(local.view(-1).view(torch.uint8), gather_list=recv, dst=0, async_op=True)

    def fence(self, slot):
        w = self.work.pop(slot, None)
        if w is not None:
            w.wait()

    def drain(self):
        for slot in list(self.work):
            self.fence(slot)


class StagedTorchTransport:
    """Test transport for bench.py's multi-process path on one GPU (``--gather-transport gloo``):
    each rank's int16 block goes through torch.distributed (gloo) on the host and lands in rank 0's
    device root buffer.  It exercises every step of the path except RCCL itself (which
    :class:`CommTransport` drives and tests/test_multi_gpu.py covers with one rank)."""

    def __init__(self, dist, world: int, rank: int):
        self.dist, self.world, self.rank = dist, world, rank

    def gather(self, slot, local, root):
        import torch
        cpu = local.detach().to("cpu").contiguous().view(-1).view(torch.uint8)
        recv = [torch.empty_like(cpu) for _ in range(self.world)] if self.rank == 0 else None
        self.dist.gather(cpu, gather_list=recv, dst=0)
        if self.rank == 0:
            root.view(-1).view(torch.uint8).copy_(torch.cat(recv).to(root.device))

    def fence(self, slot):
        pass

    def drain(self):
        pass


class PcmGather:
    """int16 audio of each step gathered to rank 0 while the next step synthesizes.

    ``submit(samples)`` converts the step's float audio to the reference's int16 format
    (``convert(samples, out)``, i.e. ``Context.to_int16`` on the synthesis stream) into one of
    ``depth`` rotating buffers and starts the gather of it into rank 0's root buffer of the
    same slot ([world][B][T], rank order = utterance order).  A buffer is rewritten only after
    its previous gather completed (``transport.fence``).  int16 quarters the bytes that cross
    xGMI compared with gathering the float64 output.
    """

    def __init__(self, convert, shape, world: int, rank: int, transport, device=None, depth: int = 2):
        import torch
        self.convert, self.world, self.rank, self.transport = convert, world, rank, transport
        self.bufs = [torch.empty(tuple(shape), dtype=torch.int16, device=device) for _ in range(depth)]
        self.roots = [torch.empty((world,) + tuple(shape), dtype=torch.int16, device=device)
                      if (rank == 0 and world > 1) else None for _ in range(depth)]
        self.k = 0

    def submit(self, samples):
        slot = self.k % len(self.bufs)
        self.k += 1
        self.transport.fence(slot)
        self.convert(samples, self.bufs[slot])
        self.transport.gather(slot, self.bufs[slot], self.roots[slot])
        return slot

    def result(self, slot):
        """Rank 0: the gathered [world, B, T] int16 audio of ``slot`` (after :meth:`drain`)."""
        return self.roots[slot] if self.world > 1 else self.bufs[slot][None]

    def drain(self):
        self.transport.drain()


def edge_utterances(world: int, per_rank: int) -> List[Tuple[int, int, int]]:
    """(rank, row in the rank's block, global utterance index) of the first and the last utterance
    of every rank's block: the rows :func:`check_gathered` verifies."""
    rows = sorted({0, per_rank - 1}) if per_rank > 0 else []
    return [(r, j, r * per_rank + j) for r in range(world) for j in rows]


def check_gathered(rows, world: int, per_rank: int, reference: Callable[[Sequence[int]], "object"]) -> dict:
    """Rank 0: the gathered int16 audio against the same utterances synthesized on rank 0 alone.

    ``rows[i]`` is the gathered row of the i-th entry of :func:`edge_utterances` (``[n, T]``
    int16, any array type with ``numpy()`` or an ndarray); ``reference(us)`` synthesizes the
    global utterances ``us`` (frames of index u, seed u + 1) in one call on rank 0 and returns their
    int16 audio ``[len(us), T]`` -- with the lane width the shards ran (the tree kernel's 16- and
    64-lane builds agree within the parity tolerances, not bit for bit; bench.py passes the
    shard's width, afs_multi_synthesize fixes one width for the whole batch).  At that width an
    utterance's audio does not depend on its batch-mates or slot, so any difference in the
    bit-for-bit comparison is a gather (or sharding) fault."""
    import numpy as np
    edges = edge_utterances(world, per_rank)
    got = rows.numpy() if hasattr(rows, "numpy") else np.asarray(rows)
    ref = np.asarray(reference([u for _, _, u in edges]))
    bad = []
    for i, (r, j, u) in enumerate(edges):
        d = int(np.count_nonzero(got[i] != ref[i])) if got[i].shape == ref[i].shape else -1
        if d != 0:
            bad.append({"utterance": u, "rank": r, "row": j, "differing_samples": d})
    return {"utterances_checked": [u for _, _, u in edges], "bitwise_equal": not bad and len(edges) > 0,
            "mismatches": bad,
            "method": "rank 0 re-synthesizes the first and last utterance of every rank's block alone "
                      "(global frames and seeds u + 1) and compares the int16 rows it received bit for bit"}
