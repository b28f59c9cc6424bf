"""Frame-parallel batch mode (BASELINE config 4).

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on the
MI355X node).  Rectified pairs are independent units: frame i of the global
batch lives on rank i // frames_per_rank and is generated / computed there; no
collective touches the data path until the final gather of the int16 maps to
the destination rank, the only exchange step of the reference's pipeline.

The per-rank compute is injected (``compute(L, R, out)``), so the same driver
runs the HIP path in bench.py and the CPU oracle in the world_size-2 gloo test.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

SEED0 = 0x5EED0000


def frame_seeds(rank: int, world: int, frames_per_rank: int, seed0: int = SEED0) -> List[int]:
    """Seeds of the frames owned by ``rank`` (contiguous block of the global batch)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return [seed0 + rank * frames_per_rank + j for j in range(frames_per_rank)]


def global_frame_index(rank: int, j: int, frames_per_rank: int) -> int:
    return rank * frames_per_rank + j


def gather_frames(out, rank: int, world: int, dst: int = 0, collective: bool = False) -> Optional[list]:
    """Gather every rank's (F, H, W) int16 block on ``dst`` (list indexed by rank).
    ``collective``: run the collective even for one rank (tests of the RCCL call)."""
    if world == 1 and not collective:
        return [out]
    import torch
    import torch.distributed as dist
    # int16 maps travel as bytes: neither gloo nor RCCL/NCCL has an int16 type
    raw = out.contiguous().view(torch.uint8)
    buf = [torch.empty_like(raw) for _ in range(world)] if rank == dst else None
    dist.gather(raw, buf, dst=dst)
    return [b.view(out.dtype) for b in buf] if buf is not None else None


class FrameBatch:
    """Holds one rank's frames and runs compute + gather per step."""

    def __init__(self, left, right, out, compute: Callable, rank: int = 0, world: int = 1,
                 gather: bool = True, dst: int = 0, collective: bool = False):
        """``collective``: gather through the process group even for one rank
        (bench.py --force-gather runs the multi-rank code path on one GPU)."""
        self.left, self.right, self.out = left, right, out
        self.compute = compute
        self.rank, self.world, self.dst = rank, world, dst
        self.collective = collective
        self.gather = gather and (world > 1 or collective)
        self.gathered: Optional[Sequence] = None

    def step(self):
        self.compute(self.left, self.right, self.out)
        if self.gather:
            self.gathered = gather_frames(self.out, self.rank, self.world, self.dst, self.collective)
        return self.gathered


class InflightBatches:
    """Consecutive steps of a FrameBatch-style workload with up to ``n`` batches in
    flight: step k runs on slot k % n -- its own HIP stream, its own mvsv context
    (cached volumes) and its own output buffer -- so the kernels of consecutive
    independent batches overlap on the GPU (the serving shape of the
    frame-parallel batch mode; every step still computes its whole batch).
    ``compute(L, R, out)`` is called inside the slot's stream and context; the
    gather (world > 1 or ``collective``) follows it on the same stream, in step
    order on every rank.

    Synchronisation contract: step() makes the slot wait for the caller's
    current stream (inputs written there are ready), but the caller's stream
    does NOT wait for the slot.  Before reading ``last_out`` / ``gathered`` or
    writing new data into ``left`` / ``right`` on the caller's stream, call
    join() (or synchronize the device); the input and output tensors are
    recorded on the slot streams, so dropping the last reference to one of
    them never hands its memory to another allocation while a slot still uses
    it."""

    def __init__(self, left, right, make_out, compute: Callable, n: int, device, rank: int = 0,
                 world: int = 1, gather: bool = True, dst: int = 0, collective: bool = False):
        import torch
        from ._lib import Context
        self.left, self.right, self.compute = left, right, compute
        self.rank, self.world, self.dst, self.collective = rank, world, dst, collective
        self.gather = gather and (world > 1 or collective)
        dev = torch.device(device)
        self.slots = [(torch.cuda.Stream(dev), Context(dev.index or 0), make_out()) for _ in range(n)]
        self.k = 0
        self.gathered: Optional[Sequence] = None
        self.last_out = None

    def step(self):
        import torch
        from ._lib import use_context
        stream, ctx, out = self.slots[self.k % len(self.slots)]
        self.k += 1
        stream.wait_stream(torch.cuda.current_stream(stream.device))  # inputs ready
        for t in (self.left, self.right, out):
            t.record_stream(stream)  # the allocator keeps them alive for this slot
        with torch.cuda.stream(stream), use_context(ctx):
            self.compute(self.left, self.right, out)
            if self.gather:
                self.gathered = gather_frames(out, self.rank, self.world, self.dst, self.collective)
        self.last_out = out
        return self.gathered

    def contexts(self):
        return [c for _, c, _ in self.slots]

    def join(self):
        """Make the caller's current stream wait for every slot: required before
        reading a step's results or refilling the inputs on that stream."""
        import torch
        cur = torch.cuda.current_stream(self.slots[0][0].device)
        for s, _, _ in self.slots:
            cur.wait_stream(s)
