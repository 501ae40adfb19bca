"""Multi-GPU data path: one process per GPU, independent sequences.

Each sequence's recursion is independent, so a batch is split into contiguous slices,
one per rank, with the (tiny) parameters replicated; there is no collective inside the
recursion.  The only exchange is the optional gather of the per-sequence results to one
rank after compute (BASELINE config 4), done with torch.distributed (RCCL on ROCm for
GPU tensors, gloo for the CPU tests).
"""
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def batch_slice(B: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced slice [start, stop) of B sequences for `rank` of `world`
    (the first B % world ranks take one extra sequence)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(B, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard(x: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """This rank's slice of a (B, ...) batch."""
    s, e = batch_slice(x.shape[0], rank, world)
    return x[s:e]


def gather_batch(local: torch.Tensor, B: int, dst: int = 0, group=None) -> Optional[torch.Tensor]:
    """Reassemble per-rank slices (as produced by `shard`) into the full (B, ...) batch on
    rank `dst` (returns None elsewhere).  Slices are padded to the largest slice so a single
    gather moves them (one RCCL gather: point-to-point transfers into dst over xGMI)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [batch_slice(B, r, world) for r in range(world)]
    cap = max(e - s for s, e in sizes)
    if local.shape[0] != sizes[rank][1] - sizes[rank][0]:
        raise ValueError(f"rank {rank}: local batch {local.shape[0]} does not match its slice {sizes[rank]}")
    padded = local
    if local.shape[0] < cap:
        pad = local.new_zeros((cap - local.shape[0],) + tuple(local.shape[1:]))
        padded = torch.cat([local, pad], 0)
    padded = padded.contiguous()
    if rank == dst:
        bufs = [torch.empty_like(padded) for _ in range(world)]
        dist.gather(padded, bufs, dst=dst, group=group)
        return torch.cat([b[: e - s] for b, (s, e) in zip(bufs, sizes)], 0)
    dist.gather(padded, None, dst=dst, group=group)
    return None


class BatchGather:
    """The per-step gather of bench.py (BASELINE config 4): every rank holds equal slices
    (B per rank) of the same outputs; `dst` receives them into buffers allocated once, so a
    timed step allocates nothing.  One dist.gather per output (RCCL on ROCm: point-to-point
    transfers into dst over xGMI).  `full(i)` is output i's (world * B, ...) batch on dst."""

    def __init__(self, like: Sequence[torch.Tensor], dst: int = 0, group=None):
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dst, self.group = dst, group
        self.bufs: List[Optional[List[torch.Tensor]]] = [
            [torch.empty_like(t) for _ in range(self.world)] if self.rank == dst else None for t in like]

    def __call__(self, *tensors: torch.Tensor) -> None:
        for t, bufs in zip(tensors, self.bufs):
            dist.gather(t.contiguous(), bufs, dst=self.dst, group=self.group)

    def full(self, i: int) -> Optional[torch.Tensor]:
        return torch.cat(self.bufs[i], 0) if self.bufs[i] is not None else None
