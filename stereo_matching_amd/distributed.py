"""Pair-sharded multi-GPU driver.

Stereo pairs are independent, so a batch shards one pair per rank with no
data-path collective; the only exchange is the final gather of the disparity
maps to rank 0 (RCCL over xGMI with backend "nccl", gloo on CPU for tests).
One process per GPU, launched by torch.distributed.run.  Within one pair the
path is serial across the image (IIR filters, scanline DPs): replicas only.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch
import torch.distributed as dist


def shard(n_items: int, rank: int, world: int) -> list[int]:
    """Indices of the items rank `rank` owns: round-robin, so with n_items ==
    world every rank gets exactly one pair (config 4: 8 pairs on 8 GPUs)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return list(range(rank, n_items, world))


def gather_maps(local: torch.Tensor, n_items: int, group=None) -> torch.Tensor | None:
    """Gathers every rank's stack of maps (k_r x H x W, k_r = len(shard(...)))
    to rank 0 and returns the n_items x H x W batch in item order there (None
    on other ranks).  Ranks holding fewer items pad with a zero map so one
    fixed-size gather serves uneven batches."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = (n_items + world - 1) // world
    h, w = local.shape[-2:]
    send = torch.zeros((per, h, w), dtype=local.dtype, device=local.device)
    if local.shape[0]:
        send[: local.shape[0]] = local
    recv = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send, gather_list=recv, dst=0, group=group)
    if rank != 0:
        return None
    out = torch.empty((n_items, h, w), dtype=local.dtype, device=local.device)
    for r in range(world):
        for k, item in enumerate(shard(n_items, r, world)):
            out[item] = recv[r][k]
    return out


def process_batch(pairs: Sequence, compute: Callable[[object], torch.Tensor], group=None):
    """Runs `compute(pair) -> H x W map` on this rank's shard of `pairs` and
    gathers the maps to rank 0 (returned there, None elsewhere)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mine = [compute(pairs[i]) for i in shard(len(pairs), rank, world)]
    if mine:
        local = torch.stack(mine)
    else:
        h, w = compute(pairs[0]).shape  # shape only; no rank holds zero pairs when n >= world
        local = torch.empty((0, h, w))
    return gather_maps(local, len(pairs), group)


class PipelinedGather:
    """Per-step gather of a rank's map to rank 0, overlapped with the next
    steps' compute.  Steps write into `buffer()` (one of `depth` rotating
    maps), then call `submit()`, which enqueues an asynchronous gather of that
    map (RCCL over xGMI: its stream waits for the map's producer, nothing
    waits for it); a buffer's previous gather is only waited for when the
    buffer comes round again, and `drain()` waits for all of them.  With
    depth 2 the gather of step k runs under the kernels of step k+1."""

    def __init__(self, shape, dtype, device, depth: int = 2, group=None):
        self.group = group
        self.depth = depth
        world = dist.get_world_size(group)
        self.root = dist.get_rank(group) == 0
        self.bufs = [torch.empty(shape, dtype=dtype, device=device) for _ in range(depth)]
        self.recv = [[torch.empty(shape, dtype=dtype, device=device) for _ in range(world)]
                     if self.root else None for _ in range(depth)]
        self.work = [None] * depth
        self.k = 0

    def buffer(self) -> torch.Tensor:
        i = self.k % self.depth
        if self.work[i] is not None:
            self.work[i].wait()
            self.work[i] = None
        return self.bufs[i]

    def submit(self) -> None:
        i = self.k % self.depth
        self.work[i] = dist.gather(self.bufs[i], gather_list=self.recv[i], dst=0, group=self.group,
                                   async_op=True)
        self.k += 1

    def drain(self) -> None:
        for i, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[i] = None

    def gathered(self, step: int):
        """Rank 0: the maps of `step` (valid after drain() and while fewer than
        `depth` later steps have been submitted); None elsewhere."""
        return None if not self.root else self.recv[step % self.depth]
