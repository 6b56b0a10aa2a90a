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
    fixed-size gather serves uneven batches.  Every rank's `local` must carry
    the same H x W, dtype and device type (a rank with no items passes an
    empty 0 x H x W stack of them); n_items == 0 gathers nothing."""
    if local.dim() != 3:
        raise ValueError(f"local must be a k x H x W stack, got shape {tuple(local.shape)}")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    h, w = local.shape[-2:]
    if n_items == 0:
        return torch.empty((0, h, w), dtype=local.dtype, device=local.device) if rank == 0 else None
    per = (n_items + world - 1) // world
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


def comm_device(group=None) -> torch.device:
    """Where a collective's buffers live: the current HIP device for RCCL
    (backend "nccl"), the host for gloo (which this module stages through)."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def agree(ok: bool, group=None) -> bool:
    """True on every rank iff `ok` is true on every rank (one small MAX
    all_reduce where the backend keeps its buffers)."""
    flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=comm_device(group))
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    return int(flag.item()) == 0


def process_batch(pairs: Sequence, compute: Callable[[object], torch.Tensor], map_shape,
                  *, dtype=torch.float32, device=None, group=None,
                  check: Callable[[], None] | None = None):
    """Runs `compute(pair) -> H x W map` on this rank's shard of `pairs` and
    gathers the maps to rank 0 (returned there, None elsewhere).

    `map_shape` (H, W) and `dtype` describe the maps `compute` returns (for an
    SGM handle: (rows, cols), float32).  The gather runs where the process
    group's backend needs its buffers (`device`, default `comm_device()`: the
    current GPU for RCCL, the host for gloo, so HIP maps are staged through
    host memory there); the batch comes back on that device.  A rank whose
    shard is empty (fewer pairs than ranks) sends a zero stack without
    computing a frame, so the gather's buffers agree on every rank.

    The maps `compute` returns must have been produced on torch's current
    stream (see PipelinedGather): the staging copy and the gather are
    ordered after that stream only.

    `check` (e.g. an SGM handle's `check`, sgm_check) runs after this rank's
    frames: it waits for them and raises if a frame's maps are invalid (a
    slanted-pass hand-off that gave up), so such a map is never gathered.

    Failures are agreed on before any gather: if `compute` or `check` raises,
    or `compute` returns a map of the wrong shape, on any rank, every rank
    raises (a rank that raised alone would leave the others blocked in the
    gather)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    h, w = map_shape
    dev = torch.device(device) if device is not None else comm_device(group)
    mine, err = [], None
    try:
        for i in shard(len(pairs), rank, world):
            m = compute(pairs[i])
            if tuple(m.shape) != (h, w):
                raise ValueError(f"compute returned a {tuple(m.shape)} map, expected {(h, w)}")
            mine.append(m)
        if check is not None and mine:
            check()
    except Exception as e:  # noqa: BLE001 -- re-raised below, on every rank
        err = e
    all_ok = agree(err is None, group)
    if err is not None:
        raise err
    if not all_ok:
        raise RuntimeError("process_batch: compute failed on another rank")
    if mine:
        local = torch.stack([m.to(device=dev, dtype=dtype) for m in mine])
    else:
        local = torch.empty((0, h, w), dtype=dtype, device=dev)
    return gather_maps(local, len(pairs), group)


class PipelinedGather:
    """Per-step gather of a rank's map to rank 0, overlapped with the next
    steps' compute.  Steps write into `buffer()` (one of `depth` rotating
    maps), then call `submit()`, which enqueues an asynchronous gather of that
    map (RCCL over xGMI: its stream waits for the map's producer, nothing
    waits for it); a buffer's previous gather is only waited for when the
    buffer comes round again, and `drain()` waits for all of them.  With
    depth 2 the gather of step k runs under the kernels of step k+1.

    With gloo and device maps (tests: several ranks sharing one GPU) each
    submit first copies the map to a host buffer and gathers that;
    `gathered()` then returns host tensors.

    Stream ordering: the gather (and the gloo path's host copy) is ordered
    after the map's producer only if that producer ran on torch's CURRENT
    stream.  Enqueue the frame with `process_device(..., stream=
    torch.cuda.current_stream().cuda_stream)`, or make the handle's own stream
    current (`torch.cuda.set_stream(torch.cuda.ExternalStream(sgm.stream))`,
    as bench.py does).  `process_device(stream=None)` alone runs on the
    handle's non-blocking stream, which torch's streams do not wait for.

    Validity: `check` (e.g. the producing handle's `check`, sgm_check) is
    called by `verify()` (and by `drain()` unless `verify=False`); a frame
    whose maps are invalid (a slanted-pass hand-off that gave up) makes every
    rank raise there.  `gathered()` returns only steps submitted before the
    last successful verification, so a timed-out frame is never handed out
    as valid.  The check is not made per submit: it waits for the frame,
    which would serialise the host with the GPU and take away the overlap
    this class exists for."""

    def __init__(self, shape, dtype, device, depth: int = 2, group=None,
                 check: Callable[[], None] | None = None):
        self.group = group
        self.check = check
        self.verified = 0  # steps [0, verified) passed verify()
        self.depth = depth
        world = dist.get_world_size(group)
        self.root = dist.get_rank(group) == 0
        device = torch.device(device)
        self.bufs = [torch.empty(shape, dtype=dtype, device=device) for _ in range(depth)]
        self.staged = dist.get_backend(group) != "nccl" and device.type != "cpu"
        cdev = torch.device("cpu") if self.staged else device
        self.host = [torch.empty(shape, dtype=dtype) for _ in range(depth)] if self.staged else None
        self.recv = [[torch.empty(shape, dtype=dtype, device=cdev) for _ in range(world)]
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
        send = self.bufs[i]
        if self.staged:
            self.host[i].copy_(send)
            send = self.host[i]
        self.work[i] = dist.gather(send, gather_list=self.recv[i], dst=0, group=self.group,
                                   async_op=True)
        self.k += 1

    def drain(self, verify: bool = True) -> None:
        for i, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[i] = None
        if verify:
            self.verify()

    def verify(self) -> None:
        """Collective: runs `check` on this rank and agrees on the result;
        raises on every rank if any rank's frames since the last verification
        are invalid."""
        err = None
        if self.check is not None:
            try:
                self.check()
            except Exception as e:  # noqa: BLE001 -- re-raised below, on every rank
                err = e
        ok = agree(err is None, self.group)
        if err is not None:
            raise err
        if not ok:
            raise RuntimeError("PipelinedGather: a frame on another rank is invalid")
        self.verified = self.k

    def gathered(self, step: int):
        """Rank 0: the maps of `step` (complete once buffer() has come round to
        its slot again, or after drain(), and while fewer than `depth` later
        steps have been submitted); None elsewhere.  Raises for a step that no
        successful verify() covers yet."""
        if step >= self.verified:
            raise RuntimeError(f"PipelinedGather: step {step} is not verified yet (drain() or verify())")
        return None if not self.root else self.recv[step % self.depth]


class ViewSplit:
    """One stereo pair over two GPUs (the optional
    split): ranks 2k and 2k+1 of `group` form a team.  The even rank computes
    the left view (SGM.cpp:32-445), the odd rank the right view (SGM.cpp:
    448-801, an `SGM(..., views=1, view="right")` handle); the odd rank sends
    its sub-pixel map F_R (rows x cols f32, 1.86 MB at K128) to the even rank
    -- RCCL point-to-point over xGMI with backend "nccl", staged through host
    memory with gloo -- and the even rank runs the LR check (SGM.cpp:803-818)
    and, as asked, post_filter and LKRefine on the map.

    `sgm` is this rank's handle (left view on even ranks, right view on odd
    ones); `device` the torch device its maps live on.  Latency per pair is
    one view plus the exchange instead of two views; throughput per GPU is
    the same or lower, which is why pair sharding stays the default."""

    def __init__(self, sgm, rows: int, cols: int, device, *, post_filter: bool = False,
                 lk_refine: bool = False, group=None):
        self.group = group
        rank = dist.get_rank(group)
        if dist.get_world_size(group) % 2:
            raise ValueError("ViewSplit needs an even number of ranks")
        self.role = rank % 2               # 0: left view + LR check, 1: right view
        self.partner = rank ^ 1
        self.partner_global = self.partner if group is None else \
            dist.get_global_rank(group, self.partner)
        self.sgm = sgm
        self.device = torch.device(device)
        self.post_filter, self.lk_refine = post_filter, lk_refine
        self.fr = torch.empty((rows, cols), dtype=torch.float32, device=self.device)
        self.staged = dist.get_backend(group) != "nccl" and self.device.type != "cpu"
        self.host = torch.empty((rows, cols), dtype=torch.float32) if self.staged else None

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0

    def step(self, d_left: int, d_right: int, out: torch.Tensor | None = None):
        """Processes the team's pair (device images at the handle's full size);
        on the even rank writes get_disp()'s map into `out` and returns it,
        on the odd rank returns None."""
        st = self._stream()
        if self.role == 1:
            self.sgm.process_device(d_left, d_right, self.fr.data_ptr(), stream=st)
            if self.staged:
                self.host.copy_(self.fr)
                dist.send(self.host, dst=self.partner_global, group=self.group)
            else:
                dist.send(self.fr, dst=self.partner_global, group=self.group)
            return None
        if out is None:
            out = torch.empty_like(self.fr)
        self.sgm.process_device(d_left, d_right, out.data_ptr(), stream=st)
        if self.staged:
            dist.recv(self.host, src=self.partner_global, group=self.group)
            self.fr.copy_(self.host)
        else:
            dist.recv(self.fr, src=self.partner_global, group=self.group)
        self.sgm.lr_check_device(out.data_ptr(), self.fr.data_ptr(), out.data_ptr(), stream=st)
        if self.post_filter:
            self.sgm.post_filter_device(out.data_ptr(), stream=st)
        if self.lk_refine:
            self.sgm.lk_refine_device(d_left, d_right, out.data_ptr(), stream=st)
        return out
