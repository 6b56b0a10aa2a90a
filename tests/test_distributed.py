"""Pair sharding + gather to rank 0 (stereo_matching_amd/distributed.py) with
world_size 2 (and 8, config 4's batch) on the gloo backend (CPU).  Each rank computes its pairs with the
oracle (test infrastructure) on tiny synthetic pairs; rank 0 checks the
gathered batch against a single-process run."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stereo_matching_amd import distributed, synthetic

H, W, D, N = 24, 80, 32, 5


def _pairs(n=N):
    return [synthetic.stereo_pair(H, W, D, pair_index=i) for i in range(n)]


def _compute(pair):
    import oracle
    return torch.from_numpy(oracle.process(pair[0], pair[1], D, views=1)["sub"])


_CALLS = []


def _counting_compute(pair):
    _CALLS.append(1)
    return _compute(pair)


def _worker(rank, world, port, q, n=N):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = distributed.process_batch(_pairs(n), _counting_compute, (H, W))
        # a rank computes exactly its shard: no extra frame to learn the shape
        assert len(_CALLS) == len(distributed.shard(n, rank, world)), (rank, len(_CALLS))
        q.put((rank, None if out is None else out.numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_round_robin():
    assert distributed.shard(8, 3, 8) == [3]
    assert distributed.shard(5, 0, 2) == [0, 2, 4]
    assert distributed.shard(5, 1, 2) == [1, 3]
    assert sorted(i for r in range(3) for i in distributed.shard(7, r, 3)) == list(range(7))
    with pytest.raises(ValueError):
        distributed.shard(4, 2, 2)


@pytest.mark.parametrize("n", [N, 1, 0])
def test_gather_world2_gloo(n):
    # n = 1: rank 1 holds no pair and sends an empty stack of the right kind;
    # n = 0: nothing to gather, rank 0 gets a 0 x H x W batch
    import oracle
    oracle.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, n)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None
    assert res[0].shape == (n, H, W) and res[0].dtype == np.float32
    if n:
        want = np.stack([_compute(p).numpy() for p in _pairs(n)])
        assert np.array_equal(res[0].view(np.uint32), want.view(np.uint32))


def test_config4_batch_of_8_world8_gloo():
    # BASELINE config 4's shape: a batch of 8 pairs, one per rank on 8 ranks,
    # maps gathered to rank 0 in pair order (the RCCL path carries the same
    # calls; 8-GPU runs are the driver's)
    import oracle
    oracle.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 8, port, q, 8)) for r in range(8)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res[r] is None for r in range(1, 8))
    want = np.stack([_compute(p).numpy() for p in _pairs(8)])
    assert res[0].shape == (8, H, W)
    assert np.array_equal(res[0].view(np.uint32), want.view(np.uint32))


def _pipe_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pipe = distributed.PipelinedGather((3, 4), torch.float32, "cpu", depth=2)
        seen = {}
        for k in range(5):
            buf = pipe.buffer()            # waits for the gather of step k-2
            if k >= 2:
                pipe.verify()              # collective: every rank's frames so far are valid
            if k >= 2 and rank == 0:       # step k-2's maps are complete now
                seen[k - 2] = [t.clone().numpy() for t in pipe.gathered(k - 2)]
            buf.fill_(100 * rank + k)      # "compute" step k into the buffer
            pipe.submit()
        pipe.drain()
        if rank == 0:
            for k in (3, 4):
                seen[k] = [t.clone().numpy() for t in pipe.gathered(k)]
        q.put((rank, seen))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_pipelined_gather_gloo(world):
    # bench.py's overlapped per-step gather: every step's maps reach rank 0
    # intact although the next step already writes the other buffer
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(res[0]) == [0, 1, 2, 3, 4]
    for k, maps in res[0].items():
        assert len(maps) == world
        for r in range(world):
            assert (maps[r] == 100 * r + k).all(), (k, r)


class _OracleView:
    """Stands in for an SGM view handle on CPU: the oracle's left or right
    sub-pixel map written through the data pointers ViewSplit passes."""

    def __init__(self, view):
        self.view = view

    @staticmethod
    def _at(ptr, ctype, shape):
        import ctypes
        n = int(np.prod(shape))
        return np.ctypeslib.as_array((ctype * n).from_address(ptr)).reshape(shape)

    def process_device(self, d_left, d_right, d_out, stream=0):
        import ctypes
        import oracle
        left = self._at(d_left, ctypes.c_uint8, (H, W)).copy()
        right = self._at(d_right, ctypes.c_uint8, (H, W)).copy()
        ref = oracle.process(left, right, D)
        self._at(d_out, ctypes.c_float, (H, W))[:] = ref["sub_beta" if self.view else "sub"]

    def lr_check_device(self, d_fl, d_fr, d_out, stream=0):
        import ctypes
        import pyref
        fl = self._at(d_fl, ctypes.c_float, (H, W)).copy()
        fr = self._at(d_fr, ctypes.c_float, (H, W)).copy()
        self._at(d_out, ctypes.c_float, (H, W))[:] = pyref.lr_check(fl, fr, D)


def _split_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        team = distributed.ViewSplit(_OracleView(rank % 2), H, W, "cpu")
        left, right = (torch.from_numpy(a) for a in synthetic.stereo_pair(H, W, D, rank // 2))
        out = team.step(left.data_ptr(), right.data_ptr())
        q.put((rank, None if out is None else out.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_view_split_world4_gloo():
    # two teams of (left view, right view): each even rank ends with the LR-
    # checked map of its team's pair, built from the partner's F_R
    import oracle
    oracle.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None and res[3] is None
    for team in range(2):
        ref = oracle.process(*synthetic.stereo_pair(H, W, D, team), D)
        assert np.array_equal(res[2 * team].view(np.uint32), ref["lr"].view(np.uint32)), team


def _bad_compute(pair):
    # rank 1's pairs come back with the wrong shape
    m = _compute(pair)
    return m[:-1] if dist.get_rank() == 1 else m


def _err_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        try:
            distributed.process_batch(_pairs(4), _bad_compute, (H, W))
            q.put((rank, "no error"))
        except ValueError as e:
            q.put((rank, f"ValueError: {e}"))
        except RuntimeError as e:
            q.put((rank, f"RuntimeError: {e}"))
    finally:
        dist.destroy_process_group()


def test_process_batch_error_reaches_every_rank():
    # a bad map on one rank must not leave the others blocked in
    # the gather -- the ranks agree on the failure first and all raise
    import oracle
    oracle.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_err_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1].startswith("ValueError") and "expected" in res[1]
    assert res[0].startswith("RuntimeError") and "another rank" in res[0]

