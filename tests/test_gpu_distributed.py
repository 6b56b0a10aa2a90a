"""The multi-GPU driver (stereo_matching_amd/distributed.py)
carrying HIP-computed disparity maps, on the one-GPU box:

* world 1 on the nccl backend (RCCL): process_batch with an SGM handle
  computing device maps, and PipelinedGather over 6 steps (bench.py's
  overlapped per-step gather) -- the code config 4 runs on 8 GPUs;
* two gloo ranks sharing cuda:0 with CUDA maps: process_batch over an uneven
  batch (maps staged through the host) and the staged PipelinedGather;
* bench.py itself under torch.distributed.run (world 1, nccl);
* config 4's batch of 8 K128 pairs on 8 gloo ranks sharing cuda:0, through
  process_batch and the batched PipelinedGather, every map bit-equal to the
  oracle's map for its pair.

Every gathered map must equal the map a single handle computes for that pair,
bit for bit.  Each case runs in fresh child processes (torch's HIP runtime
initialises before the library's, as in bench.py)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

COMMON = r"""
import os, sys, numpy as np, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from stereo_matching_amd import SGM, synthetic
from stereo_matching_amd import distributed as sd
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
H, W, D = 375, 1242, 128
PAIRS = [synthetic.stereo_pair(H, W, D, pair_index=i) for i in range(5)]

def single(pair):
    # the reference map: one handle, one pair, device in / device out
    with SGM(H, W, 1, D, device=0) as s:
        out = torch.empty((H, W), dtype=torch.float32, device=dev)
        l, r = (torch.from_numpy(a).to(dev) for a in pair)
        s.process_device(l.data_ptr(), r.data_ptr(), out.data_ptr(),
                         stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        return out.cpu()

def same(a, b):
    return torch.equal(a.cpu().contiguous().view(torch.int32), b.cpu().contiguous().view(torch.int32))

sgm = SGM(H, W, 1, D, device=0)
stream = torch.cuda.current_stream(dev)
def compute(pair):
    l, r = (torch.from_numpy(a).to(dev) for a in pair)
    out = torch.empty((H, W), dtype=torch.float32, device=dev)
    sgm.process_device(l.data_ptr(), r.data_ptr(), out.data_ptr(), stream=stream.cuda_stream)
    return out
"""

WORLD1_NCCL = COMMON + r"""
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
assert dist.get_backend() == "nccl"
want = [single(p) for p in PAIRS]
batch = sd.process_batch(PAIRS, compute, (H, W), check=sgm.check)
assert batch.is_cuda and tuple(batch.shape) == (5, H, W)
for k in range(5):
    assert same(batch[k], want[k]), k
print("process_batch ok", flush=True)
# bench.py's overlapped gather: step k writes buffer k % 2 while step k-1's
# gather may still run; each step's gathered map must be that step's pair
pipe = sd.PipelinedGather((H, W), torch.float32, dev, depth=2, check=sgm.check)
dl = [torch.from_numpy(p[0]).to(dev) for p in PAIRS]
dr = [torch.from_numpy(p[1]).to(dev) for p in PAIRS]
for k in range(6):
    buf = pipe.buffer()
    if k >= 2:
        pipe.verify()
        assert same(pipe.gathered(k - 2)[0], want[(k - 2) % 5]), k - 2
    sgm.process_device(dl[k % 5].data_ptr(), dr[k % 5].data_ptr(), buf.data_ptr(),
                       stream=stream.cuda_stream)
    pipe.submit()
pipe.drain()
for k in (4, 5):
    assert same(pipe.gathered(k)[0], want[k % 5]), k
print("pipelined gather ok", flush=True)
sgm.close()
dist.destroy_process_group()
print("world1 nccl ok")
"""

GLOO2 = COMMON + r"""
rank = int(sys.argv[3])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + sys.argv[2], rank=rank,
                        world_size=2)
pairs = PAIRS[:3]                       # uneven: rank 0 holds pairs 0, 2; rank 1 pair 1
batch = sd.process_batch(pairs, compute, (H, W), check=sgm.check)
pipe = sd.PipelinedGather((H, W), torch.float32, dev, depth=2, check=sgm.check)
seen = {}
for k in range(4):
    buf = pipe.buffer()
    if k >= 2:
        pipe.verify()
    if k >= 2 and rank == 0:
        seen[k - 2] = [t.clone() for t in pipe.gathered(k - 2)]
    p = PAIRS[(2 * k + rank) % 5]       # rank r's pair of step k
    l, r = (torch.from_numpy(a).to(dev) for a in p)
    sgm.process_device(l.data_ptr(), r.data_ptr(), buf.data_ptr(), stream=stream.cuda_stream)
    pipe.submit()
pipe.drain()
if rank == 0:
    for k in (2, 3):
        seen[k] = [t.clone() for t in pipe.gathered(k)]
    assert batch.device.type == "cpu" and tuple(batch.shape) == (3, H, W)
    for k in range(3):
        assert same(batch[k], single(pairs[k])), ("batch", k)
    for k in range(4):
        for r in range(2):
            assert same(seen[k][r], single(PAIRS[(2 * k + r) % 5])), ("pipe", k, r)
    print("gloo2 ok", flush=True)
else:
    assert batch is None
sgm.close()
dist.barrier()
dist.destroy_process_group()
"""


# BASELINE.json configs[3] ("config 4"): a batch of 8 KITTI pairs sharded one
# per rank over 8 ranks, maps gathered to rank 0 (node.cpp:49,93 is the
# per-pair call each rank makes).  The box has one GPU, so the 8 ranks share
# cuda:0 on gloo (maps staged through the host); each holds its own SGM
# handle.  Rank 0 saves what it gathered; the test compares every map with the
# oracle's map for that pair.
CONFIG4 = r"""
import os, sys, numpy as np, torch, torch.distributed as dist
root, port, rank, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
sys.path.insert(0, root)
from stereo_matching_amd import SGM, synthetic
from stereo_matching_amd import distributed as sd
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
H, W, D, N, GK = 375, 1242, 128, 8, 4
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + port, rank=rank, world_size=N)
PAIRS = [synthetic.stereo_pair(H, W, D, pair_index=i) for i in range(N)]
stream = torch.cuda.current_stream(dev)
sgm = SGM(H, W, 1, D, views=1, device=0)
def compute(pair):
    l, r = (torch.from_numpy(a).to(dev) for a in pair)
    m = torch.empty((H, W), dtype=torch.float32, device=dev)
    sgm.process_device(l.data_ptr(), r.data_ptr(), m.data_ptr(), stream=stream.cuda_stream)
    return m
batch = sd.process_batch(PAIRS, compute, (H, W), check=sgm.check)
# bench.py's batched gather (--gather-every 4): step k of rank r computes pair
# (k + r) % 8 into slot k % 4 of the rotating (4, H, W) buffer; one gather per
# 4 steps, overlapped with the next 4
pipe = sd.PipelinedGather((GK, H, W), torch.float32, dev, depth=2, check=sgm.check)
dl = [torch.from_numpy(p[0]).to(dev) for p in PAIRS]
dr = [torch.from_numpy(p[1]).to(dev) for p in PAIRS]
got = {}
for k in range(3 * GK):
    if k % GK == 0:
        buf = pipe.buffer()
        if k >= 2 * GK:
            pipe.verify()
        if k >= 2 * GK and rank == 0:
            got[k // GK - 2] = [t.clone() for t in pipe.gathered(k // GK - 2)]
    p = (k + rank) % N
    sgm.process_device(dl[p].data_ptr(), dr[p].data_ptr(), buf[k % GK].data_ptr(),
                       stream=stream.cuda_stream)
    if k % GK == GK - 1:
        pipe.submit()
pipe.drain()
if rank == 0:
    for b in (1, 2):
        got[b] = [t.clone() for t in pipe.gathered(b)]
    assert batch.device.type == "cpu" and tuple(batch.shape) == (N, H, W)
    # pipe[b][r][s]: step b*GK + s of rank r
    pipe_maps = np.stack([np.stack([t.numpy() for t in got[b]]) for b in range(3)])
    np.savez(out, batch=batch.numpy(), pipe=pipe_maps)
    print("config4 rank0 saved", flush=True)
else:
    assert batch is None
sgm.close()
dist.barrier()
dist.destroy_process_group()
"""


@pytest.mark.timeout(900)
def test_config4_batch_of_8_on_the_hip_path(tmp_path):
    import numpy as np

    import oracle
    from stereo_matching_amd import synthetic
    oracle.build()
    H, W, D, N, GK = 375, 1242, 128, 8, 4
    out = str(tmp_path / "config4.npz")
    port = _port()
    procs = [subprocess.Popen([sys.executable, "-c", CONFIG4, ROOT, port, str(r), out],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(N)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=420))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, (so, se)) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, (r, so[-2000:] + se[-4000:])
    assert "config4 rank0 saved" in outs[0][0]
    res = np.load(out)
    batch, pipe = res["batch"], res["pipe"]
    assert batch.shape == (N, H, W) and pipe.shape == (3, N, GK, H, W)
    for i in range(N):
        left, right = synthetic.stereo_pair(H, W, D, pair_index=i)
        want = oracle.process(left, right, D, views=1)["sub"].view(np.uint32)
        assert np.array_equal(batch[i].view(np.uint32), want), ("process_batch", i)
        # every (step, rank) that computed pair i: (b*GK + s + r) % N == i
        hits = 0
        for b in range(3):
            for r in range(N):
                for s in range(GK):
                    if (b * GK + s + r) % N == i:
                        assert np.array_equal(pipe[b, r, s].view(np.uint32), want), ("pipe", b, r, s)
                        hits += 1
        assert hits == 3 * GK


def _port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return str(sk.getsockname()[1])


@pytest.mark.timeout(300)
def test_world1_nccl_process_batch_and_pipelined_gather():
    r = subprocess.run([sys.executable, "-c", WORLD1_NCCL, ROOT, _port()], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "world1 nccl ok" in r.stdout, r.stdout[-3000:] + r.stderr[-4000:]


@pytest.mark.timeout(300)
def test_two_gloo_ranks_on_one_gpu():
    port = _port()
    procs = [subprocess.Popen([sys.executable, "-c", GLOO2, ROOT, port, str(rank)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for rank in range(2)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, (so, se) in zip(procs, outs):
        assert p.returncode == 0, so[-2000:] + se[-4000:]
    assert "gloo2 ok" in outs[0][0]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("extra", [[], ["--gather-every", "1"], ["--gather-every", "3"],
                                   ["--caller-stream"]],
                         ids=["default", "gather_every_step", "gather_every_3", "caller_stream"])
def test_bench_under_torch_distributed_run(extra):
    # the driver's multi-GPU launch line at N = 1: process group on nccl
    # (RCCL), the pipelined gather of the maps inside the timed region (the
    # default batches 4 steps' maps per collective: 5 timed steps end on a
    # partial batch; also one gather per step, batches of 3, and the frames
    # on a caller's stream)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", _port(), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "5", "--warmup", "2", "--no-profile-pass"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["n_gpus"] == 1 and rec["value"] > 0
    # what the process group saw, for the driver's SCALE runs to check
    assert rec["backend"] == "nccl" and rec["world_size_seen"] == 1
    assert 0 < rec["rank_timed_s"]["min"] <= rec["rank_timed_s"]["max"]
    assert abs(rec["rank_timed_s"]["max"] * 1e3 / 5 - rec["ms_per_step"]) < 1e-3 * rec["ms_per_step"] + 1e-3
    assert rec["frames_verified"] == ["warmup", "timed"]
    assert "RCCL" in rec["config"]["parallelism"]
    par = rec["config"]["parallelism"]
    if extra == ["--gather-every", "3"]:
        assert "every 3 steps" in par
    elif extra == ["--gather-every", "1"]:
        assert "every" not in par and "overlapped with the next step" in par
    else:
        assert "every 4 steps" in par
    assert rec["cpu_baseline"] is not None
