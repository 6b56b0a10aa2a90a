"""A pair's two views on separate handles (the optional
2-GPU split): an SGM_VIEW_RIGHT handle computes the right view alone
(SGM.cpp:448-801), sgm_lr_check_device joins it with the left view
(SGM.cpp:803-818), and post_filter/LKRefine then run on the left view's
device.  The joined map must equal the two-view handle's output bit for bit,
and the right view must equal the oracle's filtered_disp_beta.

The device-pointer cases run in child processes so torch's HIP runtime
initialises before the library's (as bench.py does); the two-rank case
runs both ranks on cuda:0 over gloo (the box has one GPU; RCCL needs a GPU
per rank), which exercises ViewSplit's protocol and its host staging.
"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SPLIT = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
dev = torch.device("cuda", 0)
torch.cuda.init()
import oracle
from stereo_matching_amd import SGM, synthetic

def bits(t):
    a = t.cpu().numpy() if isinstance(t, torch.Tensor) else t
    return np.ascontiguousarray(a, np.float32).view(np.uint32)

def u8(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

CASES = [  # h, w, D, scale, kind, sky, sky_detect
    (96, 260, 64, 1, "noise", False, False),
    (120, 330, 128, 1, "road", True, False),
    (100, 300, 32, 2, "road", False, False),
    (72, 200, 256, 1, "road", True, False),
    (160, 420, 64, 1, "road", False, True),
    (375, 1242, 128, 1, "road", False, False),
]
for h, w, D, s, kind, sky, detect in CASES:
    left, right = synthetic.stereo_pair(h, w, D, pair_index=3, kind=kind)
    H, W = h // s, w // s
    mask = synthetic.sky_mask(H, W) if sky else None
    dl, dr = u8(left), u8(right)
    dm = u8(mask) if sky else None
    mp = dm.data_ptr() if sky else 0
    kw = dict(device=0, sky_detect=detect)
    full = torch.empty((H, W), dtype=torch.float32, device=dev)
    fullpf = torch.empty_like(full)
    with SGM(h, w, s, D, **kw) as a:
        a.process_device(dl.data_ptr(), dr.data_ptr(), full.data_ptr(), d_sky_l=mp, d_sky_r=mp)
    with SGM(h, w, s, D, post_filter=True, **kw) as a:
        a.process_device(dl.data_ptr(), dr.data_ptr(), fullpf.data_ptr(), d_sky_l=mp, d_sky_r=mp)
    # the split: pitched maps, the right map in its own buffer
    fl = torch.full((H, W + 5), -3.0, dtype=torch.float32, device=dev)
    fr = torch.full((H, W + 3), -3.0, dtype=torch.float32, device=dev)
    out = torch.full((H, W + 9), -3.0, dtype=torch.float32, device=dev)
    raw_r = torch.zeros((H, W), dtype=torch.int16, device=dev)
    with SGM(h, w, s, D, views=1, **kw) as L, SGM(h, w, s, D, views=1, view="right", **kw) as R:
        L.process_device(dl.data_ptr(), dr.data_ptr(), fl.data_ptr(), out_pitch=W + 5,
                         d_sky_l=mp, d_sky_r=0)
        R.process_device(dl.data_ptr(), dr.data_ptr(), fr.data_ptr(), out_pitch=W + 3,
                         d_sky_l=0, d_sky_r=mp, d_raw=raw_r.data_ptr())
        torch.cuda.synchronize(dev)
        L.lr_check_device(fl.data_ptr(), fr.data_ptr(), out.data_ptr(), fl_pitch=W + 5,
                          fr_pitch=W + 3, out_pitch=W + 9)
        torch.cuda.synchronize(dev)
        assert np.array_equal(bits(out[:, :W]), bits(full)), (h, w, D, s, kind, "lr")
        assert (out[:, W:] == -3.0).all()
        # in place (d_out == d_fl), then the post stages on the same device
        L.lr_check_device(fl.data_ptr(), fr.data_ptr(), fl.data_ptr(), fl_pitch=W + 5,
                          fr_pitch=W + 3, out_pitch=W + 5)
        L.post_filter_device(fl.data_ptr(), pitch=W + 5)
        torch.cuda.synchronize(dev)
        assert np.array_equal(bits(fl[:, :W]), bits(fullpf)), (h, w, D, s, kind, "post_filter")
        assert (fl[:, W:] == -3.0).all()
    if not detect and h * w <= 200000:
        ref = oracle.process(left, right, D, scale=s, sky_l=mask, sky_r=mask)
        assert np.array_equal(bits(fr[:, :W]), bits(ref["sub_beta"])), (h, w, D, s, kind, "F_R")
        assert np.array_equal(raw_r.cpu().numpy().astype(np.int32), ref["disp_beta"]), "disp_beta"
    print("case ok", h, w, D, s, kind, sky, detect, flush=True)
print("split ok")
"""

TEAM = r"""
import os, sys, numpy as np, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
rank = int(sys.argv[2])
dev = torch.device("cuda", 0)
torch.cuda.init()
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + sys.argv[3], rank=rank,
                        world_size=2)
from stereo_matching_amd import SGM, synthetic
from stereo_matching_amd.distributed import ViewSplit
h, w, D = 150, 400, 64
left, right = synthetic.stereo_pair(h, w, D, pair_index=6, kind="road")
dl = torch.from_numpy(left).to(dev)
dr = torch.from_numpy(right).to(dev)
sgm = SGM(h, w, 1, D, device=0, views=1, view="right" if rank else "left")
team = ViewSplit(sgm, h, w, dev, post_filter=True)
for _ in range(3):
    out = team.step(dl.data_ptr(), dr.data_ptr())
torch.cuda.synchronize(dev)
if rank == 0:
    with SGM(h, w, 1, D, device=0, post_filter=True) as full:
        want = torch.empty((h, w), dtype=torch.float32, device=dev)
        full.process_device(dl.data_ptr(), dr.data_ptr(), want.data_ptr())
        torch.cuda.synchronize(dev)
    assert torch.equal(out.view(torch.int32), want.view(torch.int32))
    print("team ok")
else:
    assert out is None
sgm.close()
dist.barrier()
dist.destroy_process_group()
"""


def _run(script, *args, timeout=300):
    return subprocess.run([sys.executable, "-c", script, ROOT, *args], capture_output=True,
                          text=True, timeout=timeout)


def test_view_split_matches_two_view_handle():
    r = _run(SPLIT)
    assert r.returncode == 0 and "split ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_view_split_team_over_gloo():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = str(sk.getsockname()[1])
    procs = [subprocess.Popen([sys.executable, "-c", TEAM, ROOT, str(rank), port],
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
        assert p.returncode == 0, so[-2000:] + se[-3000:]
    assert "team ok" in outs[0][0]
