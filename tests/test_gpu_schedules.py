"""The frame schedules give the same maps bit for bit.

run_frame (sgm_capi.hip) picks the schedule by volume size: joint two-view
launches when both cost volumes fit the 256 MB Infinity Cache together,
per-view whole-volume passes below 256 MB per view, bands above it
(SGM_BAND_ROWS overrides the band size, 0 = whole-volume passes and the joint
final launch), and the slanted-tile passes (SGM_SLANT=1, sgm_slant.hip).  The
default schedule is pinned against the oracle by test_gpu_parity.py /
test_gpu_fullsize.py; these tests pin the others to it at sizes where the
library would not pick them.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from stereo_matching_amd import SGM, synthetic

pytestmark = pytest.mark.gpu


def _run(h, w, D, sky_l, sky_r, env):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        left, right = synthetic.stereo_pair(h, w, D, pair_index=5, kind="road")
        mask = synthetic.sky_mask(h, w)
        with SGM(h, w, 1, D, device=0) as s:
            s.process(left, right, mask if sky_l else None, mask if sky_r else None)
            return s.get_lr_disp().copy(), s.get_raw_disp().copy()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _same(a, b):
    assert np.array_equal(np.ascontiguousarray(a[0], np.float32).view(np.uint32),
                          np.ascontiguousarray(b[0], np.float32).view(np.uint32)), "LR map differs"
    assert np.array_equal(a[1], b[1]), "raw WTA map differs"


@pytest.mark.parametrize("h,w,D,sky_l,sky_r", [
    (120, 330, 64, False, False),
    (96, 260, 128, True, True),
    (80, 240, 256, True, True),
    (100, 300, 64, True, False),   # one mask only: per-view cost launches
    (375, 1242, 128, True, True),
])
@pytest.mark.parametrize("env", [{"SGM_BAND_ROWS": "16"}, {"SGM_BAND_ROWS": "32"}, {"SGM_SLANT": "1"}],
                         ids=["bands16", "bands32", "slant"])
def test_schedules_match_default(h, w, D, sky_l, sky_r, env):
    _same(_run(h, w, D, sky_l, sky_r, {}), _run(h, w, D, sky_l, sky_r, env))


def test_whole_volume_joint_final_matches_bands():
    # 512 x 1056 x 128 f32 = 277 MB per volume: above the Infinity Cache, so
    # the default runs bands; SGM_BAND_ROWS=0 runs whole-volume passes with
    # both views' final passes in one launch (pair_final2_kernel)
    h, w, D = 512, 1056, 128
    assert h * w * D * 4 > 256 * 1024 * 1024
    base = _run(h, w, D, False, False, {})
    _same(base, _run(h, w, D, False, False, {"SGM_BAND_ROWS": "0"}))
    _same(base, _run(h, w, D, False, False, {"SGM_SLANT": "1"}))


CROSS_STREAM = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
dev = torch.device("cuda", 0)
torch.cuda.init()
import oracle
from stereo_matching_amd import SGM, synthetic
h, w, D = 200, 640, 128
pairs = [synthetic.stereo_pair(h, w, D, pair_index=k, kind=("road", "noise")[k % 2]) for k in range(4)]
want = [oracle.process(l, r, D)["final"] for l, r in pairs]
streams = [torch.cuda.Stream(dev) for _ in range(3)]
imgs = [(torch.from_numpy(l).to(dev), torch.from_numpy(r).to(dev)) for l, r in pairs]
outs = [torch.empty((h, w), dtype=torch.float32, device=dev) for _ in pairs]
torch.cuda.synchronize(dev)
with SGM(h, w, 1, D, device=0) as sgm:
    # frame k on stream k % 3, its post filter on stream (k + 1) % 3, with no
    # host synchronisation in between: the handle orders the calls (they
    # share its cost volumes and post-filter scratch)
    for k, ((l, r), out) in enumerate(zip(imgs, outs)):
        sa, sb = streams[k % 3], streams[(k + 1) % 3]
        for t in (l, r, out):
            t.record_stream(sa)
        out.record_stream(sb)
        sgm.process_device(l.data_ptr(), r.data_ptr(), out.data_ptr(), stream=sa.cuda_stream)
        sgm.post_filter_device(out.data_ptr(), stream=sb.cuda_stream)
    torch.cuda.synchronize(dev)
for k, out in enumerate(outs):
    got = out.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), want[k].view(np.uint32)), k
# the handle's own stream (sgm_get_stream) as torch's stream, mixed with NULL
# and a caller's stream: torch work on it is ordered with the handle's calls
outs2 = [torch.empty((h, w), dtype=torch.float32, device=dev) for _ in pairs]
with SGM(h, w, 1, D, device=0) as sgm:
    assert sgm.stream != 0
    hs = torch.cuda.ExternalStream(sgm.stream, device=dev)
    for k, ((l, r), out) in enumerate(zip(imgs, outs2)):
        with torch.cuda.stream(hs):
            out.fill_(-1.0)
        st = (hs.cuda_stream, None, streams[k % 3].cuda_stream, None)[k]
        if st not in (None, hs.cuda_stream):
            out.record_stream(streams[k % 3])
        sgm.process_device(l.data_ptr(), r.data_ptr(), out.data_ptr(), stream=st)
        sgm.post_filter_device(out.data_ptr(), stream=None)
    torch.cuda.synchronize(dev)
for k, out in enumerate(outs2):
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want[k].view(np.uint32)), k
print("cross-stream ok")
"""


def test_calls_on_different_streams_are_ordered():
    # per-handle scratch shared by calls on different streams
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", CROSS_STREAM, root], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "cross-stream ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.timeout(120)
@pytest.mark.parametrize("views", [2, 1])
def test_slant_default_by_size(views, monkeypatch):
    # sgm_capi.hip slant_default: at D = 256 above the Infinity Cache the
    # slanted passes run once every workgroup gets 0.5 full-height tiles of
    # work (views x W >= 0.5 x 14 x CUs; on a 256-CU MI355X HD256 with two
    # views, 3840 >= 1792, and with one view, 1920: both slanted since round
    # 6's dataflow passes), else the bands; re-checked on the strip pass
    # (profiles/r06_experiments/r06r_sizes_vstrip.txt: HD256 one view -3.8%,
    # 720p D = 256 two views -10.9%).  The expectation uses the device's own
    # CU count, as the library does.
    import torch
    monkeypatch.delenv("SGM_SLANT", raising=False)
    h, w, D = 1080, 1920, 256
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    slanted = 10 * views * w >= 5 * 14 * cus
    left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
    with SGM(h, w, 1, D, views=views) as sgm:
        sgm.set_profiling(True)
        sgm.process(left, right)
        prof = sgm.get_profile()
    assert ("slant_up" in prof) == slanted, sorted(prof)
    assert ("stage_a_d" in prof) == (not slanted), sorted(prof)

