"""The slanted passes' hang guard surfaces through sgm_check and stays
bounded, the next frame is bit-exact, and the 1-, 2- and 3-workgroup grids
are bit-exact (tools/slant_guard.py on the -DSGM_SLANT_DEBUG build)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DBG = os.path.join(ROOT, "stereo_matching_amd", "libsgm_hip_slantdbg.so")


@pytest.fixture(scope="module", autouse=True)
def dbg_lib():
    # the debug library is built with the release one (__graft_entry__.build,
    # `make dbg`); a tree built with plain `make` gets it here
    if not os.path.exists(DBG):
        from stereo_matching_amd import _capi
        _capi.build(debug=True)
    return DBG


@pytest.mark.gpu
@pytest.mark.parametrize("D", [64, 256])
def test_slant_guard_and_small_grids(D):
    # D = 256 runs the receiver's other give-up loop (two re-polls in flight,
    # sgm_slant.hip V >= 4) and the four-step LDS ring at its largest
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "slant_guard.py"), "--D", str(D)],
                       capture_output=True, text=True, timeout=180, cwd=ROOT)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads(lines[-1])
    assert rec["baseline_exact"]
    st = rec["stall"]
    assert st["code"] == 3 and "timed out" in st["message"], st
    assert st["frame_s"] < 20, st          # bounded: one spin limit, not one per step
    # the release build's limit (2^22 polls) gives up within a minute
    assert 0 < st["release_give_up_s"] < 60, st
    assert rec["recovery"] == {"exact": True, "check_ok": True}
    assert all(v["exact"] for v in rec["grids"].values()), rec["grids"]
    assert r.returncode == 0


@pytest.mark.gpu
def test_bench_refuses_invalid_frames():
    # bench.py checks every pass's frames (sgm_check) before it reports a
    # time: with a forced hand-off stall (debug build, slanted schedule
    # forced on the K128 frame) it prints no JSON line and exits 3
    env = {**os.environ, "SGM_HIP_LIB": DBG,
           "SGM_SLANT": "1", "SGM_SLANT_STALL": "20", "SGM_SLANT_SPIN_LIMIT": "2000"}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-profile-pass"],
                       capture_output=True, text=True, timeout=180, cwd=ROOT, env=env)
    assert r.returncode == 3, r.stdout[-2000:] + r.stderr[-3000:]
    assert "the warmup pass produced invalid frames" in r.stderr and "timed out" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


FALLBACK = r"""
import json, os, sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
torch.cuda.init()
from stereo_matching_amd import SGM, SGMError, synthetic
h, w, D = 240, 1600, 256      # 393 MB per volume, 2 x 1600 columns: slanted by size (<= 326 CUs)
left, right = synthetic.stereo_pair(h, w, D, pair_index=3, kind="road")
def run():
    with SGM(h, w, 1, D) as s:
        s.set_profiling(True)
        s.process(left, right)
        s.check()
        return s.get_lr_disp().copy(), sorted(s.get_profile()), s.device_bytes
base = run()
os.environ["SGM_SLANT_NO_MEMORY"] = "1"
fb = run()
os.environ["SGM_SLANT"] = "1"
try:
    SGM(h, w, 1, D)
    forced = "created"
except SGMError as e:
    forced = str(e)
print(json.dumps({"base_slant": "slant_up" in base[1], "fb_slant": "slant_up" in fb[1],
                  "fb_bands": "stage_a_d" in fb[1], "exact": bool(np.array_equal(base[0].view(np.uint32), fb[0].view(np.uint32))),
                  "bytes": [base[2], fb[2]], "forced": forced}))
"""


@pytest.mark.gpu
def test_slanted_schedule_falls_back_to_bands_without_memory():
    # sgm_create (sgm_capi.hip): the slanted schedule's buffers failing to
    # allocate (forced on the debug build) -> the banded schedule, same maps;
    # with SGM_SLANT=1 the failure is returned
    env = {**os.environ, "SGM_HIP_LIB": DBG}
    env.pop("SGM_SLANT", None)
    env.pop("SGM_SLANT_NO_MEMORY", None)
    r = subprocess.run([sys.executable, "-c", FALLBACK, ROOT], capture_output=True, text=True, timeout=240,
                       cwd=ROOT, env=env)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads(lines[-1])
    if not rec["base_slant"]:
        pytest.skip("this device's CU count keeps the frame on the bands (sgm_capi.hip slant_default)")
    assert not rec["fb_slant"] and rec["fb_bands"], rec
    assert rec["exact"], rec
    assert rec["bytes"][1] < rec["bytes"][0], rec
    assert rec["forced"] != "created", rec
    assert "sgm_create: hipMalloc: out of memory (forced" in r.stderr, r.stderr[-2000:]
