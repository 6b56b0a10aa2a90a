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


@pytest.mark.gpu
def test_slant_guard_and_small_grids():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "slant_guard.py")],
                       capture_output=True, text=True, timeout=180, cwd=ROOT)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads(lines[-1])
    assert rec["baseline_exact"]
    st = rec["stall"]
    assert st["code"] == 3 and "timed out" in st["message"], st
    assert st["frame_s"] < 20, st          # bounded: one spin limit, not one per step
    assert rec["recovery"] == {"exact": True, "check_ok": True}
    assert all(v["exact"] for v in rec["grids"].values()), rec["grids"]
    assert r.returncode == 0


@pytest.mark.gpu
def test_bench_refuses_invalid_frames():
    # bench.py checks every pass's frames (sgm_check) before it reports a
    # time: with a forced hand-off stall (debug build, slanted schedule
    # forced on the K128 frame) it prints no JSON line and exits 3
    env = {**os.environ, "SGM_HIP_LIB": os.path.join(ROOT, "stereo_matching_amd", "libsgm_hip_slantdbg.so"),
           "SGM_SLANT": "1", "SGM_SLANT_STALL": "20", "SGM_SLANT_SPIN_LIMIT": "2000"}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-profile-pass"],
                       capture_output=True, text=True, timeout=180, cwd=ROOT, env=env)
    assert r.returncode == 3, r.stdout[-2000:] + r.stderr[-3000:]
    assert "the warmup pass produced invalid frames" in r.stderr and "timed out" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]
