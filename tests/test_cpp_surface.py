"""The reference's C++ class surface (include/sgm_amd/SGM.h, mirroring
inc/Solver.h:23-70 and inc/SGM.h:10-26) compiles with g++ against the C-ABI
library, enforces the reference's constructor asserts, and -- on the GPU --
returns get_disp() bit-identical to the oracle's SGM::process (LR check +
post_filter, src/SGM.cpp:32-826)."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from stereo_matching_amd import _capi, synthetic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "sgm_class_surface.cpp")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if not os.path.exists(_capi.LIB_PATH):
        _capi.build()
    out = str(tmp_path_factory.mktemp("cpp") / "sgm_class_surface")
    libdir = os.path.dirname(_capi.LIB_PATH)
    # BatchSGM.h uses the HIP runtime API on the host (plain g++, no hipcc)
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                    SRC, "-L", libdir, "-lsgm_hip", f"-Wl,-rpath,{libdir}", "-L", "/opt/rocm/lib",
                    "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-pthread", "-o", out],
                   check=True, capture_output=True, text=True)
    return out


def _has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_header_compiles_and_asserts(exe):
    if _has_gpu():
        pytest.skip("the no-device case needs a machine without a GPU")
    r = subprocess.run([exe, "nodevice"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("threw as expected") == 4
    assert "BatchSGM threw" in r.stdout
    assert r.stdout.count("check_batch threw") == 3


@pytest.mark.gpu
def test_class_surface_matches_oracle(exe, tmp_path):
    import oracle
    oracle.build()
    h, w, D = 96, 208, 64
    left, right = synthetic.stereo_pair(h, w, D, pair_index=3)
    fl, fr, fo = (str(tmp_path / n) for n in ("l.raw", "r.raw", "out.raw"))
    left.tofile(fl)
    right.tofile(fr)
    r = subprocess.run([exe, "run", fl, fr, str(h), str(w), str(D), fo],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(fo, dtype=np.float32).reshape(h, w)
    want = oracle.process(left, right, D, views=2)["final"]
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_bm_class_surface_matches_oracle(exe, tmp_path):
    # BM(h, w, s, d) through the same Solver pointer the node holds (node.cpp:49-50)
    import oracle
    oracle.build()
    h, w, D = 80, 240, 64
    left, right = synthetic.stereo_pair(h, w, D, pair_index=4)
    fl, fr, fo = (str(tmp_path / n) for n in ("l.raw", "r.raw", "out.raw"))
    left.tofile(fl)
    right.tofile(fr)
    r = subprocess.run([exe, "runbm", fl, fr, str(h), str(w), str(D), fo],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(fo, dtype=np.float32).reshape(h, w)
    want = oracle.post_filter(oracle.bm_process(left, right, D).astype(np.float32), D)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("scale,D", [(1, 64), (2, 64), (1, 128)])
def test_gpu_sgm_class_matches_oracle(exe, tmp_path, scale, D):
    # GPU_SGM (gpu_sgm/inc/SGM.cuh:23-62) built as node.cpp:50 would build it:
    # the left view's sub-pixel map (SGM.cpp:32-443), post_filter()ed
    # (GPU_SGM::process, gpu_sgm/src/SGM.cu:217-225), with the reference CPU
    # semantics; show_disp() then marks the left d/s columns invalid in place
    # (SGM.cu:238-246)
    import oracle
    oracle.build()
    h, w = 90, 236
    left, right = synthetic.stereo_pair(h, w, D, pair_index=6)
    fl, fr, fo, fo2 = (str(tmp_path / n) for n in ("l.raw", "r.raw", "out.raw", "out2.raw"))
    left.tofile(fl)
    right.tofile(fr)
    r = subprocess.run([exe, "rungpu", fl, fr, str(h), str(w), str(scale), str(D), fo, fo2],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    H, W = h // scale, w // scale
    got = np.fromfile(fo, dtype=np.float32).reshape(H, W)
    sub = oracle.process(left, right, D, scale=scale, views=1)["sub"]
    want = oracle.post_filter(sub, D, scale=scale)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    after = np.fromfile(fo2, dtype=np.float32).reshape(H, W)
    want[:, :D // scale] = D + 1
    assert np.array_equal(after.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_sky_detector_wrapper_matches_reference_example(exe, tmp_path):
    # sky_detector::SkyAreaDetector as node.cpp:51,83 uses it, on the
    # reference's own example (tests/golden/sky_000017_14.npz)
    g = np.load(os.path.join(ROOT, "tests", "golden", "sky_000017_14.npz"))
    img, want = g["image"], g["mask"]
    fi, fo = str(tmp_path / "img.raw"), str(tmp_path / "mask.raw")
    img.tofile(fi)
    h, w = img.shape
    r = subprocess.run([exe, "sky", fi, str(h), str(w), "1", fo], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert np.array_equal(np.fromfile(fo, np.uint8).reshape(h, w), want)


@pytest.mark.gpu
def test_lk_wrapper_matches_oracle(exe, tmp_path):
    import oracle
    oracle.build()
    h, w, D = 64, 200, 64
    left, right = synthetic.stereo_pair(h, w, D, pair_index=5)
    disp = oracle.process(left, right, D)["final"]
    paths = [str(tmp_path / n) for n in ("l.raw", "r.raw", "d.raw", "out.raw")]
    left.tofile(paths[0])
    right.tofile(paths[1])
    disp.tofile(paths[2])
    r = subprocess.run([exe, "lk", *paths[:3], str(h), str(w), str(D), paths[3]],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(paths[3], np.float32).reshape(h, w)
    want = oracle.lk_refine(left, right, disp, D)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("masks", ["left", "right", "both"])
def test_class_surface_one_sided_sky_masks(exe, tmp_path, masks):
    # process(l, r, sky, sky_beta): each mask applies to its own view
    # (Solver.cpp:146-178 left DSI, :200-232 right DSI), also when the other
    # one is empty; the beta mask comes with a different row pitch
    import oracle
    oracle.build()
    h, w, D = 72, 220, 64
    left, right = synthetic.stereo_pair(h, w, D, pair_index=8)
    sky = synthetic.sky_mask(h, w)
    sl = sky if masks in ("left", "both") else None
    sr = sky if masks in ("right", "both") else None
    paths = {n: str(tmp_path / n) for n in ("l", "r", "sl", "sr", "out")}
    left.tofile(paths["l"])
    right.tofile(paths["r"])
    args = [exe, "runsky", paths["l"], paths["r"], "-", "-", str(h), str(w), str(D), paths["out"]]
    if sl is not None:
        sl.tofile(paths["sl"])
        args[4] = paths["sl"]
    if sr is not None:
        sr.tofile(paths["sr"])
        args[5] = paths["sr"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(paths["out"], dtype=np.float32).reshape(h, w)
    want = oracle.process(left, right, D, sky_l=sl, sky_r=sr)["final"]
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    if masks != "both":   # a one-sided mask is not silently dropped
        none = oracle.process(left, right, D)["final"]
        assert not np.array_equal(got.view(np.uint32), none.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [3, 5])
def test_batch_sgm_matches_oracle(exe, tmp_path, n):
    # include/sgm_amd/BatchSGM.h: SGM(h, w, s, d) per device, one host thread
    # per device, sgm_check, then sgm_batch_gather_all (ncclGather) to the
    # first device; on a one-GPU box 2N+1 = 3 (and 5) pairs run in rounds of
    # 1, so the double-buffered maps, root buffers and host staging each
    # cycle, and each round's gather and copy-out overlap the next round's
    # frame.  Every get_disp(k) equals the oracle's post-filtered map for pair k.
    import oracle
    oracle.build()
    h, w, D = 72, 200, 64
    prefix = str(tmp_path / "pair")
    want = []
    for k in range(n):
        left, right = synthetic.stereo_pair(h, w, D, pair_index=60 + k)
        left.tofile(f"{prefix}_l{k}.raw")
        right.tofile(f"{prefix}_r{k}.raw")
        want.append(oracle.process(left, right, D)["final"])
    fo = str(tmp_path / "out.raw")
    r = subprocess.run([exe, "batch", prefix, str(n), str(h), str(w), str(D), fo],
                       capture_output=True, text=True, timeout=120,
                       env={**os.environ, "SGM_AMD_DEVICES": "0"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"batch of {n} pairs on 1 device(s)" in r.stdout
    got = np.fromfile(fo, dtype=np.float32).reshape(n, h, w)
    for k in range(n):
        assert np.array_equal(got[k].view(np.uint32), want[k].view(np.uint32)), k
