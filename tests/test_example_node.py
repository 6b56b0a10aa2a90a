"""examples/stereo_node.cpp -- the ROS node's per-frame flow (node.cpp:25-151:
sky detector on both images, SGM::process with the masks, get_disp, show_disp,
the point cloud) through the drop-in headers -- compiles with g++ against
libsgm_hip.so and, on the GPU, writes the oracle's results bit for bit."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

import pyref
from stereo_matching_amd import _capi, synthetic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "examples", "stereo_node.cpp")
CAM = (721.5377, 721.5377, 609.5593, 172.854)   # the example's defaults (KITTI image_0)


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if not os.path.exists(_capi.LIB_PATH):
        _capi.build()
    out = str(tmp_path_factory.mktemp("node") / "stereo_node")
    libdir = os.path.dirname(_capi.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    SRC, "-L", libdir, "-lsgm_hip", f"-Wl,-rpath,{libdir}", "-o", out],
                   check=True, capture_output=True, text=True)
    return out


def _pgm(path, img):
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (img.shape[1], img.shape[0]))
        f.write(np.ascontiguousarray(img, np.uint8).tobytes())


def test_example_builds_and_checks_arguments(exe, tmp_path):
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr
    bad = tmp_path / "bad.pgm"
    bad.write_bytes(b"P2\n1 1\n255\n0\n")
    r = subprocess.run([exe, str(bad), str(bad), str(tmp_path / "o")], capture_output=True, text=True)
    assert r.returncode == 2


@pytest.mark.gpu
@pytest.mark.parametrize("scale,D", [(1, 64), (2, 64), (1, 128)])
def test_example_node_flow_matches_oracle(exe, tmp_path, scale, D):
    import oracle
    oracle.build()
    h, w = 150 * scale, 420 * scale
    left, right = synthetic.stereo_pair(h, w, D, pair_index=21, kind="road")
    left[: h // 5] //= 4          # a darker, flat band on top for the sky detector
    right[: h // 5] //= 4
    _pgm(tmp_path / "l.pgm", left)
    _pgm(tmp_path / "r.pgm", right)
    prefix = str(tmp_path / "out")
    r = subprocess.run([exe, str(tmp_path / "l.pgm"), str(tmp_path / "r.pgm"), prefix, str(scale), str(D)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    H, W = h // scale, w // scale
    sky_l, sky_r = oracle.sky_detect(left, scale), oracle.sky_detect(right, scale)
    want = oracle.process(left, right, D, scale=scale, sky_l=sky_l, sky_r=sky_r)["final"]
    got = np.fromfile(prefix + "_disp.f32", np.float32).reshape(H, W)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    # show_disp (Solver.cpp:55-93): gray left image on top, the colormap from row H-1
    with open(prefix + "_debug.ppm", "rb") as f:
        assert f.readline() == b"P6\n" and f.readline() == b"%d %d\n" % (W, 2 * H) and f.readline() == b"255\n"
        view = np.frombuffer(f.read(), np.uint8).reshape(2 * H, W, 3)[..., ::-1]   # RGB -> BGR
    small = left[: H * scale: scale, : W * scale: scale]
    assert np.array_equal(view[: H - 1], np.repeat(small[: H - 1, :, None], 3, axis=2))
    assert np.array_equal(view[H - 1: 2 * H - 1], pyref.colormap(want, D))
    assert not view[2 * H - 1].any()   # the debug view's last row is never written
    # the point cloud (node.cpp:113-143), push_back order
    want_xyz, want_pix = pyref.point_cloud(want, left, D, scale, *CAM)
    raw = open(prefix + "_cloud.bin", "rb").read()
    n = len(want_pix)
    assert len(raw) == n * 25
    xyz = np.frombuffer(raw[: n * 24], np.float64).reshape(n, 3)
    assert np.array_equal(xyz.view(np.uint64), want_xyz.view(np.uint64))
    assert np.array_equal(np.frombuffer(raw[n * 24:], np.uint8), want_pix)
    assert f"pointcloud size: {n}, {n}" in r.stdout
