"""GPU post_filter() (src/Solver.cpp:600-649) against the CPU oracle, bit-exact.

The oracle (oracle/sgm_oracle.c:orc_post_filter) runs the reference's
sequential in-place median fill and the single-thread semantics of
speckle_filter_new; the GPU path (sgm_post.hip) must reproduce both exactly
on every map, including fills that chain across its 64x4 / 64x8 / 64x16 tiles and
components that straddle the 1000/scale size limit.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
import postfilter_maps
from stereo_matching_amd import BM, SGM, synthetic

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def check_map(sgm, F, D, scale):
    want = oracle.post_filter(F.copy(), D, scale)
    got = sgm.post_filter(F)
    bad = np.flatnonzero(bits(got).ravel() != bits(want).ravel())
    assert bad.size == 0, (f"{bad.size} mismatches, first at {np.unravel_index(bad[0], F.shape)}: "
                           f"got {got.ravel()[bad[0]]!r} want {want.ravel()[bad[0]]!r}")
    return got


SIZES = [(48, 96), (61, 203), (130, 257), (375, 1242)]


@pytest.mark.parametrize("kind", postfilter_maps.KINDS)
@pytest.mark.parametrize("hw", SIZES, ids=[f"{h}x{w}" for h, w in SIZES])
def test_post_filter_maps(kind, hw):
    H, W = hw
    D = 64
    with SGM(H, W, 1, D, device=0) as sgm:
        for seed in range(2):
            check_map(sgm, postfilter_maps.make(kind, H, W, D, seed), D, 1)


@pytest.mark.parametrize("rows", ["4", "8", "16"])
@pytest.mark.parametrize("hw", [(61, 203), (375, 1242)], ids=["61x203", "375x1242"])
def test_post_filter_tile_heights(rows, hw, monkeypatch):
    """Every tile height of the median fill (the default picks 4 or 8 rows by
    frame size; SGM_MF_ROWS forces one) gives the same bits."""
    monkeypatch.setenv("SGM_MF_ROWS", rows)
    H, W = hw
    D = 64
    with SGM(H, W, 1, D, device=0) as sgm:
        for kind in postfilter_maps.KINDS:
            check_map(sgm, postfilter_maps.make(kind, H, W, D, 3), D, 1)


@pytest.mark.parametrize("D", [32, 128, 256])
@pytest.mark.parametrize("scale", [1, 2])
def test_post_filter_disparity_range_and_scale(D, scale):
    # scale 2 halves the speckle limit (SPECKLE_SIZE/scale, Solver.cpp:645)
    h, w = 160 * scale, 300 * scale
    with SGM(h, w, scale, D, device=0) as sgm:
        for kind in ("random_holes", "speckle", "diag", "threshold"):
            check_map(sgm, postfilter_maps.make(kind, h // scale, w // scale, D, 7), D, scale)


@pytest.mark.parametrize("hw", [(3, 5), (4, 7), (5, 5), (6, 70), (17, 65), (200, 6), (33, 129)])
def test_post_filter_small_and_ragged(hw):
    # frames whose interior (rows/cols 2..n-3) is empty, one pixel, or ends
    # just past a tile boundary
    H, W = hw
    with SGM(H, W, 1, 32, device=0) as sgm:
        for kind in ("random_holes", "dense_holes", "all_invalid", "speckle"):
            check_map(sgm, postfilter_maps.make(kind, H, W, 32, 3), 32, 1)


def test_post_filter_component_size_limit():
    # one component of exactly 1000 pixels survives, 999+... : a 1000-pixel
    # and a 1001-pixel bar crossing tile borders, in an invalid sea
    H, W, D = 64, 300, 64
    F = np.full((H, W), D + 1, np.float32)
    F[10:15, 0:200] = 10.0        # 1000 pixels: removed (area <= 1000)
    F[30:35, 0:200] = 20.0
    F[35, 0] = 20.0               # 1001 pixels: kept
    with SGM(H, W, 1, D, device=0) as sgm:
        got = check_map(sgm, F, D, 1)
    assert (got[10:15, 0:200] == D + 1).all() and (got[30:35, 0:200] == 20.0).all()


@pytest.mark.parametrize("kind", ["noise", "road"])
def test_post_filter_after_pipeline(kind):
    # the map post_filter sees in SGM::process: the LR-checked output
    h, w, D = 120, 330, 64
    left, right = synthetic.stereo_pair(h, w, D, pair_index=5, kind=kind)
    with SGM(h, w, 1, D, device=0) as sgm:
        sgm.process(left, right)
        lr = sgm.get_lr_disp().copy()
        got = sgm.get_disp()
    ref = oracle.process(left, right, D)
    assert np.array_equal(bits(lr), bits(ref["lr"]))
    assert np.array_equal(bits(got), bits(ref["final"]))


def test_process_with_post_filter_param():
    h, w, D = 96, 260, 64
    left, right = synthetic.stereo_pair(h, w, D, pair_index=2, kind="noise")
    ref = oracle.process(left, right, D)
    # sgm_process with params.post_filter = 1 returns get_disp() directly
    with SGM(h, w, 1, D, device=0, post_filter=True) as sgm:
        sgm.process(left, right)
        assert np.array_equal(bits(sgm.get_disp()), bits(ref["final"]))


PITCHED = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
dev = torch.device("cuda", 0)
torch.cuda.init()                      # torch's runtime first, as in bench.py
import oracle
from stereo_matching_amd import BM, SGM, synthetic
h, w, D = 96, 260, 64
left, right = synthetic.stereo_pair(h, w, D, pair_index=2, kind="noise")
ref = oracle.process(left, right, D)
pitch = w + 37
buf = torch.full((h, pitch), -7.0, dtype=torch.float32, device=dev)
buf[:, :w] = torch.from_numpy(ref["lr"]).to(dev)
with SGM(h, w, 1, D, device=0) as sgm:
    sgm.post_filter_device(buf.data_ptr(), pitch=pitch)
    torch.cuda.synchronize(dev)
out = buf.cpu().numpy()
assert np.array_equal(out[:, :w].view(np.uint32), ref["final"].view(np.uint32))
assert (out[:, w:] == -7.0).all()
print("pitched ok")
"""


def test_post_filter_device_pitched_map():
    # sgm_post_filter_device in place on a pitched device map (pitch > cols),
    # in a child process so torch's HIP runtime initialises before the library's
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", PITCHED, root], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "pitched ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_post_filter_repeatable():
    # the chaotic tile relaxation must land on the same fixed point every time
    H, W, D = 200, 700, 64
    F = postfilter_maps.make("diag", H, W, D, 11)
    with SGM(H, W, 1, D, device=0) as sgm:
        first = check_map(sgm, F, D, 1)
        for _ in range(3):
            assert np.array_equal(bits(sgm.post_filter(F)), bits(first))


@pytest.mark.parametrize("kind", ["post_filter", "lk_refine", "bm"])
def test_process_twice_on_one_handle(kind):
    # every process() on a post_filter / lk_refine / BM handle writes a fresh
    # final map (the second call used to pass a NULL output), and
    # the map handed out for frame 1 is not overwritten by frame 2
    h, w, D = 64, 200, 64
    pairs = [synthetic.stereo_pair(h, w, D, pair_index=k, kind=("noise" if k else "road"))
             for k in range(3)]
    if kind == "bm":
        want = [oracle.post_filter(oracle.bm_process(l, r, D, 1).astype(np.float32), D, 1)
                for l, r in pairs]
        handle = BM(h, w, 1, D, device=0)
    elif kind == "lk_refine":
        want = [oracle.lk_refine(l, r, oracle.process(l, r, D)["final"], D) for l, r in pairs]
        handle = SGM(h, w, 1, D, device=0, post_filter=True, lk_refine=True)
    else:
        want = [oracle.process(l, r, D)["final"] for l, r in pairs]
        handle = SGM(h, w, 1, D, device=0, post_filter=True)
    with handle as sgm:
        kept = []
        for l, r in pairs:
            sgm.process(l, r)
            kept.append(sgm.get_disp())
        for k in range(len(pairs)):
            assert np.array_equal(bits(kept[k]), bits(want[k])), k
