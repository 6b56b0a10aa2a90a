"""GPU LKRefine (LKRefine/LKSubPixelImpl.cpp:13-235) against the CPU oracle.

Bar: bit-exact against oracle/sgm_oracle.c:orc_lk_refine, which pins the fp32
evaluation order of the reference's Eigen expressions (DESIGN.md "LKRefine");
north_star's 1e-4 tolerance is for the reference's own (unpinned) order.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from stereo_matching_amd import SGM, synthetic

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def check(sgm, left, right, disp, D, s):
    L, R = left[::s, ::s][:sgm.rows, :sgm.cols], right[::s, ::s][:sgm.rows, :sgm.cols]
    want = oracle.lk_refine(L, R, disp, D)
    got = sgm.lk_refine(left, right, disp)
    bad = np.flatnonzero(bits(got).ravel() != bits(want).ravel())
    assert bad.size == 0, (f"{bad.size} mismatches, first at {np.unravel_index(bad[0], disp.shape)}"
                           f": got {got.ravel()[bad[0]]!r} want {want.ravel()[bad[0]]!r}")
    return got, want


CASES = [(48, 96, 32, 1), (61, 203, 64, 1), (120, 330, 128, 1), (64, 300, 256, 1),
         (90, 180, 64, 2), (7, 9, 32, 1), (6, 70, 32, 1), (375, 1242, 128, 1)]


@pytest.mark.parametrize("case", CASES, ids=[f"{h}x{w}_D{D}_s{s}" for h, w, D, s in CASES])
@pytest.mark.parametrize("kind", ["road", "noise"])
def test_lk_refine_on_pipeline_output(case, kind):
    # the map SGM.cpp:824 would hand it: post_filter()ed LR output
    h, w, D, s = case
    left, right = synthetic.stereo_pair(h, w, D, pair_index=4, kind=kind)
    with SGM(h, w, s, D, device=0) as sgm:
        sgm.process(left, right)
        final = sgm.get_disp().copy()
        got, _ = check(sgm, left, right, final, D, s)
    if kind == "road" and h >= 48 and w // s >= 2 * D:
        inner = np.s_[3:-3, 3:-3]
        assert (got[inner] != np.trunc(final[inner])).any(), "nothing was refined"


@pytest.mark.parametrize("seed", range(3))
def test_lk_refine_random_maps(seed):
    # arbitrary maps: offsets that push samples off both image edges, invalid
    # and zero disparities, neighbours just inside / outside |d0 - dm| <= 2
    rng = np.random.default_rng(seed)
    h, w, D = 80, 150, 64
    left = rng.integers(0, 256, (h, w), dtype=np.uint8)
    left[:, ::3] = np.clip(left[:, ::3].astype(int) + 60, 0, 255).astype(np.uint8)
    right = np.roll(left, -7, axis=1)
    right[:, -20:] = rng.integers(0, 256, (h, 20), dtype=np.uint8)
    disp = (7 + rng.normal(0, 1.5, (h, w))).astype(np.float32)
    disp[rng.random((h, w)) < 0.1] = D + 1
    disp[rng.random((h, w)) < 0.05] = 0.4
    disp[:, :10] = rng.uniform(0, 30, (h, 10)).astype(np.float32)
    with SGM(h, w, 1, D, device=0) as sgm:
        check(sgm, left, right, disp, D, 1)


def test_lk_refine_known_answer():
    # pure shift by 5 on a ramp: Ires = 0 everywhere, result exactly 5
    H, W, D = 20, 60, 32
    L = np.tile((np.arange(W) * 3) % 256, (H, 1)).astype(np.uint8)
    R = np.zeros_like(L)
    R[:, :W - 5] = L[:, 5:]
    disp = np.full((H, W), 5.7, np.float32)
    with SGM(H, W, 1, D, device=0) as sgm:
        got, _ = check(sgm, L, R, disp, D, 1)
    assert (got[3:-3, 3:W - 15] == 5.0).all()
    assert (got[:3] == np.float32(5.7)).all()   # border rows untouched


def test_process_full_pipeline_with_lk():
    # sgm_process with post_filter + lk_refine: SGM.cpp:821 then :824
    h, w, D = 96, 260, 64
    left, right = synthetic.stereo_pair(h, w, D, pair_index=6, kind="road")
    ref = oracle.process(left, right, D)
    want = oracle.lk_refine(left, right, ref["final"], D)
    with SGM(h, w, 1, D, device=0, post_filter=True, lk_refine=True) as sgm:
        sgm.process(left, right)
        got = sgm.get_disp()
    assert np.array_equal(bits(got), bits(want))
