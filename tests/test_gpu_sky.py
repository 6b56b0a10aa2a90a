"""GPU sky detector (sky_detector/imageSkyDetector.cpp:166-208) against the
reference's own output and the CPU oracle, bit-exact (u8 masks)."""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle
import sky_images
from stereo_matching_amd import SGM

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "sky_000017_14.npz")


def test_sky_detect_matches_reference_example():
    g = np.load(GOLDEN)
    img, want = g["image"], g["mask"]
    with SGM(img.shape[0], img.shape[1], 1, 64, device=0) as sgm:
        got = sgm.sky_detect(img)
    assert np.array_equal(got, want), int((got != want).sum())


@pytest.mark.parametrize("kind", sky_images.KINDS)
@pytest.mark.parametrize("hw,scale", [((60, 150), 1), ((47, 93), 1), ((90, 200), 2), ((11, 40), 1),
                                      ((375, 1242), 1), ((1080, 1920), 2)],
                         ids=["60x150", "47x93", "90x200s2", "11x40", "375x1242", "1080x1920s2"])
def test_sky_detect_synthetic(kind, hw, scale):
    img = sky_images.make(kind, hw[0], hw[1], seed=5)
    want = oracle.sky_detect(img, scale)
    with SGM(hw[0], hw[1], scale, 32, device=0) as sgm:
        got = sgm.sky_detect(img)
    assert np.array_equal(got, want), int((got != want).sum())


def test_sky_detect_4k():
    img = sky_images.make("horizon", 2160, 3840, seed=1)
    want = oracle.sky_detect(img, 1)
    with SGM(2160, 3840, 1, 256, device=0) as sgm:
        got = sgm.sky_detect(img)
    assert np.array_equal(got, want)
    assert (got == 255).any()


def test_process_with_sky_detect():
    # node.cpp:80-93: detect on both inputs, then process(l, r, sky, sky_beta)
    h, w, D = 96, 300, 64
    left = sky_images.make("horizon", h, w, seed=3)
    right = np.roll(left, -6, axis=1)
    ml, mr = oracle.sky_detect(left), oracle.sky_detect(right)
    assert (ml == 255).any()
    ref = oracle.process(left, right, D, sky_l=ml, sky_r=mr)
    with SGM(h, w, 1, D, device=0, sky_detect=True) as sgm:
        sgm.process(left, right)
        got = sgm.get_lr_disp()
    assert np.array_equal(got.view(np.uint32), ref["lr"].view(np.uint32))


@pytest.mark.parametrize("hw", [(96, 300), (375, 1242), (61, 203)])
def test_process_with_sky_detect_odd_sizes(hw):
    # both views' detections share one launch sequence with per-view scratch;
    # H*W not a multiple of 8 once misaligned the second view's totals
    h, w = hw
    D = 64
    left = sky_images.make("horizon", h, w, seed=7)
    right = np.roll(left, -5, axis=1)
    ml, mr = oracle.sky_detect(left), oracle.sky_detect(right)
    ref = oracle.process(left, right, D, sky_l=ml, sky_r=mr)
    with SGM(h, w, 1, D, device=0, sky_detect=True) as sgm:
        sgm.process(left, right)
        got = sgm.get_lr_disp()
    assert np.array_equal(got.view(np.uint32), ref["lr"].view(np.uint32))
