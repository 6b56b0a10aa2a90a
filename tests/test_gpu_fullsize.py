"""GPU parity at BASELINE.json's full sizes, bit for bit against the oracle.

K64 (1242x375, D=64, config 1's frame, both views), K128 (config 2) and
HD256 (1920x1080, D=256, config 3) against orc_process (10 volumes).  4K256
(3840x2160, D=256, config 5's frame) against orc_process_lean, the oracle's
3-volume schedule (25.5 GB instead of 85 GB; bit-identical to orc_process,
tests/test_oracle_schedules.py): both views with sky masks (disp, disp_beta,
F_R, the LR-checked map) and config 5's whole pipeline in one handle (sky
detector on both views + SGM + LR + post_filter + LKRefine).  Plus
size-independent properties: determinism, recovery of the synthetic pair's
known disparity field, and agreement of the banded schedules.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from stereo_matching_amd import SGM, synthetic

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("h,w,D,views", [(375, 1242, 64, 2), (375, 1242, 128, 1),
                                         (375, 1242, 128, 2), (1080, 1920, 256, 2)],
                         ids=["K64_lr", "K128_left", "K128_lr", "HD256_lr"])
def test_fullsize_vs_oracle(h, w, D, views):
    left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
    with SGM(h, w, 1, D, views=views) as sgm:
        sgm.process(left, right)
        got_raw = sgm.get_raw_disp().copy()
        got = sgm.get_lr_disp().copy()
    ref = oracle.process(left, right, D, 1, views=views)
    assert np.array_equal(got_raw.astype(np.int64), ref["disp"].astype(np.int64))
    want = ref["lr"] if views == 2 else ref["sub"]
    mism = int(np.count_nonzero(_bits(got) != _bits(want)))
    assert mism == 0, f"{mism} mismatching pixels"


def _config5_images(h, w, pair_index):
    # a bright, smooth sky band with a wavy horizon above the synthetic road
    left, right = synthetic.stereo_pair(h, w, 256, pair_index=pair_index)
    yy, xx = np.mgrid[0:h, 0:w]
    band = yy < (230 + 140 * np.sin(xx / 500.0)).astype(int)
    left = np.where(band, 200 + (yy // 17) % 2, left).astype(np.uint8)
    right = np.where(band, 200 + (yy // 17) % 2, right).astype(np.uint8)
    return left, right


@pytest.mark.timeout(600)
def test_4k256_lr_vs_lean_oracle():
    """Both views of config 5's frame with the synthetic sky masks (rows <
    H/6), the default schedule (slanted tiles at this size, sgm_capi.hip
    slant_default), against orc_process_lean: WTA
    disparities of both views, F_R and the LR-checked map, bit for bit.  The
    frame contains pixels where the parabola's denominator (a+b)-2c rounds to
    0 (Solver.cpp:589: x = +inf -> std::min -> D-1 while disp < D-1)."""
    h, w, D = 2160, 3840, 256
    left, right = synthetic.stereo_pair(h, w, D, pair_index=1)
    sky = synthetic.sky_mask(h, w)
    ref = oracle.process(left, right, D, sky_l=sky, sky_r=sky, schedule="lean", final=False)
    cancels = (ref["sub"] == D - 1) & (ref["disp"] < D - 1)
    assert cancels.any()
    with SGM(h, w, 1, D, views=2) as sgm:
        sgm.process(left, right, sky, sky)
        got_raw = sgm.get_raw_disp().copy()
        got = sgm.get_lr_disp().copy()
    assert np.array_equal(got_raw.astype(np.int64), ref["disp"].astype(np.int64))
    mism = int(np.count_nonzero(_bits(got) != _bits(ref["lr"])))
    assert mism == 0, f"{mism} mismatching pixels in the LR map"
    with SGM(h, w, 1, D, views=1, view="right") as sgm:
        sgm.process(left, right, None, sky)
        assert np.array_equal(sgm.get_raw_disp().astype(np.int64), ref["disp_beta"].astype(np.int64))
        assert np.array_equal(_bits(sgm.get_lr_disp()), _bits(ref["sub_beta"]))


@pytest.mark.timeout(600)
def test_4k256_config5_pipeline_vs_lean_oracle():
    """config 5 in one handle (node.cpp:80-107 + SGM.cpp:821-824): the sky
    detector on both views, SGM with those masks, LR check, post_filter and
    LKRefine, all on the GPU, against the oracle run stage by stage (sky
    detector, orc_process_lean, post_filter, LKRefine) on the same images."""
    h, w, D = 2160, 3840, 256
    left, right = _config5_images(h, w, 4)
    ml, mr = oracle.sky_detect(left), oracle.sky_detect(right)
    assert (ml == 255).mean() > 0.01 and (mr == 255).mean() > 0.01
    ref = oracle.process(left, right, D, sky_l=ml, sky_r=mr, schedule="lean")
    want = oracle.lk_refine(left, right, ref["final"], D)
    with SGM(h, w, 1, D, sky_detect=True) as sgm:
        assert np.array_equal(sgm.sky_detect(left), ml)
        assert np.array_equal(sgm.sky_detect(right), mr)
        sgm.process(left, right)
        assert np.array_equal(sgm.get_raw_disp().astype(np.int64), ref["disp"].astype(np.int64))
        assert np.array_equal(_bits(sgm.get_lr_disp()), _bits(ref["lr"]))
    with SGM(h, w, 1, D, post_filter=True, lk_refine=True, sky_detect=True) as sgm:
        sgm.process(left, right)
        got = sgm.get_disp().copy()
    mism = int(np.count_nonzero(_bits(got) != _bits(want)))
    assert mism == 0, f"{mism} mismatching pixels"


@pytest.mark.timeout(300)
def test_parabola_denominator_cancels():
    """A tall frame (2160 x 288, D=256, sky rows) whose left view has pixels
    where (a+b)-2c rounds to 0 in compute_subpixel (Solver.cpp:589): the
    vertex is +inf and std::min clamps it to D-1 (a "jump" far from the WTA
    index).  GPU == oracle bit for bit there, including the LR check, whose
    column read then stays inside the row (dl >= 0)."""
    h, w, D = 2160, 288, 256
    left, right = synthetic.stereo_pair(h, w, D, pair_index=9)
    sky = synthetic.sky_mask(h, w)
    ref = oracle.process(left, right, D, sky_l=sky, sky_r=sky, final=False)
    cancels = (ref["sub"] == D - 1) & (ref["disp"] > 0) & (ref["disp"] < D - 1)
    assert cancels.sum() >= 3
    with SGM(h, w, 1, D, views=2) as sgm:
        sgm.process(left, right, sky, sky)
        assert np.array_equal(sgm.get_raw_disp().astype(np.int64), ref["disp"].astype(np.int64))
        assert np.array_equal(_bits(sgm.get_lr_disp()), _bits(ref["lr"]))
    with SGM(h, w, 1, D, views=1) as sgm:
        sgm.process(left, right, sky, sky)
        assert np.array_equal(_bits(sgm.get_lr_disp()), _bits(ref["sub"]))


def test_lr_check_arbitrary_maps():
    """sgm_stage_lr on maps no frame produces (negative, huge, infinite, NaN
    disparities): the column read is clamped to the row exactly as the
    oracle's orc_lr_check (the reference would read another row there)."""
    rng = np.random.default_rng(11)
    h, w, D = 37, 300, 64
    fl = rng.uniform(-80, 80, (h, w)).astype(np.float32)
    fr = rng.uniform(-5, 70, (h, w)).astype(np.float32)
    fl[::5, ::7] = -np.inf
    fl[1::5, ::11] = np.inf
    fl[2::5, ::13] = np.nan
    fl[3::5, ::3] = -3e30
    fl[4::5, ::9] = D + 1
    for scale in (1, 2):
        with SGM(h * scale, w * scale, scale, D) as sgm:
            got = sgm.stage_lr(fl, fr)
        want = oracle.lr_check(fl, fr, D, scale)
        assert np.array_equal(_bits(got), _bits(want)), scale


def test_4k256_properties():
    h, w, D = 2160, 3840, 256
    left, right = synthetic.stereo_pair(h, w, D, pair_index=1)
    sky = synthetic.sky_mask(h, w)
    with SGM(h, w, 1, D, views=2) as sgm:
        sgm.process(left, right, sky, sky)
        lr1 = sgm.get_lr_disp().copy()
        raw1 = sgm.get_raw_disp().copy()
        sgm.process(left, right, sky, sky)
        lr2 = sgm.get_lr_disp().copy()
    # deterministic, bit for bit
    assert np.array_equal(_bits(lr1), _bits(lr2))
    # sky rows: the override forces d = 0 (Solver.cpp:165-178)
    assert np.all(raw1[: h // 6] == 0)
    # LR-checked pixels are either invalid or (almost always) within 1 of the
    # raw WTA index; the parabola (Solver.cpp:592-593) may jump further where
    # its denominator cancels (e.g. next to the 999999-cost sky rows)
    valid = lr1 <= D - 1
    near = np.abs(lr1[valid] - raw1[valid].astype(np.float32)) <= 1.0
    assert near.mean() > 0.999, near.mean()
    # the road field g[i] is recovered on most non-sky textured pixels
    g = synthetic.ground_truth(h, D)
    rows = np.arange(h // 6 + 8, h - 8)
    est = raw1[rows][:, D + 8: w - 8].astype(np.int64)
    hit = np.mean(np.abs(est - g[rows][:, None]) <= 1)
    assert hit > 0.9, hit


@pytest.mark.timeout(300)
def test_4k256_schedules_agree(monkeypatch):
    """config 5's frame through the schedules of a volume above the Infinity
    Cache -- the slanted tiles (the default at this size), forward and
    backward bands (SGM_SLANT=0) and whole-volume passes (SGM_SLANT=0,
    SGM_BAND_ROWS=0, the schedule the oracle pins at K128) -- bit for bit."""
    h, w, D = 2160, 3840, 256
    left, right = synthetic.stereo_pair(h, w, D, pair_index=2)
    sky = synthetic.sky_mask(h, w)
    maps = []
    for env in ({}, {"SGM_SLANT": "0"}, {"SGM_SLANT": "0", "SGM_BAND_ROWS": "0"}):
        for k in ("SGM_BAND_ROWS", "SGM_SLANT"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with SGM(h, w, 1, D, views=2) as sgm:
            sgm.process(left, right, sky, sky)
            maps.append((sgm.get_lr_disp().copy(), sgm.get_raw_disp().copy()))
    for lr, raw in maps[1:]:
        assert np.array_equal(raw, maps[0][1])
        assert np.array_equal(_bits(lr), _bits(maps[0][0]))


def test_k128_full_pipeline_vs_oracle():
    # node.cpp:80-107 at config 2's size: sky detector on both views, SGM,
    # LR check, post_filter, then LKRefine (SGM.cpp:821-824), all on the GPU,
    # against the oracle run stage by stage on the same inputs
    h, w, D = 375, 1242, 128
    left, right = synthetic.stereo_pair(h, w, D, pair_index=2)
    # a bright, smooth sky band so the detector has something to find
    yy, xx = np.mgrid[0:h, 0:w]
    band = yy < (40 + 25 * np.sin(xx / 90.0)).astype(int)
    left = np.where(band, 200 + (yy // 9) % 2, left).astype(np.uint8)
    right = np.where(band, 200 + (yy // 9) % 2, right).astype(np.uint8)
    ml, mr = oracle.sky_detect(left), oracle.sky_detect(right)
    assert (ml == 255).any()
    ref = oracle.process(left, right, D, sky_l=ml, sky_r=mr)
    want = oracle.lk_refine(left, right, ref["final"], D)
    with SGM(h, w, 1, D, post_filter=True, lk_refine=True, sky_detect=True) as sgm:
        sgm.process(left, right)
        got = sgm.get_disp().copy()
    mism = int(np.count_nonzero(_bits(got) != _bits(want)))
    assert mism == 0, f"{mism} mismatching pixels"


def test_4k256_side_stages_vs_oracle():
    # config 5's frame: the SGM map comes from the GPU (the oracle's 4K SGM
    # needs ~76 GB); post_filter, LKRefine and the sky detector are checked
    # bit for bit against the oracle on that map and those images
    h, w, D = 2160, 3840, 256
    left, right = synthetic.stereo_pair(h, w, D, pair_index=3)
    with SGM(h, w, 1, D, views=2) as sgm:
        sgm.process(left, right)
        lr = sgm.get_lr_disp().copy()
        post = sgm.post_filter(lr)
        lk = sgm.lk_refine(left, right, post)
        sky = sgm.sky_detect(left)
    want_post = oracle.post_filter(lr, D)
    assert np.array_equal(_bits(post), _bits(want_post))
    assert np.array_equal(_bits(lk), _bits(oracle.lk_refine(left, right, want_post, D)))
    assert np.array_equal(sky, oracle.sky_detect(left))
