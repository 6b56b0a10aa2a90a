"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar (DESIGN.md "Parity"): bit-exact for every stage -- census words, cost
volumes, path costs, WTA indices, sub-pixel floats, LR-checked floats --
compared as raw bits.  Oracle: oracle/sgm_oracle.c ("parity unpinned": the
reference itself cannot be built here).
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from stereo_matching_amd import SGM, synthetic

pytestmark = pytest.mark.gpu

# (h, w, D, scale, kind, sky, blur)
CASES = [
    (48, 96, 32, 1, "road", False, True),
    (40, 120, 64, 1, "noise", True, True),
    (64, 200, 128, 1, "road", False, True),
    (30, 290, 256, 1, "road", True, True),
    (50, 98, 32, 2, "road", False, True),
    (42, 150, 128, 2, "noise", True, True),
    (20, 70, 64, 1, "road", False, False),   # border-heavy: W just above D
    (3, 5, 32, 1, "noise", False, True),     # smallest legal frame (5x3 window)
    (200, 60, 32, 1, "road", False, True),   # tall: diagonal chains wrap 3+ times (H > W)
    (24, 130, 128, 1, "noise", False, True), # W just above D = 128
    (37, 257, 64, 1, "road", True, True),    # odd sizes with a sky mask
    (9, 300, 256, 1, "noise", False, True),  # few rows: one partial vertical segment
    (130, 66, 64, 2, "noise", True, True),   # tall, decimated, sky
]
IDS = [f"{h}x{w}_D{D}_s{s}_{k}{'_sky' if sk else ''}{'' if b else '_noblur'}"
       for h, w, D, s, k, sk, b in CASES]


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32 if a.dtype == np.float32 else a.dtype)


def assert_bits_equal(got, want, what):
    got = np.asarray(got)
    want = np.asarray(want)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    if got.dtype == np.float32 or want.dtype == np.float32:
        g, w = bits(got.astype(np.float32)), bits(want.astype(np.float32))
    else:
        g, w = got.astype(np.int64), want.astype(np.int64)
    bad = np.flatnonzero(g.ravel() != w.ravel())
    assert bad.size == 0, (f"{what}: {bad.size}/{g.size} mismatches, first at flat index "
                           f"{bad[0]}: got {got.ravel()[bad[0]]!r} want {want.ravel()[bad[0]]!r}")


def make_inputs(h, w, D, s, kind, sky):
    left, right = synthetic.stereo_pair(h, w, D, pair_index=3, kind=kind)
    H, W = h // s, w // s
    m = synthetic.sky_mask(H, W) if sky else None
    return left, right, m


def working(img, s):
    h, w = img.shape
    return np.ascontiguousarray(img[: (h // s) * s: s, : (w // s) * s: s])


@pytest.fixture(scope="module", params=CASES, ids=IDS)
def case(request):
    h, w, D, s, kind, sky, blur = request.param
    left, right, m = make_inputs(h, w, D, s, kind, sky)
    sgm = SGM(h, w, s, D, blur=blur)
    yield dict(h=h, w=w, D=D, s=s, blur=blur, left=left, right=right, sky=m, sgm=sgm)
    sgm.close()


def oracle_census(img, s, blur):
    wimg = working(img, s)
    return oracle.census(oracle.blur(wimg) if blur else wimg, s)


def test_census(case):
    for img in (case["left"], case["right"]):
        got = case["sgm"].stage_census(img)
        assert_bits_equal(got, oracle_census(img, case["s"], case["blur"]), "census")


def test_cost_volumes(case):
    s, D = case["s"], case["D"]
    ctl = oracle_census(case["left"], s, case["blur"])
    ctr = oracle_census(case["right"], s, case["blur"])
    for view in (0, 1):
        raw = oracle.dsi(ctl, ctr, D, s, view, case["sky"])
        hf = oracle.hfilter(raw, 5 // s)
        full = oracle.vfilter(hf, 3 // s)
        sgm = case["sgm"]
        assert_bits_equal(sgm.stage_cost(ctl, ctr, view, case["sky"], filters=0), raw, f"dsi v{view}")
        assert_bits_equal(sgm.stage_cost(ctl, ctr, view, case["sky"], filters=1), hf, f"hfilter v{view}")
        assert_bits_equal(sgm.stage_cost(ctl, ctr, view, case["sky"], filters=3), full, f"vfilter v{view}")


def _cost(case, view=0):
    s, D = case["s"], case["D"]
    ctl = oracle_census(case["left"], s, case["blur"])
    ctr = oracle_census(case["right"], s, case["blur"])
    c = oracle.dsi(ctl, ctr, D, s, view, case["sky"])
    return oracle.vfilter(oracle.hfilter(c, 5 // s), 3 // s)


@pytest.mark.parametrize("direction", range(8), ids=[f"L{k + 1}" for k in range(8)])
def test_path(case, direction):
    cost = _cost(case)
    L, m = case["sgm"].stage_path(direction, cost)
    Lo, mo = oracle.path(cost, direction)
    assert_bits_equal(L, Lo, f"L{direction + 1}")
    assert_bits_equal(m, mo, f"minL{direction + 1}")


def test_aggregate_wta_subpixel(case):
    for view in (0, 1):
        cost = _cost(case, view)
        d, f = case["sgm"].stage_aggregate(cost)
        S = oracle.aggregate([oracle.path(cost, k)[0] for k in range(8)])
        do = oracle.wta(S)
        assert_bits_equal(d, do, f"wta v{view}")
        assert_bits_equal(f, oracle.subpixel(do, S), f"subpixel v{view}")


def test_lr_check(case):
    rng = np.random.default_rng(7)
    H, W, D, s = case["h"] // case["s"], case["w"] // case["s"], case["D"], case["s"]
    fl = (rng.integers(0, D + 2, (H, W)) + rng.uniform(-0.5, 0.5, (H, W))).astype(np.float32)
    fl[rng.random((H, W)) < 0.1] = D + 1
    fl = np.clip(fl, 0, D + 1).astype(np.float32)
    fr = (fl + rng.normal(0, 1.2, (H, W))).astype(np.float32)
    assert_bits_equal(case["sgm"].stage_lr(fl, fr), oracle.lr_check(fl, fr, D, s), "lr")


def test_full_process(case):
    sgm = case["sgm"]
    sgm.process(case["left"], case["right"], case["sky"], case["sky"])
    ref = oracle.process(case["left"], case["right"], case["D"], case["s"], case["sky"],
                         case["sky"], blur=case["blur"])
    assert_bits_equal(sgm.get_raw_disp(), ref["disp"], "raw disp")
    assert_bits_equal(sgm.get_lr_disp(), ref["lr"], "lr-checked disp")
    assert_bits_equal(sgm.get_disp(), ref["final"], "post-filtered disp")
