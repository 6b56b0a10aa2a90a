"""GPU BM solver (src/BM.cpp:9-97) against the CPU oracle, bit-exact."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from stereo_matching_amd import BM, synthetic

pytestmark = pytest.mark.gpu

CASES = [(48, 96, 32, 1, "road"), (40, 120, 64, 1, "noise"), (64, 200, 128, 1, "road"),
         (30, 290, 256, 1, "road"), (50, 98, 32, 2, "road"), (42, 150, 128, 2, "noise"),
         (3, 5, 32, 1, "noise"), (375, 1242, 128, 1, "road")]


@pytest.mark.parametrize("case", CASES, ids=[f"{h}x{w}_D{D}_s{s}_{k}" for h, w, D, s, k in CASES])
def test_bm_matches_oracle(case):
    h, w, D, s, kind = case
    left, right = synthetic.stereo_pair(h, w, D, pair_index=7, kind=kind)
    H, W = h // s, w // s
    sky = synthetic.sky_mask(H, W) if kind == "noise" else None
    want = oracle.bm_process(left, right, D, s, sky=sky)
    with BM(h, w, s, D, device=0) as bm:
        bm.process(left, right, sky, sky)
        raw = bm.get_raw_disp().copy()
        got = bm.get_disp().copy()
    assert np.array_equal(raw.astype(np.int64), want.astype(np.int64))
    # get_disp: post_filter of the integer disparity (BM deviation)
    post = oracle.post_filter(want.astype(np.float32), D, s)
    assert np.array_equal(got.view(np.uint32), post.view(np.uint32))
    if kind == "road" and W >= 2 * D:
        assert (want <= D - 1).mean() > 0.5
