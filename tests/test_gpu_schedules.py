"""The frame schedule's variants give the same maps bit for bit.

run_frame (sgm_capi.hip) picks between launch groupings that must not change
results: both views' DSI + horizontal IIR in one launch (cost_h2_kernel) or
one launch per view, and -- for volumes above the 256 MB Infinity Cache --
both views' final passes in one launch (pair_final2_kernel) or one per view.
SGM_CONCURRENT_VIEWS=1 (read at sgm_create) runs the right view on a second
stream with per-view launches; SGM_SPLIT_FINAL=1 (read per frame) keeps the
per-view final passes.  The default schedule is pinned against the oracle by
test_gpu_parity.py / test_gpu_fullsize.py; these tests pin the variants to it.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from stereo_matching_amd import SGM, synthetic

pytestmark = pytest.mark.gpu


def _run(h, w, D, sky_l, sky_r, env):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        left, right = synthetic.stereo_pair(h, w, D, pair_index=5, kind="road")
        mask = synthetic.sky_mask(h, w)
        with SGM(h, w, 1, D, device=0) as s:
            s.process(left, right, mask if sky_l else None, mask if sky_r else None)
            return s.get_lr_disp().copy(), s.get_raw_disp().copy()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _same(a, b):
    assert np.array_equal(np.ascontiguousarray(a[0], np.float32).view(np.uint32),
                          np.ascontiguousarray(b[0], np.float32).view(np.uint32)), "LR map differs"
    assert np.array_equal(a[1], b[1]), "raw WTA map differs"


@pytest.mark.parametrize("h,w,D,sky_l,sky_r", [
    (120, 330, 64, False, False),
    (96, 260, 128, True, True),
    (80, 240, 256, True, True),
    (100, 300, 64, True, False),   # one mask only: per-view cost launches either way
    (375, 1242, 128, True, True),
])
def test_joint_cost_launch_matches_per_view(h, w, D, sky_l, sky_r):
    _same(_run(h, w, D, sky_l, sky_r, {}), _run(h, w, D, sky_l, sky_r, {"SGM_CONCURRENT_VIEWS": "1"}))


def test_joint_final_matches_per_view():
    # 512 x 1056 x 128 f32 = 277 MB per volume: above the Infinity Cache, so
    # the default schedule runs both final passes as one launch
    h, w, D = 512, 1056, 128
    assert h * w * D * 4 > 256 * 1024 * 1024
    _same(_run(h, w, D, False, False, {}), _run(h, w, D, False, False, {"SGM_SPLIT_FINAL": "1"}))
