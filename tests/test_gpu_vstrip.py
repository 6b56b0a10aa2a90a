"""The strip pass of the slanted schedule (sgm_vstrip.hip):
checkpoints of the horizontal IIR at every 24-column strip edge
(launch_cost_ck), then one pass that runs the horizontal IIR across each
strip from its checkpoint, the vertical IIR and the L3 forward pass, writing
C and the L3 volume.  It replaces cost_h + vfwd_l3 on slanted frames
(SGM_VSTRIP=0 restores those), so the maps must be bit-identical to the
oracle and to the two-pass path -- at the strip edges where the horizontal
filter's boundary columns meet the strips: W below, at and just above one
strip, a strip starting at W-3 (its first column is the last filtered one,
read from a checkpoint with no update after it), at W-2 and W-1 (raw columns
only), the 3-row and 5-column minimum frame, each D, one and two views, the
right-view handle, sky masks (staged as one word per pixel), and scale 2,
where the strip pass does not apply and the two-pass path runs."""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle
from stereo_matching_amd import SGM, synthetic

pytestmark = pytest.mark.gpu

CASES = [
    # h, w, s, D, views, sky
    (3, 5, 1, 32, 2, False),      # the minimum frame, one partial strip
    (4, 23, 1, 64, 2, False),     # W below one strip
    (5, 24, 1, 64, 1, False),     # W = one strip
    (7, 25, 1, 128, 2, False),    # strip 1 = column W-1 (raw)
    (9, 26, 1, 128, 2, False),    # strip 1 starts at W-2 (raw)
    (10, 27, 1, 256, 2, False),   # strip 1 starts at W-3 (checkpoint, no update)
    (11, 28, 1, 256, 1, False),   # strip 1 starts at W-4
    (33, 300, 1, 32, 2, False),
    (20, 70, 1, 64, 2, True),     # sky masks
    (40, 97, 1, 64, 2, True),
    (64, 200, 1, 256, 2, True),
    (50, 241, 1, 128, 1, False),
    (40, 100, 2, 64, 2, True),    # scale 2: the two-pass path
]


def _run(c, env, view="left"):
    h, w, s, D, views, use_sky = c
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        left, right = synthetic.stereo_pair(h, w, D, pair_index=7, kind="road")
        H, W = h // s, w // s
        sky = synthetic.sky_mask(H, W) if use_sky else None
        with SGM(h, w, s, D, views=views, view=view) as sgm:
            sgm.set_profiling(True)
            sgm.process(left, right, sky, sky)
            prof = sgm.get_profile()
            return sgm.get_lr_disp().copy(), sgm.get_raw_disp().copy(), prof, (left, right, sky)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("c", CASES, ids=[f"{c[0]}x{c[1]}_s{c[2]}_D{c[3]}_V{c[4]}{'_sky' if c[5] else ''}"
                                          for c in CASES])
def test_strips_vs_oracle_and_two_pass(c):
    h, w, s, D, views, _ = c
    m, raw, prof, (left, right, sky) = _run(c, {"SGM_SLANT": "1"})
    strips = s == 1
    assert ("vstrip" in prof) == strips and ("vfwd_l3" in prof) == (not strips), sorted(prof)
    ref = oracle.process(left, right, D, scale=s, sky_l=sky, sky_r=sky, views=views)
    want = ref["lr"] if views == 2 else ref["sub"]
    assert np.array_equal(raw.astype(np.int64), ref["disp"].astype(np.int64)), "WTA"
    assert np.array_equal(m.view(np.uint32), want.view(np.uint32)), "map"
    m2, raw2, prof2, _ = _run(c, {"SGM_SLANT": "1", "SGM_VSTRIP": "0"})
    assert "vstrip" not in prof2 and "vfwd_l3" in prof2, sorted(prof2)
    assert np.array_equal(m.view(np.uint32), m2.view(np.uint32))
    assert np.array_equal(raw, raw2)


@pytest.mark.parametrize("c", [(30, 130, 1, 128, 1, True), (12, 49, 1, 256, 1, False)],
                         ids=["130_D128_sky", "49_D256"])
def test_right_view_handle(c):
    # a right-view handle runs the right-view DSI in slot 0 (dsi0 = 1)
    m, raw, prof, _ = _run(c, {"SGM_SLANT": "1"}, view="right")
    assert "vstrip" in prof, sorted(prof)
    m2, raw2, _, _ = _run(c, {"SGM_SLANT": "1", "SGM_VSTRIP": "0"}, view="right")
    assert np.array_equal(m.view(np.uint32), m2.view(np.uint32))
    assert np.array_equal(raw, raw2)
