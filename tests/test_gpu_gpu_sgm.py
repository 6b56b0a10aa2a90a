"""stereo_matching_amd.GPU_SGM, the Python mirror of the reference's CUDA
backend class (gpu_sgm/inc/SGM.cuh:23-62): the left view's sub-pixel map
(src/SGM.cpp:32-443) post_filter()ed (gpu_sgm/src/SGM.cu:217-225), equal to
the oracle bit for bit, frame after frame on one handle."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from stereo_matching_amd import GPU_SGM, synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scale,D,kind", [(1, 32, "road"), (1, 128, "noise"), (2, 64, "road"),
                                          (1, 256, "road")])
def test_gpu_sgm_matches_oracle(scale, D, kind):
    h, w = 84, 300
    with GPU_SGM(h, w, scale, D) as g:
        for idx in (11, 12):   # the handle is reused; every frame gets fresh maps
            left, right = synthetic.stereo_pair(h, w, D, pair_index=idx, kind=kind)
            g.process(left, right)
            got = g.get_disp()
            sub = oracle.process(left, right, D, scale=scale, views=1)["sub"]
            want = oracle.post_filter(sub, D, scale=scale)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (idx, D, scale)
            assert np.array_equal(g.get_raw_disp().astype(np.int64),
                                  oracle.process(left, right, D, scale=scale, views=1)["disp"]
                                  .astype(np.int64))
