"""GPU consumers of the disparity map against numpy restatements, bit-exact:
Solver::colormap (src/Solver.cpp:652-707) and the point cloud of
node.cpp:119-143.  Also the aux_only light handle the C++ wrappers use."""
from __future__ import annotations

import numpy as np
import pytest

import postfilter_maps
import pyref
from stereo_matching_amd import SGM, SGMError, synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D", [32, 64, 128, 256])
def test_colormap(D):
    H, W = 40, 300
    F = postfilter_maps.make("random_holes", H, W, D, 3)
    F[0, :D] = np.arange(D, dtype=np.float32)            # every integer band edge
    F[1, :10] = (np.array([51, 51.1, 102, 102.5, 153, 153.2, 204, 204.9, 0, D - 1], np.float32)
                 / np.float32(256 // D))
    with SGM(H, W, 1, D, device=0, aux_only=True) as sgm:
        got = sgm.colormap(F)
    assert np.array_equal(got, pyref.colormap(F, D))


@pytest.mark.parametrize("scale", [1, 2])
def test_point_cloud(scale):
    h, w, D = 60 * scale, 150 * scale, 64
    left, right = synthetic.stereo_pair(h, w, D, pair_index=1, kind="road")
    with SGM(h, w, scale, D, device=0) as sgm:
        sgm.process(left, right)
        F = sgm.get_disp().copy()
        F[5, :7] = np.float32([0.0, 0.004, 1.0, 2.5, D + 1, D + 0.5, 63.0])  # Z cut-offs, invalid
        xyz, pix = sgm.point_cloud(F, left, 721.5377, 721.5377, 609.5593, 172.854)
    want_xyz, want_pix = pyref.point_cloud(F, left, D, scale, 721.5377, 721.5377, 609.5593, 172.854)
    assert xyz.shape == want_xyz.shape and xyz.shape[0] > 0
    assert np.array_equal(xyz.view(np.uint64), want_xyz.view(np.uint64))
    assert np.array_equal(pix, want_pix)


def test_aux_only_handle():
    # a light handle: the side stages run, the SGM frame refuses
    h, w, D = 48, 96, 32
    left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
    with SGM(h, w, 1, D, device=0, aux_only=True) as aux, SGM(h, w, 1, D, device=0) as full:
        assert aux.device_bytes < full.device_bytes / 4
        with pytest.raises(SGMError):
            aux.process(left, right)
        full.process(left, right)
        lr = full.get_lr_disp()
        assert np.array_equal(aux.post_filter(lr).view(np.uint32), full.get_disp().view(np.uint32))
        assert np.array_equal(aux.sky_detect(left), full.sky_detect(left))
