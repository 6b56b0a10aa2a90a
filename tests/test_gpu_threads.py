"""Several handles used at once from several host threads (a serving process:
one handle per worker thread, each on its own streams).  The reference's
`SGM` object is not reentrant but separate objects are independent
(SURVEY.md section 8b); the library keeps no per-process mutable state a
handle could see from another.  Every frame of every thread must equal the
same handle's frame run alone, bit for bit, including handles of different
frame sizes whose sky detector launches need different LDS sizes."""
from __future__ import annotations

import threading

import numpy as np
import pytest

from stereo_matching_amd import SGM, synthetic

pytestmark = pytest.mark.gpu

# (h, w, D, handle options): frame sizes, D and stage sets all differ
CASES = [
    (60, 200, 64, dict(views=2)),
    (96, 320, 128, dict(views=1)),
    (120, 256, 64, dict(views=2, post_filter=True, lk_refine=True, sky_detect=True)),
    (240, 300, 64, dict(views=2, sky_detect=True)),
    (48, 400, 32, dict(views=2, post_filter=True)),
    (375, 1242, 128, dict(views=1)),
]
FRAMES = 4


def _inputs(k, h, w, D):
    return [synthetic.stereo_pair(h, w, D, pair_index=10 * k + f) for f in range(FRAMES)]


def _run(k, out, errors, barrier=None):
    h, w, D, opts = CASES[k]
    try:
        if barrier:
            barrier.wait(timeout=120)
        with SGM(h, w, 1, D, **opts) as sgm:
            res = []
            for left, right in _inputs(k, h, w, D):
                sgm.process(left, right)
                res.append((sgm.get_disp().copy(), sgm.get_raw_disp().copy()))
        out[k] = res
    except Exception as e:  # noqa: BLE001 -- reported by the main thread
        errors.append((k, repr(e)))


@pytest.mark.timeout(300)
def test_handles_on_threads_match_serial():
    alone = {}
    errors = []
    for k in range(len(CASES)):
        _run(k, alone, errors)
    assert not errors, errors
    together = {}
    barrier = threading.Barrier(len(CASES))
    threads = [threading.Thread(target=_run, args=(k, together, errors, barrier))
               for k in range(len(CASES))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads)
    assert not errors, errors
    for k in range(len(CASES)):
        for f in range(FRAMES):
            (a_map, a_raw), (t_map, t_raw) = alone[k][f], together[k][f]
            assert np.array_equal(a_map.view(np.uint32), t_map.view(np.uint32)), (CASES[k], f)
            assert np.array_equal(a_raw, t_raw), (CASES[k], f)
