"""A frame captured once as a HIP graph (torch.cuda.graph on the handle's own
stream) and replayed: the replay computes what an eager sgm_process_device
call computes, from whatever the captured input buffers hold at replay time
(a serving loop that refills fixed buffers).  bench.py --graph times this;
profiles/r03_experiments/hip_graph.txt measured it equal to eager launches."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from stereo_matching_amd import SGM, synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(120)
@pytest.mark.parametrize("h,w,D,views,sky,slant", [(96, 320, 64, 2, False, False),
                                                   (375, 1242, 128, 1, False, False),
                                                   (120, 256, 128, 2, True, False),
                                                   # the slanted passes: their tickets and
                                                   # granule tags live on the device and move
                                                   # on every launch, replays included
                                                   (96, 320, 64, 2, False, True),
                                                   (120, 256, 256, 2, True, True),
                                                   (80, 200, 128, 1, False, True)])
def test_frame_replays_from_a_hip_graph(h, w, D, views, sky, slant, monkeypatch):
    monkeypatch.setenv("SGM_SLANT", "1" if slant else "0")
    dev = torch.device("cuda", 0)
    with SGM(h, w, 1, D, views=views) as sgm:
        stream = torch.cuda.ExternalStream(sgm.stream, device=dev)
        d_l = torch.empty((h, w), dtype=torch.uint8, device=dev)
        d_r = torch.empty_like(d_l)
        d_sky = torch.from_numpy(synthetic.sky_mask(h, w)).to(dev) if sky else None
        skyp = d_sky.data_ptr() if sky else 0
        out_e = torch.empty((h, w), dtype=torch.float32, device=dev)
        out_g = torch.empty_like(out_e)

        def frame(out):
            sgm.process_device(d_l.data_ptr(), d_r.data_ptr(), out.data_ptr(), d_sky_l=skyp,
                               d_sky_r=skyp if views == 2 else 0, stream=stream.cuda_stream)

        def load(k):
            left, right = synthetic.stereo_pair(h, w, D, pair_index=k)
            with torch.cuda.stream(stream):
                d_l.copy_(torch.from_numpy(left))
                d_r.copy_(torch.from_numpy(right))

        load(0)
        with torch.cuda.stream(stream):
            frame(out_e)  # warm-up (the capture needs no first-call work)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream, capture_error_mode="relaxed"):
            frame(out_g)
        torch.cuda.synchronize(dev)
        for k in (1, 2, 3):
            load(k)
            with torch.cuda.stream(stream):
                graph.replay()
                frame(out_e)
            torch.cuda.synchronize(dev)
            g, e = out_g.cpu().numpy(), out_e.cpu().numpy()
            assert np.array_equal(g.view(np.uint32), e.view(np.uint32)), k


@pytest.mark.timeout(120)
def test_capture_with_post_filter_is_rejected():
    # post_filter's median-fill launch count comes from a counter read back to
    # the host each round, which a capture never runs: the library refuses
    # the capture instead of recording a fixed fill, and the
    # handle keeps working eagerly afterwards
    from stereo_matching_amd import SGMError
    import oracle
    h, w, D = 96, 320, 64
    dev = torch.device("cuda", 0)
    left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
    with SGM(h, w, 1, D, views=2, post_filter=True) as sgm:
        stream = torch.cuda.ExternalStream(sgm.stream, device=dev)
        d_l = torch.from_numpy(left).to(dev)
        d_r = torch.from_numpy(right).to(dev)
        out = torch.empty((h, w), dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)

        def frame():
            sgm.process_device(d_l.data_ptr(), d_r.data_ptr(), out.data_ptr(),
                               stream=stream.cuda_stream)

        graph = torch.cuda.CUDAGraph()
        with pytest.raises(SGMError, match="HIP graph"):
            with torch.cuda.graph(graph, stream=stream, capture_error_mode="relaxed"):
                frame()
        torch.cuda.synchronize(dev)
        with torch.cuda.stream(stream):
            frame()
        torch.cuda.synchronize(dev)
        want = oracle.process(left, right, D)["final"]
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
