"""The C-ABI multi-GPU exchange (include/sgm_hip.h "multi-GPU")
on the one GPU of a test box: a communicator at world 1, built both ways
(ncclCommInitAll from a device list, ncclCommInitRank from a unique id), and
the gather of HIP-computed maps (dense and pitched, per rank and as one
group) bit-equal to the oracle's maps for those pairs.  The C++ form
(include/sgm_amd/BatchSGM.h) is tested in test_cpp_surface.py."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

H, W, D = 60, 200, 64


@pytest.fixture(scope="module")
def setup():
    import torch

    import oracle
    from stereo_matching_amd import SGM, synthetic
    oracle.build()
    dev = torch.device("cuda", 0)
    pairs = [synthetic.stereo_pair(H, W, D, pair_index=40 + k) for k in range(3)]
    want = [oracle.process(l, r, D)["lr"] for l, r in pairs]
    sgm = SGM(H, W, 1, D, device=0)
    yield torch, dev, sgm, pairs, want
    sgm.close()


def _frame(torch, dev, sgm, pair, pitch=W):
    l, r = (torch.from_numpy(a).to(dev) for a in pair)
    m = torch.zeros((H, pitch), dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)
    sgm.process_device(l.data_ptr(), r.data_ptr(), m.data_ptr(), out_pitch=pitch, stream=None)
    sgm.check()  # the frame is done and valid before its map is gathered
    return m


def _same(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("pitch", [W, W + 24])
def test_gather_world1_init_all(setup, pitch):
    torch, dev, sgm, pairs, want = setup
    from stereo_matching_amd.comm import Comm
    with Comm(devices=[0]) as comm:
        assert (comm.nranks, comm.first_rank, comm.nlocal) == (1, 0, 1)
        root = torch.full((1, H, W), -7.0, dtype=torch.float32, device=dev)
        for k, p in enumerate(pairs):
            m = _frame(torch, dev, sgm, p, pitch)
            comm.gather(0, m.data_ptr(), H, W, root.data_ptr(), pitch=pitch, stream=sgm.stream)
            torch.cuda.synchronize(dev)
            assert _same(root[0].cpu().numpy(), want[k]), k


def test_gather_all_world1(setup):
    torch, dev, sgm, pairs, want = setup
    from stereo_matching_amd.comm import Comm
    with Comm(devices=[0]) as comm:
        root = torch.zeros((1, H, W), dtype=torch.float32, device=dev)
        m = _frame(torch, dev, sgm, pairs[1])
        comm.gather_all([m.data_ptr()], H, W, root.data_ptr(), streams=[sgm.stream])
        torch.cuda.synchronize(dev)
        assert _same(root[0].cpu().numpy(), want[1])


def test_gather_world1_init_rank(setup):
    torch, dev, sgm, pairs, want = setup
    from stereo_matching_amd.comm import Comm, unique_id
    uid = unique_id()
    assert len(uid) == 128
    with Comm(uid=uid, nranks=1, rank=0, device=0) as comm:
        assert (comm.nranks, comm.first_rank, comm.nlocal) == (1, 0, 1)
        root = torch.zeros((1, H, W), dtype=torch.float32, device=dev)
        m = _frame(torch, dev, sgm, pairs[2])
        comm.gather(0, m.data_ptr(), H, W, root.data_ptr(), stream=sgm.stream)
        torch.cuda.synchronize(dev)
        assert _same(root[0].cpu().numpy(), want[2])


def test_gather_argument_checks(setup):
    torch, dev, sgm, pairs, want = setup
    from stereo_matching_amd import SGMError
    from stereo_matching_amd.comm import Comm
    with Comm(devices=[0]) as comm:
        m = torch.zeros((H, W), dtype=torch.float32, device=dev)
        with pytest.raises(SGMError, match="not held"):
            comm.gather(1, m.data_ptr(), H, W, m.data_ptr())
        with pytest.raises(SGMError, match="rank 0 needs d_root_out"):
            comm.gather(0, m.data_ptr(), H, W, 0)
        with pytest.raises(SGMError, match="pitch"):
            comm.gather(0, m.data_ptr(), H, W, m.data_ptr(), pitch=W - 1)
    with pytest.raises(SGMError, match="listed twice"):
        Comm(devices=[0, 0])
    with pytest.raises(SGMError, match="not a HIP ordinal"):
        Comm(devices=[torch.cuda.device_count()])
