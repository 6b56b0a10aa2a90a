"""Seeded random frames through the C-ABI against the oracle, bit for bit:
random shapes (down to the 5x3 cost window, W below and above D, both
scales), D, input kinds, sky masks, blur on/off, one or two views, and the
SGM parameters the C-ABI exposes beyond the reference's constants -- P1, P2
(SGM.cpp:27-28: 10, 100), the uniqueness ratio (inc/Solver.h:14: 0.7) and
the LR threshold (inc/Solver.h:16: 1).  The oracle (oracle/sgm_oracle.c)
takes the same parameters.  Every case runs with both bodies of the diagonal
L8 sweep (SGM_SWEEP_SPLIT: the one-wave sweep and the memory-wave + DP-wave
split, which the library picks by volume size), in bands (SGM_BAND_ROWS) and
through the slanted-tile passes (SGM_SLANT; those frames run no L8 sweep, so
their second axis is the output form instead)."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from stereo_matching_amd import SGM, synthetic

pytestmark = pytest.mark.gpu

N_CASES = 24


def _case(k: int):
    rng = np.random.default_rng(0x5EED + k)
    D = int(rng.choice([32, 64, 128, 256]))
    s = int(rng.choice([1, 1, 2]))
    h = int(rng.integers(3 * s, 72 * s + 1))
    w = int(rng.integers(5 * s, 3 * D + 40))
    p1 = int(rng.choice([0, 1, 3, 10, 25]))
    p2 = int(rng.choice([p1, 40, 100, 300]))
    uniq = float(rng.choice([0.5, 0.7, 0.9, 1.0]))
    lr = float(rng.choice([0.0, 1.0, 2.5]))
    return dict(h=h, w=w, D=D, s=s, p1=p1, p2=p2, uniq=uniq, lr=lr,
                kind=str(rng.choice(["road", "noise"])), sky=bool(rng.integers(0, 2)),
                blur=bool(rng.integers(0, 4) > 0), views=int(rng.choice([1, 2, 2])), seed=k)


CASES = [_case(k) for k in range(N_CASES)]


@pytest.mark.parametrize("c", CASES, ids=[
    f"{c['h']}x{c['w']}_D{c['D']}_s{c['s']}_P{c['p1']}-{c['p2']}_u{c['uniq']}_lr{c['lr']}"
    f"_{c['kind']}{'_sky' if c['sky'] else ''}{'' if c['blur'] else '_noblur'}_V{c['views']}"
    for c in CASES])
@pytest.mark.parametrize("split", ["0", "1"], ids=["onewave", "split"])
def test_random_frame(c, split, monkeypatch):
    monkeypatch.setenv("SGM_SWEEP_SPLIT", split)
    _check(c)


@pytest.mark.parametrize("c", CASES, ids=[f"{c['h']}x{c['w']}_D{c['D']}_s{c['s']}_V{c['views']}" for c in CASES])
@pytest.mark.parametrize("rows", ["16", "32"])
def test_random_frame_banded(c, rows, monkeypatch):
    """Bands (the schedule of volumes above the Infinity Cache): the forward
    phase (vfwd, L5, L6) band by band top down, both views' H pairs in one
    launch, then the backward phase (stage B's diagonal pair, L8 and the final
    pass) band by band bottom up, chain and filter states carried across band
    edges."""
    monkeypatch.setenv("SGM_BAND_ROWS", rows)
    _check(c)


def _check(c):
    h, w, D, s = c["h"], c["w"], c["D"], c["s"]
    left, right = synthetic.stereo_pair(h, w, D, pair_index=100 + c["seed"], kind=c["kind"])
    H, W = h // s, w // s
    sky = synthetic.sky_mask(H, W) if c["sky"] else None
    with SGM(h, w, s, D, blur=c["blur"], views=c["views"], p1=c["p1"], p2=c["p2"],
             uniqueness=c["uniq"], lr_max_diff=c["lr"]) as sgm:
        sgm.process(left, right, sky, sky)
        got_map = sgm.get_lr_disp()
        got_raw = sgm.get_raw_disp()
    ref = oracle.process(left, right, D, scale=s, sky_l=sky, sky_r=sky, P1=c["p1"], P2=c["p2"],
                         uniq=c["uniq"], lr_dis=c["lr"], blur=c["blur"], views=c["views"])
    want_map = ref["lr"] if c["views"] == 2 else ref["sub"]
    assert np.array_equal(got_raw.astype(np.int64), ref["disp"].astype(np.int64)), "WTA"
    assert np.array_equal(got_map.view(np.uint32), want_map.view(np.uint32)), "map"


@pytest.mark.parametrize("c", CASES, ids=[f"{c['h']}x{c['w']}_D{c['D']}_s{c['s']}_V{c['views']}" for c in CASES])
@pytest.mark.parametrize("out", ["dense_raw", "pitched_noraw"])
def test_random_frame_slant(c, out, monkeypatch):
    """The slanted-tile schedule (sgm_slant.hip, DESIGN.md "Slanted tiles"):
    vfwd writing C and the full L3 volume, the top-down pass (14-column tiles
    leaning along L5: T56 = L5 + L6, L6 handed to the next tile) beside the H
    pair, then the bottom-up pass (tiles leaning along L7: L4, L7 and L8
    together, states handed between tiles as tagged granules) with the WTA
    and sub-pixel.  Through sgm_process_device, two ways the pass's outputs
    differ: a dense output map with the raw WTA map asked for (a one-view
    frame's sub-pixel map goes straight into the caller's map, and the raw
    map is stored), or a pitched output map without the raw map (the
    sub-pixel map goes to the handle's scratch and is copied out; no raw
    stores)."""
    monkeypatch.setenv("SGM_SLANT", "1")
    _check_device(c, pitch_extra=0 if out == "dense_raw" else 24, want_raw=out == "dense_raw")


def _check_device(c, pitch_extra, want_raw):
    import torch
    h, w, D, s = c["h"], c["w"], c["D"], c["s"]
    left, right = synthetic.stereo_pair(h, w, D, pair_index=100 + c["seed"], kind=c["kind"])
    H, W = h // s, w // s
    sky = synthetic.sky_mask(H, W) if c["sky"] else None
    dev = torch.device("cuda", 0)
    dl, dr = (torch.from_numpy(a).to(dev) for a in (left, right))
    dsky = torch.from_numpy(sky).to(dev) if sky is not None else None
    pitch = W + pitch_extra
    out = torch.empty((H, pitch), dtype=torch.float32, device=dev)
    raw = torch.empty((H, W), dtype=torch.int16, device=dev) if want_raw else None
    torch.cuda.synchronize(dev)
    with SGM(h, w, s, D, blur=c["blur"], views=c["views"], p1=c["p1"], p2=c["p2"],
             uniqueness=c["uniq"], lr_max_diff=c["lr"]) as sgm:
        sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr(), out_pitch=pitch,
                           d_sky_l=dsky.data_ptr() if dsky is not None else 0,
                           d_sky_r=dsky.data_ptr() if dsky is not None else 0,
                           d_raw=raw.data_ptr() if want_raw else 0, stream=None)
        sgm.check()
        got_map = out[:, :W].cpu().numpy()
        got_raw = raw.cpu().numpy().view(np.uint16) if want_raw else None
    ref = oracle.process(left, right, D, scale=s, sky_l=sky, sky_r=sky, P1=c["p1"], P2=c["p2"],
                         uniq=c["uniq"], lr_dis=c["lr"], blur=c["blur"], views=c["views"])
    want_map = ref["lr"] if c["views"] == 2 else ref["sub"]
    if want_raw:
        assert np.array_equal(got_raw.astype(np.int64), ref["disp"].astype(np.int64)), "WTA"
    assert np.array_equal(np.ascontiguousarray(got_map).view(np.uint32), want_map.view(np.uint32)), "map"
