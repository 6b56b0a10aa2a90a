"""The oracle's three schedules give identical bits (oracle/sgm_oracle.c):
orc_process (10 volumes, the parity checker up to HD256), orc_process_lean
(3 volumes, streamed path states: what the 4K256 GPU parity tests use) and
orc_process_refplace (the reference's OpenMP placement: bench.py's CPU
baseline).  Checked on every golden fixture and on the GPU fuzz shapes, with
non-default P1/P2/uniqueness/LR parameters, at several thread counts.  Also
the LR check's column clamp (the build's choice where SGM.cpp:812 reads
outside the row) and the property that makes it a no-op on pipeline maps."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

import oracle
import pyref
from stereo_matching_amd import synthetic

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
SCHEDULES = ("lean", "refplace")


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _same(a, b):
    assert sorted(a) == sorted(b)
    for k in a:
        x, y = np.asarray(a[k]), np.asarray(b[k])
        assert x.dtype == y.dtype and np.array_equal(x.view(np.uint32), y.view(np.uint32)), k


def _golden():
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz") and not f.startswith("sky_"))


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("name", _golden())
def test_schedule_matches_golden(name, schedule):
    g = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    sky = g["sky"] if meta["sky"] else None
    out = oracle.process(g["left"], g["right"], meta["D"], meta["scale"], sky, sky,
                         blur=meta["blur"], schedule=schedule)
    for key in ("disp", "disp_beta", "sub", "sub_beta", "lr", "final"):
        assert np.array_equal(np.asarray(out[key]).view(np.uint32), g[key].view(np.uint32)), key


def _fuzz_case(k):
    # the shapes and parameters of tests/test_gpu_fuzz.py (same generator)
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


@pytest.mark.parametrize("k", range(24))
def test_schedules_agree_on_fuzz_shapes(k):
    c = _fuzz_case(k)
    h, w, D, s = c["h"], c["w"], c["D"], c["s"]
    left, right = synthetic.stereo_pair(h, w, D, pair_index=100 + c["seed"], kind=c["kind"])
    sky = synthetic.sky_mask(h // s, w // s) if c["sky"] else None
    kw = dict(scale=s, sky_l=sky, sky_r=sky, P1=c["p1"], P2=c["p2"], uniq=c["uniq"],
              lr_dis=c["lr"], blur=c["blur"], views=c["views"])
    ref = oracle.process(left, right, D, **kw)
    for sch in SCHEDULES:
        _same(ref, oracle.process(left, right, D, schedule=sch, **kw))


@pytest.mark.parametrize("schedule", SCHEDULES)
def test_schedule_thread_count_invariance(schedule):
    left, right = synthetic.stereo_pair(70, 300, 64, 5)
    sky = np.zeros((70, 300), np.uint8)
    sky[:9, 40:200] = 255
    n = oracle.max_threads()
    try:
        oracle.set_threads(1)
        a = oracle.process(left, right, 64, sky_l=sky, sky_r=sky, schedule=schedule)
        oracle.set_threads(max(3, n))
        b = oracle.process(left, right, 64, sky_l=sky, sky_r=sky, schedule=schedule)
    finally:
        oracle.set_threads(n)
    _same(a, b)
    _same(a, oracle.process(left, right, 64, sky_l=sky, sky_r=sky))


def test_wta_stale_second_minimum_across_pixels():
    # a pixel whose aggregated costs are all equal has no second minimum: the
    # reference's sec_min_d then keeps the previous pixel's value (SGM.cpp:
    # 374-375, 398-407), which the lean schedule resolves in a sequential pass
    # after a parallel one.  The stale index only matters when min/FLT_MAX >
    # uniqueness, i.e. for a negative ratio: flat images (every cost 0) with
    # uniqueness -1 make every pixel take the initial sec_min_d = D+1 -> invalid
    flat = np.full((10, 40), 77, np.uint8)
    for sch in ("parity",) + SCHEDULES:
        o = oracle.process(flat, flat, 32, uniq=-1.0, schedule=sch)
        assert (o["disp"] == 33).all() and (o["disp_beta"] == 33).all(), sch
    left, right = synthetic.stereo_pair(12, 40, 32, 7, kind="noise")
    for sch in SCHEDULES:
        _same(oracle.process(left, right, 32, uniq=-1.0),
              oracle.process(left, right, 32, uniq=-1.0, schedule=sch))


def test_lr_check_clamps_outside_columns():
    # arbitrary maps (not from compute_subpixel): a negative dl sends the
    # reference's read past the row end (SGM.cpp:812 reads cv::Mat::at(i, col)
    # = the next row's memory, or outside the buffer); the build clamps the
    # column to the row, in the oracle as in lr_kernel
    D = 16
    fl = np.array([[-3.0, -1e30, -np.inf, 5.0, np.nan, 0.4],
                   [2.0, 9.0, -0.5, 3.0, 1.0, 40.0]], np.float32)
    fr = np.array([[0.0, 1.0, 2.0, 3.0, 4.0, -5.0],
                   [7.0, 7.0, -1.0, 1.0, 1.0, 0.0]], np.float32)
    out = oracle.lr_check(fl, fr, D)
    assert np.array_equal(bits(out), bits(pyref.lr_check(fl, fr, D)))
    # (0,0): column (int)(0 + 3) = 3 -> |-3 - 3| > 1 -> D+1; (0,1)/(0,2):
    # clamped to column 5 -> D+1; (0,4): NaN fails j >= dl -> kept;
    # (1,2): 2 - (-0.5) = 2.5 -> column 2 -> |-0.5 - -1| = 0.5 -> kept
    assert out[0, 0] == D + 1 and out[0, 1] == D + 1 and out[0, 2] == D + 1
    assert np.isnan(out[0, 4]) and out[1, 2] == -0.5


@pytest.mark.parametrize("kind", ["road", "noise"])
def test_pipeline_maps_keep_lr_columns_in_row(kind):
    # why the clamp never acts on a frame: compute_subpixel's values are NaN,
    # D+1, an integer d, min(x, D-1) or a parabola vertex near [d-1/2, d+1/2],
    # all >= 0 or NaN, so j >= dl gives 0 <= j - dl/s <= j
    left, right = synthetic.stereo_pair(60, 260, 64, 3, kind=kind)
    sky = np.zeros((60, 260), np.uint8)
    sky[:12] = 255
    o = oracle.process(left, right, 64, sky_l=sky, sky_r=sky, final=False)
    for k in ("sub", "sub_beta"):
        v = o[k][~np.isnan(o[k])]
        assert (v >= 0).all() and (v <= 65).all(), k
