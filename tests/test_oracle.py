"""CPU tests of the oracle (oracle/sgm_oracle.c).

The reference ships no tests or golden vectors and cannot be built here, so
the oracle is pinned by (1) an independent numpy restatement (tests/pyref.py),
(2) hand-derived known answers for each stage, and (3) the committed golden
fixtures in tests/golden/ (regression vectors produced by
tests/golden/make_golden.py).  Parity status: "parity unpinned" (DESIGN.md),
except the sky detector, pinned by the reference's own example output
(tests/golden/sky_000017_14.npz, tests/golden/make_sky_golden.py).
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import pyref
from stereo_matching_amd import synthetic

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


# ------------------------------------------------------- known answers

def test_census_known_answer():
    # constant image: no neighbour is brighter -> all-zero words
    img = np.full((9, 11), 77, np.uint8)
    assert not oracle.census(img).any()
    # single bright pixel at (4,5): the centre pixel sees it at window offset
    # (0,+1) -> bit index (row 3 of 7, col 5 of 9) in MSB-first order with the
    # centre skipped: position 3*9+5 = 32, minus 1 for the skipped centre = 31
    # counted from the first bit; 62 bits total -> value bit 62-1-31 = 30.
    img = np.zeros((9, 11), np.uint8)
    img[4, 5] = 200
    ct = oracle.census(img)
    assert ct[4, 4] == np.uint64(1) << np.uint64(30)
    # the bright pixel itself sees nothing brighter
    assert ct[4, 5] == 0
    # 62 significant bits at scale 1, 14 at scale 2 (cost.cpp:107-122)
    img = np.zeros((9, 11), np.uint8)
    img[4, 5] = 0
    ones = np.full((9, 11), 255, np.uint8)
    ones[4, 5] = 0
    assert int(oracle.census(ones)[4, 5]) == (1 << 62) - 1
    assert int(oracle.census(ones, 2)[4, 5]) == (1 << 14) - 1


def test_census_edge_clamp():
    # coordinates are clamped (cost.cpp:109-118): at the corner the window
    # repeats the edge pixels instead of reading outside the image
    img = np.arange(30, dtype=np.uint8).reshape(5, 6) * 7
    want = pyref.census(img)
    assert np.array_equal(oracle.census(img), want)


def test_blur_known_answer():
    # constant 100: kernel sum 257*256 -> (100*65792 + 32768) >> 16 = 100
    img = np.full((5, 7), 100, np.uint8)
    assert (oracle.blur(img) == 100).all()
    # saturation: 255 * 65792 / 65536 rounds to 256 -> clamped to 255
    assert (oracle.blur(np.full((4, 4), 255, np.uint8)) == 255).all()
    # impulse response at the centre = round(116*93*200 / 65536) etc.
    img = np.zeros((5, 5), np.uint8)
    img[2, 2] = 200
    out = oracle.blur(img)
    assert out[2, 2] == (116 * 93 * 200 + 32768) >> 16
    assert out[2, 1] == (116 * 82 * 200 + 32768) >> 16
    assert out[1, 2] == (70 * 93 * 200 + 32768) >> 16
    assert out[1, 1] == (70 * 82 * 200 + 32768) >> 16
    # REFLECT_101 at the border: column -1 reads column 1
    img = np.zeros((3, 4), np.uint8)
    img[:, 1] = 100
    # column 0: both horizontal neighbours are column 1 -> (82+82)*100 per row,
    # rows sum to 256 -> (256*164*100 + 32768) >> 16
    assert oracle.blur(img)[1, 0] == (256 * 164 * 100 + 32768) >> 16
    assert np.array_equal(oracle.blur(img), pyref.blur(img))


def test_dsi_known_answer():
    ctl = np.array([[0b1011, 0b0001, 0b1111]], np.uint64)
    ctr = np.array([[0b0000, 0b0011, 0b0111]], np.uint64)
    c = oracle.dsi(ctl, ctr, 4, 1, 0)
    # left view: C[j,d] = popcount(ctl[j] ^ ctr[max(j-d,0)])
    assert c[0, 2].tolist() == [1, 2, 4, 4]
    c = oracle.dsi(ctl, ctr, 4, 1, 1)
    # right view: C[j,d] = popcount(ctl[min(j+d,W-1)] ^ ctr[j])
    assert c[0, 0].tolist() == [3, 1, 4, 4]
    sky = np.array([[0, 255, 0]], np.uint8)
    c = oracle.dsi(ctl, ctr, 4, 1, 0, sky)
    assert c[0, 1].tolist() == [0, 999999, 999999, 999999]


def test_hfilter_is_the_reference_iir_not_a_box():
    # one row, D=1: the in-place recurrence of Solver.cpp:296-330
    a = np.array([[[5.], [0.], [10.], [0.], [0.], [20.], [0.], [0.]]], np.float32)
    got = oracle.hfilter(a, 5)[0, :, 0]
    r = a[0, :, 0].astype(np.float32).copy()
    s = np.float32(0)
    for k in range(5):
        s = np.float32(s + r[k])
    out = r.copy()
    for j in range(2, 6):
        out[j] = np.float32(s / np.float32(5))
        if j == 5:
            break
        s = np.float32(s + out[j + 3])
        s = np.float32(s - out[j - 2])
    assert np.array_equal(got, out)
    # edges stay raw; from j=5 on the window subtracts an already filtered
    # value (a[2] = 3, not 10): 27/5 = 5.4 where a box filter gives 20/5 = 4
    assert got[0] == 5 and got[1] == 0 and got[6] == 0 and got[7] == 0
    assert got[5] == np.float32(27) / np.float32(5)
    assert got[5] != np.float32((0 + 0 + 20 + 0 + 0) / 5)


def test_path_known_answer():
    # W=3, D=3, one row, direction L1 (left -> right)
    cost = np.array([[[1, 5, 9], [4, 0, 8], [7, 7, 0]]], np.float32)
    L, m = oracle.path(cost, oracle.L1, P1=10, P2=100)
    assert L[0, 0].tolist() == [1, 5, 9]
    # j=1: prev=[1,5,9], minp=1:
    # d0: min(1, 5+10, 1+100)=1 -> 1+(4-1)=4 ; d1: min(5, 1+10, 9+10, 101)=5 -> 5+(0-1)=4
    # d2: min(9, 5+10, 9+10, 101) = 9 -> 9+(8-1)=16
    assert L[0, 1].tolist() == [4, 4, 16]
    assert m[0, 1] == 4
    L2, _ = oracle.path(cost, oracle.L2, P1=10, P2=100)
    assert L2[0, 2].tolist() == [7, 7, 0]


def test_wta_ties_and_uniqueness():
    S = np.array([[[3, 1, 1, 5],      # tie: first index wins -> 1; second min 3 at d=0
                   [2, 2, 2, 2],      # all equal: no second minimum -> d=0 valid
                   [10, 9, 50, 9.5],  # 9/9.5 > 0.7 and |1-3| > 1 -> invalid (D+1)
                   [10, 9, 9.5, 50]]], np.float32)  # 9/9.5 > 0.7 but |1-2| = 1 -> 1
    d = oracle.wta(S)
    assert d.tolist() == [[1, 0, 5, 1]]
    sub = oracle.subpixel(d, S)
    assert sub[0, 1] == 0 and sub[0, 2] == 5
    x = np.float32(1) + (np.float32(3) - np.float32(1)) / (
        np.float32(2) * ((np.float32(3) + np.float32(1)) - np.float32(2) * np.float32(1)))
    assert sub[0, 0] == x


def test_lr_known_answer():
    D = 8
    fl = np.array([[0, 0, 9, 2.4, 3.0, 1.0]], np.float32)
    fr = np.array([[2.0, 0, 5.0, 0, 2.0, 1.0]], np.float32)
    out = oracle.lr_check(fl, fr, D)
    # j=0: FR[0]=2 -> |0-2|>1 -> D+1 ; j=2: 2 < 9 -> untouched
    # j=3: dl=2.4 -> FR[(int)(0.6)=0]=2 -> |0.4| kept ; j=4: FR[1]=0 -> D+1
    # j=5: FR[4]=2 -> |1-2| = 1 is not > 1 -> kept
    assert np.array_equal(out, np.array([[9, 0, 9, 2.4, 9, 1]], np.float32))
    assert np.array_equal(out, pyref.lr_check(fl, fr, D))


def test_post_filter_speckle_and_median():
    D = 16
    F = np.full((40, 40), 5.0, np.float32)    # one 1600-px component: kept
    F[10:14, 10:14] = 12.0                      # 16-px island: removed (<= 1000)
    F[30, 30] = D + 1                           # isolated invalid: median-filled to 5
    out = oracle.post_filter(F, D)
    assert out[30, 30] == 5
    assert (out[10:14, 10:14] == D + 1).all()
    assert out[0, 0] == 5
    assert np.array_equal(out, pyref.post_filter(F, D))


# ----------------------------------------- oracle vs numpy restatement

CASES = [(24, 40, 16, 1, "road", False), (20, 48, 32, 1, "noise", True),
         (26, 44, 16, 2, "road", False), (15, 37, 32, 1, "road", True),
         (3, 5, 8, 1, "noise", False)]


@pytest.mark.parametrize("h,w,D,s,kind,sky", CASES)
def test_oracle_matches_pyref(h, w, D, s, kind, sky):
    l, r = synthetic.stereo_pair(h, w, max(D, 16), 1, kind)
    H, W = h // s, w // s
    l2, r2 = l[: H * s: s, : W * s: s], r[: H * s: s, : W * s: s]
    m = synthetic.sky_mask(H, W) if sky else None
    bl = pyref.blur(l2)
    assert np.array_equal(bl, oracle.blur(l2))
    cl = pyref.census(bl, s)
    assert np.array_equal(cl, oracle.census(bl, s))
    cr = pyref.census(pyref.blur(r2), s)
    subs = []
    for view in (0, 1):
        c1 = pyref.dsi(cl, cr, D, s, view, m)
        assert np.array_equal(c1, oracle.dsi(cl, cr, D, s, view, m))
        h1 = pyref.hfilter(c1, 5 // s)
        assert np.array_equal(bits(h1), bits(oracle.hfilter(c1, 5 // s)))
        v1 = pyref.vfilter(h1, 3 // s)
        assert np.array_equal(bits(v1), bits(oracle.vfilter(h1, 3 // s)))
        Ls = []
        for k in range(8):
            a, am = pyref.path(v1, k)
            b, bm = oracle.path(v1, k)
            assert np.array_equal(bits(a), bits(b)), k
            assert np.array_equal(bits(am), bits(bm)), k
            Ls.append(b)
        S = oracle.aggregate(Ls)
        assert np.array_equal(bits(pyref.aggregate(Ls)), bits(S))
        d = oracle.wta(S)
        assert np.array_equal(pyref.wta(S), d)
        f = oracle.subpixel(d, S)
        assert np.array_equal(bits(pyref.subpixel(d, S)), bits(f))
        subs.append(f)
    lr = oracle.lr_check(subs[0], subs[1], D, s)
    assert np.array_equal(bits(pyref.lr_check(subs[0], subs[1], D, s)), bits(lr))
    full = oracle.process(l, r, D, s, m, m)
    assert np.array_equal(bits(full["lr"]), bits(lr))
    assert np.array_equal(bits(full["final"]), bits(pyref.post_filter(lr, D, s)))


def test_oracle_thread_count_invariance():
    l, r = synthetic.stereo_pair(40, 96, 32, 0)
    n = oracle.max_threads()
    try:
        oracle.set_threads(1)
        a = oracle.process(l, r, 32)
        oracle.set_threads(max(2, n))
        b = oracle.process(l, r, 32)
    finally:
        oracle.set_threads(n)
    for k in a:
        assert np.array_equal(np.asarray(a[k]).view(np.uint32), np.asarray(b[k]).view(np.uint32))


# ------------------------------------------------------ golden fixtures

def _golden_files():
    if not os.path.isdir(GOLDEN):
        return []
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz") and not f.startswith("sky_"))


@pytest.mark.parametrize("name", _golden_files())
def test_oracle_against_golden(name):
    g = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    sky = g["sky"] if meta["sky"] else None
    out = oracle.process(g["left"], g["right"], meta["D"], meta["scale"], sky, sky,
                         blur=meta["blur"])
    for key in ("disp", "disp_beta", "sub", "sub_beta", "lr", "final"):
        assert np.array_equal(np.asarray(out[key]).view(np.uint32), g[key].view(np.uint32)), key
    with open(os.path.join(GOLDEN, "hashes.json")) as fh:
        hashes = json.load(fh)[name]
    s, D = meta["scale"], meta["D"]
    H, W = g["left"].shape[0] // s, g["left"].shape[1] // s
    wl = g["left"][: H * s: s, : W * s: s]
    wr = g["right"][: H * s: s, : W * s: s]
    if meta["blur"]:
        wl, wr = oracle.blur(wl), oracle.blur(wr)
    cl, cr = oracle.census(wl, s), oracle.census(wr, s)
    assert hashlib.sha256(cl.tobytes()).hexdigest() == hashes["census_l"]
    cost = oracle.vfilter(oracle.hfilter(oracle.dsi(cl, cr, D, s, 0, sky), 5 // s), 3 // s)
    assert hashlib.sha256(cost.tobytes()).hexdigest() == hashes["cost_l"]
    for k in range(8):
        L, _ = oracle.path(cost, k)
        assert hashlib.sha256(L.tobytes()).hexdigest() == hashes[f"L{k + 1}"], k


@pytest.mark.parametrize("kind", __import__("postfilter_maps").KINDS)
def test_post_filter_oracle_vs_numpy_on_stress_maps(kind):
    # the oracle's sequential median fill + component test against the
    # independent numpy restatement, on the maps the GPU parity tests use
    import postfilter_maps
    for (H, W, D, s) in ((40, 90, 64, 1), (23, 70, 32, 2)):
        F = postfilter_maps.make(kind, H, W, D, 1)
        got = oracle.post_filter(F.copy(), D, s)
        want = pyref.post_filter(F, D, s)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (kind, H, W)


def test_post_filter_median_fill_is_sequential():
    # Known answer: the in-place raster order of Solver.cpp:604-630.  Row 5
    # holds an invalid run; (5, 3) is filled first and its value joins the
    # window of (5, 4), so the run fills left to right from earlier fills.
    # 40x40 (one component of 1600 > 1000 pixels, so the speckle pass keeps it)
    D = 64
    F = np.zeros((40, 40), np.float32)
    F[:, :] = np.arange(40, dtype=np.float32)[None, :]   # column index as disparity
    F[5, 2:9] = D + 1
    out = oracle.post_filter(F.copy(), D)
    assert np.array_equal(out.view(np.uint32), pyref.post_filter(F, D).view(np.uint32))
    # (5,2): 4 full rows {0..4} + (5,0), (5,1) = 22 samples, v[11] = 2; (5,3)
    # then sees the fill 2 at (5,2): {1..5}x4 + {1, 2}, v[11] = 3; and so on
    assert np.array_equal(out[5, 2:9], np.arange(2, 9, dtype=np.float32))
    # a second run right below: row 5's fills are in row 6's windows
    G = F.copy()
    G[6, 3:6] = D + 1
    out = oracle.post_filter(G.copy(), D)
    assert np.array_equal(out.view(np.uint32), pyref.post_filter(G, D).view(np.uint32))


@pytest.mark.parametrize("kind", ["road", "noise"])
def test_lk_refine_oracle_vs_numpy(kind):
    # LKRefine (LKSubPixelImpl.cpp:56-235) on the map SGM::process hands it
    # (post-filtered, SGM.cpp:821-824), C oracle vs the numpy restatement
    from stereo_matching_amd import synthetic
    h, w, D = 30, 72, 32
    left, right = synthetic.stereo_pair(h, w, D, pair_index=1, kind=kind)
    ref = oracle.process(left, right, D, blur=False)
    disp = ref["final"]
    got = oracle.lk_refine(left, right, disp, D)
    want = pyref.lk_refine(left, right, disp, D)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    inner = np.s_[3:-3, 3:-3]
    # interior: truncated or refined; border: untouched
    assert np.array_equal(got[:3].view(np.uint32), disp[:3].view(np.uint32))
    if kind == "road":
        assert (got[inner] != np.trunc(disp[inner])).any()


def test_lk_refine_known_answer():
    # A pure shift by 5 on a ramp (Ix = 3 > 2): R(x - 5) = L(x), so every
    # slot has Ires = 0, doff = 0 after one iteration, and a truncated
    # disparity of 5 (from 5.7) is the answer.
    H, W, D = 20, 60, 32
    L = np.tile((np.arange(W) * 3) % 256, (H, 1)).astype(np.uint8)
    R = np.zeros_like(L)
    R[:, :W - 5] = L[:, 5:]
    disp = np.full((H, W), 5.7, np.float32)
    got = oracle.lk_refine(L, R, disp, D)
    assert np.array_equal(got.view(np.uint32), pyref.lk_refine(L, R, disp, D).view(np.uint32))
    assert np.allclose(got[3:-3, 3:-3][:, 3:W - 15], 5.0)


def test_sky_detect_reproduces_reference_example():
    # golden: the reference's own detect() output for example/000017_14
    # (tests/golden/make_sky_golden.py recovers input and mask from its PNGs)
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "sky_000017_14.npz"))
    got = oracle.sky_detect(g["image"])
    assert np.array_equal(got, g["mask"]), int((got != g["mask"]).sum())
    assert np.array_equal(pyref.sky_detect(g["image"]), g["mask"])


@pytest.mark.parametrize("kind", __import__("sky_images").KINDS)
@pytest.mark.parametrize("hw,scale", [((60, 150), 1), ((47, 93), 1), ((90, 200), 2), ((11, 40), 1)])
def test_sky_detect_oracle_vs_numpy(kind, hw, scale):
    import sky_images
    img = sky_images.make(kind, hw[0], hw[1], seed=2)
    assert np.array_equal(oracle.sky_detect(img, scale), pyref.sky_detect(img, scale)), kind


@pytest.mark.parametrize("scale,kind", [(1, "road"), (1, "noise"), (2, "road")])
def test_bm_oracle_vs_numpy(scale, kind):
    # BM::process (BM.cpp:9-97), including its unstrided-row decimation
    from stereo_matching_amd import synthetic
    h, w, D = 28 * scale, 70 * scale, 32
    left, right = synthetic.stereo_pair(h, w, D, pair_index=2, kind=kind)
    got = oracle.bm_process(left, right, D, scale)
    want = pyref.bm_process(left, right, D, scale)
    assert np.array_equal(got, want)
    if kind == "road":
        assert (got <= D - 1).mean() > 0.5
