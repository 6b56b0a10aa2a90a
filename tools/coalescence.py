"""Exact (bitwise) coalescence of SGM path states: how many steps a path
started from the zero-state at an arbitrary column needs before its state
vector equals the true path's, bit for bit (SGM.cpp:81-159's L1/L2 recurrence,
fp32 in the reference's operation order, checked against oracle.path).

A path split into segments with warm-up (the idea behind segmented H pairs in
bands) is exact only where that happens inside the warm-up.  Usage:
  python tools/coalescence.py D [sky] [--synthetic]
Input: the KITTI left image of tests/golden/sky_000017_14.npz, right image =
left shifted by the synthetic road field (or the synthetic noise pair).
Results: profiles/r03_experiments/coalescence.txt
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from stereo_matching_amd import synthetic  # noqa: E402

P1, P2 = np.float32(10), np.float32(100)


def step(Lp, c):
    """One L1 step for every row at once: SGM.cpp:102-105 in its order."""
    m = Lp.min(axis=-1, keepdims=True)
    dm = np.concatenate([Lp[..., :1], Lp[..., :-1]], -1)
    dp = np.concatenate([Lp[..., 1:], Lp[..., -1:]], -1)
    x = np.minimum(Lp, dm + P1)
    x = np.minimum(x, dp + P1)
    x = np.minimum(x, m + P2)
    return x + (c - m)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    D = int(args[0]) if args else 128
    if "--synthetic" in sys.argv:
        H, W = 375, 1242
        left, right = synthetic.stereo_pair(H, W, D, pair_index=0)
        sky = None
    else:
        z = np.load(os.path.join(ROOT, "tests", "golden", "sky_000017_14.npz"))
        left = z["image"]
        H, W = left.shape
        g = synthetic.ground_truth(H, D)
        x = np.arange(W)[None, :]
        right = np.ascontiguousarray(np.take_along_axis(left, np.minimum(x + g[:, None], W - 1), axis=1))
        sky = z["mask"] if "sky" in args[1:] else None
    ctl, ctr = oracle.census(oracle.blur(left)), oracle.census(oracle.blur(right))
    C = oracle.vfilter(oracle.hfilter(oracle.dsi(ctl, ctr, D, sky=sky), 5), 3)
    C = C.reshape(H, W, D).astype(np.float32)
    Lt = np.empty_like(C)
    Lt[:, 0] = C[:, 0]
    for j in range(1, W):
        Lt[:, j] = step(Lt[:, j - 1], C[:, j])
    assert np.array_equal(oracle.path(C, 0)[0].reshape(H, W, D).view(np.uint32), Lt.view(np.uint32))
    for name, Cd in (("L1", C), ("L2", C[:, ::-1])):
        if name == "L2":
            Lt = np.empty_like(Cd)
            Lt[:, 0] = Cd[:, 0]
            for j in range(1, W):
                Lt[:, j] = step(Lt[:, j - 1], Cd[:, j])
        fails, dist = 0, []
        for s in range(64, W - 64, 96):
            L = Cd[:, s].copy()  # the zero-state start: L = C at the first step
            first = np.full(H, -1)
            for j in range(s + 1, min(W, s + 512)):
                L = step(L, Cd[:, j])
                eq = (L.view(np.uint32) == Lt[:, j].view(np.uint32)).all(-1)
                first[eq & (first < 0)] = j - s
                if (first >= 0).all():
                    break
            fails += int((first < 0).sum())
            dist += list(first[first >= 0])
        dist = np.array(dist)
        print(f"{name} {H}x{W} D={D} sky={sky is not None}: {len(dist) + fails} (row, start) pairs; "
              f"not coalesced within 512 steps: {fails}; steps p50/p90/p99/p99.9/max: "
              f"{np.percentile(dist, [50, 90, 99, 99.9, 100]).round(1).tolist()}; "
              f"share > 64: {(dist > 64).mean():.4f}, > 128: {(dist > 128).mean():.5f}", flush=True)


if __name__ == "__main__":
    main()
