"""Disparity maps that stress post_filter() (src/Solver.cpp:600-649).

The median fill is sequential and in place (a fill is seen by every later
window), and the speckle filter is a connected-component size test.  These
generators build maps whose fills chain across rows, columns and the GPU's
64x16 tiles, and whose components straddle the size limit (1000/scale) and
the |a-b| < 2 join threshold.  Seeded numpy only; used by the CPU oracle
tests and the GPU parity tests alike.
"""
from __future__ import annotations

import numpy as np


def _smooth(rng, H, W, D):
    """Piecewise-planar disparity field with sub-pixel values in [0, D-1]."""
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    f = np.zeros((H, W), np.float32)
    for _ in range(4):
        a, b = rng.uniform(-0.05, 0.05, 2)
        c = rng.uniform(0, D - 1)
        cut = rng.uniform(0, W)
        part = xx >= cut
        f = np.where(part, (a * xx + b * yy + c).astype(np.float32), f)
    f = np.clip(f + rng.uniform(-0.45, 0.45, (H, W)).astype(np.float32), 0, D - 1)
    return f.astype(np.float32)


def make(kind: str, H: int, W: int, D: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    inv = np.float32(D + 1)
    f = _smooth(rng, H, W, D)
    if kind == "random_holes":           # scattered invalid pixels, ~35%
        f[rng.random((H, W)) < 0.35] = inv
    elif kind == "dense_holes":          # ~60% invalid: most windows fail the >12 test
        f[rng.random((H, W)) < 0.6] = inv
    elif kind == "hrun":                 # long invalid runs inside rows, across tile columns
        for i in range(2, H - 2, 3):
            a = int(rng.integers(0, max(1, W // 2)))
            f[i, a:a + int(rng.integers(W // 4, W))] = inv
    elif kind == "vstrip":               # occlusion-like strips, 1-9 px wide, across tile rows
        for _ in range(max(1, W // 40)):
            a = int(rng.integers(0, W))
            f[:, a:a + int(rng.integers(1, 10))] = inv
    elif kind == "blocks":               # invalid blocks on tile corners (64 x 16 grid)
        for ty in range(0, H, 16):
            for tx in range(0, W, 64):
                h, w = int(rng.integers(2, 9)), int(rng.integers(2, 9))
                f[max(0, ty - h // 2):ty + h // 2 + 1, max(0, tx - w // 2):tx + w // 2 + 1] = inv
    elif kind == "diag":                 # diagonal invalid bands: fills chain through tiles
        yy, xx = np.mgrid[0:H, 0:W]
        f[((xx + 3 * yy) % 37) < 3] = inv
        f[rng.random((H, W)) < 0.1] = inv
    elif kind == "speckle":              # small islands near the size limit, in a flat sea
        f[:] = np.float32(D // 2)
        yy, xx = np.mgrid[0:H, 0:W]
        for _ in range(max(1, H * W // 3000)):
            cy, cx = rng.integers(0, H), rng.integers(0, W)
            r = rng.uniform(3, 22)
            f[(yy - cy) ** 2 + (xx - cx) ** 2 < r * r] = np.float32(rng.uniform(0, D - 1))
        f[rng.random((H, W)) < 0.05] = inv
    elif kind == "snake":                # one thin component winding through many tiles
        f[:] = inv
        v = np.float32(D / 3)
        for i in range(0, H, 4):
            f[i, :] = v
            f[i:i + 4, (W - 1) if (i // 4) % 2 == 0 else 0] = v
        f += np.where(f <= D - 1, rng.uniform(-0.4, 0.4, (H, W)), 0).astype(np.float32)
    elif kind == "threshold":            # neighbours exactly 2 apart (not joined) and just under
        base = rng.integers(0, max(1, D - 4), (H, W)).astype(np.float32)
        step = rng.choice(np.array([0.0, 1.9999999, 2.0, 1.0, 2.0000002], np.float32), (H, W))
        f = np.clip(base + step, 0, D - 1).astype(np.float32)
        f[rng.random((H, W)) < 0.2] = inv
    elif kind == "odd_invalid":          # invalid values other than D+1 (any x > D-1)
        m = rng.random((H, W)) < 0.3
        f[m] = np.float32(D - 1) + rng.choice(np.array([0.5, 1.0, 2.0, 37.0], np.float32),
                                              int(m.sum()))
    elif kind == "all_invalid":
        f[:] = inv
    elif kind == "all_valid":
        pass
    else:
        raise ValueError(kind)
    return np.ascontiguousarray(f, np.float32)


KINDS = ("random_holes", "dense_holes", "hrun", "vstrip", "blocks", "diag", "speckle", "snake",
         "threshold", "odd_invalid", "all_invalid", "all_valid")
