"""Portable synthetic stereo pairs.

splitmix64 noise for the left image, a slanted "road" disparity field
g[i] = floor(D/16 + 0.6*D*i/H) and the right image R[i, x] = L[i, min(x+g[i], W-1)].
The same generator feeds the tests, the smoke check and bench.py, so every
consumer sees identical bytes for a given (seed, size).
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x53474D0000
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z & _M64


def noise_image(h: int, w: int, seed: int) -> np.ndarray:
    idx = np.arange(h * w, dtype=np.uint64)
    v = splitmix64(np.uint64(seed) ^ idx)
    return (v >> np.uint64(56)).astype(np.uint8).reshape(h, w)


def ground_truth(h: int, D: int) -> np.ndarray:
    """g[i] = floor(D/16 + 0.6*D*i/H), exact in integers (D is a multiple of 16)."""
    i = np.arange(h, dtype=np.int64)
    return (D // 16 + (6 * D * i) // (10 * h)).astype(np.int64)


def stereo_pair(h: int, w: int, D: int, pair_index: int = 0, kind: str = "road"):
    """Returns (left, right) uint8 images of shape (h, w).

    kind="road": right is the left image shifted by the slanted field g[i].
    kind="noise": independent left and right (exercises the rejection paths).
    """
    seed = SEED_BASE + pair_index
    left = noise_image(h, w, seed)
    if kind == "noise":
        right = noise_image(h, w, seed ^ 0xA5A5A5A5A5)
        return left, right
    g = ground_truth(h, D)
    x = np.arange(w, dtype=np.int64)[None, :]
    src = np.minimum(x + g[:, None], w - 1)
    right = np.take_along_axis(left, src, axis=1)
    return left, np.ascontiguousarray(right)


def sky_mask(h: int, w: int) -> np.ndarray:
    """Config-5 sky: rows < H/6 are sky (255) in both views."""
    m = np.zeros((h, w), np.uint8)
    m[: h // 6] = 255
    return m
