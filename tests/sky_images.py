"""Synthetic single-channel frames for the sky detector
(sky_detector/imageSkyDetector.cpp): a bright, smooth sky over a textured
ground, with horizons, dark specks, narrow sky runs, inverted edges and zero
pixels that exercise every branch of extract_border and
check_sky_border_by_gray_value.  Seeded numpy only."""
from __future__ import annotations

import numpy as np


def make(kind: str, H: int, W: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    ground = rng.integers(10, 150, (H, W)).astype(np.int64)
    yy, xx = np.mgrid[0:H, 0:W]
    sky = 190 + 20 * np.sin(xx / 37.0) + 8 * np.cos(yy / 5.0) + rng.integers(0, 3, (H, W))
    horizon = (H * 0.12 + H * 0.2 * (0.5 + 0.5 * np.sin(np.arange(W) / (W / 7.0 + 1)))).astype(int)
    img = np.where(yy < horizon[None, :], sky, ground)
    if kind == "horizon":
        pass
    elif kind == "dark_specks":         # a sky pixel < 128 drops its column (:101-109)
        cols = rng.choice(W, max(1, W // 9), replace=False)
        img[np.minimum(horizon[cols] // 2, H - 1), cols] = 60
    elif kind == "narrow_runs":         # sky runs of 1..45 columns: < 30 are removed (:116-164)
        img = ground.copy()
        c = 0
        while c < W:
            run = int(rng.integers(1, 46))
            if rng.random() < 0.5:
                img[:horizon[c], c:c + run] = sky[:horizon[c], c:c + run]
            c += run + int(rng.integers(1, 8))
    elif kind == "inverted":            # dark above, bright below: grad_y > 0 -> -1 (:309-320)
        img = np.where(yy < horizon[None, :], 40, 220) + rng.integers(0, 3, (H, W))
    elif kind == "zeros":               # exact zeros are skipped by the energy (:626-628)
        img[rng.random((H, W)) < 0.1] = 0
    elif kind == "flat":                # no gradient anywhere
        img = np.full((H, W), 200)
    elif kind == "right_edge":          # a sky run touching the last column
        img = ground.copy()
        img[:H // 4, W - 31:] = 200
        img[:H // 4, W - 70:W - 41] = 210
    else:
        raise ValueError(kind)
    return np.clip(img, 0, 255).astype(np.uint8)


KINDS = ("horizon", "dark_specks", "narrow_runs", "inverted", "zeros", "flat", "right_edge")
