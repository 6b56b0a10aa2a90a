"""Generate the golden regression fixtures in tests/golden/.

Run from the repo root:  python tests/golden/make_golden.py
Inputs are the portable splitmix64 synthetic pairs of
stereo_matching_amd/synthetic.py; outputs come from the CPU oracle
(oracle/sgm_oracle.c), whose parity with the reference is UNPINNED (the
reference cannot be built in this image and ships no vectors).
Each fixture stores inputs and every H x W output in full, and sha256 hashes
of the census words, the left cost volume and the eight left path volumes
(hashes.json) to keep the fixtures small.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from stereo_matching_amd import synthetic  # noqa: E402

# name: (h, w, D, scale, kind, sky, blur, pair_index)
CASES = {
    "road_48x96_D32": (48, 96, 32, 1, "road", False, True, 0),
    "noise_sky_40x120_D64": (40, 120, 64, 1, "noise", True, True, 1),
    "road_64x160_D128": (64, 160, 128, 1, "road", False, True, 2),
    "road_s2_50x98_D32": (50, 98, 32, 2, "road", False, True, 3),
    "road_noblur_24x80_D64": (24, 80, 64, 1, "road", False, False, 4),
    "road_sky_36x300_D256": (36, 300, 256, 1, "road", True, True, 5),
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    hashes = {}
    for name, (h, w, D, s, kind, sky, blur, idx) in CASES.items():
        left, right = synthetic.stereo_pair(h, w, D, idx, kind)
        H, W = h // s, w // s
        m = synthetic.sky_mask(H, W) if sky else np.zeros((H, W), np.uint8)
        out = oracle.process(left, right, D, s, m if sky else None, m if sky else None, blur=blur)
        meta = dict(h=h, w=w, D=D, scale=s, kind=kind, sky=sky, blur=blur, pair_index=idx)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), left=left,
                            right=right, sky=m, **{k: np.asarray(v) for k, v in out.items()})
        wl, wr = left[: H * s: s, : W * s: s], right[: H * s: s, : W * s: s]
        if blur:
            wl, wr = oracle.blur(wl), oracle.blur(wr)
        cl, cr = oracle.census(wl, s), oracle.census(wr, s)
        cost = oracle.vfilter(oracle.hfilter(oracle.dsi(cl, cr, D, s, 0, m if sky else None),
                                             5 // s), 3 // s)
        hv = {"census_l": sha(cl), "census_r": sha(cr), "cost_l": sha(cost)}
        for k in range(8):
            hv[f"L{k + 1}"] = sha(oracle.path(cost, k)[0])
        hashes[name + ".npz"] = hv
        print(name, "valid(lr) = %.3f" % float(np.mean(out["lr"] <= D - 1)))
    with open(os.path.join(HERE, "hashes.json"), "w") as fh:
        json.dump(hashes, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
