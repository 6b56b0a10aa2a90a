"""Stress test of the slanted-tile passes (hand-off races): random frame sizes
and disparity ranges, each frame through SGM_SLANT=1 and SGM_SLANT=0 (the
pair/band schedules, themselves pinned to the oracle by the test suite), maps
compared bit for bit, several frames per handle (epochs and graph-free
replays of the tickets).  Usage: python tools/slant_stress.py [N] [seed]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stereo_matching_amd import SGM, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 4)
bad = 0
for it in range(n):
    D = int(rng.choice([32, 64, 128, 256]))
    h = int(rng.integers(3, 260))
    w = int(rng.integers(5, 700))  # (the 5x3 cost window: sgm_create rejects W < 5)
    views = int(rng.integers(1, 3))
    maps = {}
    for m in ("0", "1"):
        os.environ["SGM_SLANT"] = m
        with SGM(h, w, 1, D, views=views) as sgm:
            out = []
            for k in range(3):
                left, right = synthetic.stereo_pair(h, w, D, pair_index=it * 3 + k)
                sgm.process(left, right)
                raw = sgm.get_raw_disp().copy()
                lr = sgm.get_lr_disp().copy() if views == 2 else None
                out.append((raw, lr))
        maps[m] = out
    ok = all(np.array_equal(a[0], b[0]) and (a[1] is None or np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32)))
             for a, b in zip(maps["0"], maps["1"]))
    bad += not ok
    print(f"{it:4d} {h}x{w} D={D} V={views}: {'ok' if ok else 'MISMATCH'}", flush=True)
print("ALL OK" if not bad else f"{bad} MISMATCHES")
sys.exit(1 if bad else 0)
