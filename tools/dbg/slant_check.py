"""Debug driver: SGM_SLANT=1 frames against the oracle, first mismatches printed."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["SGM_SLANT"] = "1"
import numpy as np
import oracle
from stereo_matching_amd import SGM, synthetic

cases = [(3, 5, 32, 1), (8, 20, 32, 1), (20, 40, 64, 1), (40, 100, 64, 2), (60, 200, 128, 2),
         (50, 300, 256, 2), (96, 320, 64, 2)]
if len(sys.argv) > 1:
    cases = [tuple(int(x) for x in a.split("x")) for a in sys.argv[1:]]
bad = 0
for (h, w, D, views) in cases:
    left, right = synthetic.stereo_pair(h, w, D, pair_index=1)
    with SGM(h, w, 1, D, views=views) as sgm:
        sgm.process(left, right)
        raw = sgm.get_raw_disp().astype(np.int64)
        got = sgm.get_lr_disp() if views == 2 else None
    ref = oracle.process(left, right, D, views=views)
    want = ref["disp"].astype(np.int64)
    diff = np.argwhere(raw != want)
    print(f"{h}x{w} D={D} V={views}: raw mismatches {len(diff)} / {raw.size}", flush=True)
    if len(diff):
        bad += 1
        for (i, j) in diff[:8]:
            print("   ", i, j, "got", raw[i, j], "want", want[i, j])
        # which rows/cols
        print("    rows", np.unique(diff[:, 0])[:20], "cols", np.unique(diff[:, 1])[:20])
    elif views == 2:
        ok = np.array_equal(got.view(np.uint32), ref["lr"].view(np.uint32))
        print("    lr map equal:", ok)
        bad += not ok
print("BAD" if bad else "ALL OK")
