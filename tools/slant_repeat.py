"""Repeatability of the slanted schedule at full size (hand-off races that
only a long run would show): one handle per size, N frames of the same pair
back to back on the handle's stream, each checked by sgm_check and its map
compared bit for bit with the first frame's; the first frame itself is
compared with the banded schedule's (SGM_SLANT=0, pinned to the oracle by the
test suite).  Usage: python tools/slant_repeat.py [N] [HxWxDxV ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from stereo_matching_amd import SGM, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
sizes = [tuple(int(x) for x in a.split("x")) for a in sys.argv[2:]] or [(1080, 1920, 256, 2)]
dev = torch.device("cuda", 0)
bad = 0
for (h, w, D, V) in sizes:
    left, right = synthetic.stereo_pair(h, w, D, pair_index=7)
    dl, dr = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
    outs = {}
    for m in ("0", "1"):
        os.environ["SGM_SLANT"] = m
        out = torch.empty((h, w), dtype=torch.float32, device=dev)
        with SGM(h, w, 1, D, views=V, device=0) as sgm:
            sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
            sgm.check()
            first = out.cpu().numpy().view(np.uint32).copy()
            outs[m] = first
            if m == "0":
                continue
            t0 = time.perf_counter()
            diff = 0
            for k in range(n):
                sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
                sgm.check()
                if not np.array_equal(out.cpu().numpy().view(np.uint32), first):
                    diff += 1
            dt = time.perf_counter() - t0
    same = np.array_equal(outs["0"], outs["1"])
    bad += diff + (not same)
    print(f"{h}x{w} D={D} V={V}: slanted == banded: {same}; {n} repeats, {diff} differ from the first, "
          f"every sgm_check ok ({dt:.1f} s)", flush=True)
print("ALL OK" if not bad else f"{bad} MISMATCHES")
sys.exit(1 if bad else 0)
