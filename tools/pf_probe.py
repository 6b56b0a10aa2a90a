#!/usr/bin/env python3
"""Post-filter timing probe: K128/HD LR maps from the GPU pipeline (road and
noise pairs), then sgm_post_filter_device repeatedly with per-launch events.
Prints median-fill launches per call and per-kernel averages."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
dev = torch.device("cuda", 0)
torch.cuda.init()
from stereo_matching_amd import SGM, synthetic  # noqa: E402

QUICK = len(sys.argv) > 1 and sys.argv[1] == "quick"
for (h, w, D) in ((375, 1242, 128),) if QUICK else ((375, 1242, 128), (1080, 1920, 256)):
    for kind in ("road", "noise"):
        left, right = synthetic.stereo_pair(h, w, D, pair_index=0, kind=kind)
        with SGM(h, w, 1, D, device=0) as sgm:
            sgm.process(left, right)
            lr = torch.from_numpy(sgm.get_lr_disp().copy()).to(dev)
            work = torch.empty_like(lr)
            st = torch.cuda.current_stream(dev).cuda_stream
            for _ in range(3):
                work.copy_(lr)
                sgm.post_filter_device(work.data_ptr(), stream=st)
            torch.cuda.synchronize(dev)
            n = 3 if QUICK else 20
            t0 = time.perf_counter()
            for _ in range(n):
                work.copy_(lr)
                sgm.post_filter_device(work.data_ptr(), stream=st)
            torch.cuda.synchronize(dev)
            wall = (time.perf_counter() - t0) / n * 1e3
            sgm.set_profiling(True)
            for _ in range(n):
                work.copy_(lr)
                sgm.post_filter_device(work.data_ptr(), stream=st)
            prof = sgm.get_profile()
            sgm.set_profiling(False)
        inv = float((lr > D - 1).float().mean())
        print(f"{w}x{h} D={D} {kind}: invalid {inv:.3f}, wall {wall:.3f} ms/call, "
              + ", ".join(f"{k} {c / n:.1f}x{t / c * 1e3:.1f}us" for k, (c, t, _) in prof.items()),
              flush=True)
