"""The slanted passes' hang guard and ticket order, exercised once
(sgm_slant.hip receiver wave, sgm_capi.hip sgm_check).

Runs on the debug build of the library (stereo_matching_amd/
libsgm_hip_slantdbg.so: the release objects plus sgm_slant/sgm_capi built
with -DSGM_SLANT_DEBUG), on a small two-view frame forced onto the slanted
schedule (SGM_SLANT=1), and prints one JSON line:

  * stall: SGM_SLANT_STALL=<tile> makes that tile's bottom-up receiver (view
    0) refuse every granule and SGM_SLANT_SPIN_LIMIT bounds its polls: the
    frame must end in bounded time and sgm_check must report SGM_ERR_HIP with
    the hand-off message (the give-up is sticky for the launch, so the other
    tiles' waits are skipped instead of timing out one by one);
  * recovery: the next frame, without the stall, is bit-exact against the
    oracle and sgm_check is clean;
  * grids: SGM_SLANT_GRID = 1, 2, 3 workgroups per pass (tiles claimed in the
    order T-1 .. 0, so a tile's producer always holds a workgroup or has
    finished) give bit-exact maps: the deadlock-freedom argument of
    sgm_slant.hip at the smallest grids;
  * the give-up's cost per poll (the stall at ten times the spin limit) and
    the release build's give-up time it extrapolates to (kSlantSpinLimit).

Usage (GPU): python tools/slant_guard.py [--h 64 --w 200 --D 64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DBG = os.path.join(ROOT, "stereo_matching_amd", "libsgm_hip_slantdbg.so")
os.environ["SGM_HIP_LIB"] = DBG      # before the package loads the library
os.environ["SGM_SLANT"] = "1"
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=64)
    ap.add_argument("--w", type=int, default=200)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--spin-limit", type=int, default=2000)
    args = ap.parse_args()
    h, w, D = args.h, args.w, args.D
    if not os.path.exists(DBG):
        raise SystemExit(f"{DBG} is missing (make -C stereo_matching_amd/csrc)")
    import torch

    import oracle
    from stereo_matching_amd import SGM, SGMError, synthetic
    oracle.build()
    dev = torch.device("cuda", 0)
    left, right = synthetic.stereo_pair(h, w, D, pair_index=11)
    ref = oracle.process(left, right, D)["lr"]
    dl = torch.from_numpy(left).to(dev)
    dr = torch.from_numpy(right).to(dev)
    torch.cuda.synchronize(dev)  # the frames run on the handle's own (non-blocking) stream
    out = {"frame": f"{w}x{h} D={D} two views, slanted schedule forced", "lib": os.path.basename(DBG)}
    with SGM(h, w, 1, D, device=0) as sgm:
        ntiles = (w + h - 1 + 13) // 14

        def frame():
            m = torch.empty((h, w), dtype=torch.float32, device=dev)
            torch.cuda.synchronize(dev)
            sgm.process_device(dl.data_ptr(), dr.data_ptr(), m.data_ptr(), stream=None)
            return m

        def exact(m):
            return bool(np.array_equal(m.cpu().numpy().view(np.uint32), ref.view(np.uint32)))

        # warm (and a clean check before anything is forced)
        m = frame()
        sgm.check()
        out["baseline_exact"] = exact(m)
        # 1. forced give-up
        os.environ["SGM_SLANT_SPIN_LIMIT"] = str(args.spin_limit)
        os.environ["SGM_SLANT_STALL"] = str(ntiles // 2)
        t0 = time.perf_counter()
        m = frame()
        torch.cuda.synchronize(dev)
        err = None
        try:
            sgm.check()
        except SGMError as e:
            err = e
        out["stall"] = {"tile": ntiles // 2, "tiles": ntiles, "spin_limit": args.spin_limit,
                        "frame_s": round(time.perf_counter() - t0, 4),
                        "code": None if err is None else err.code,
                        "message": None if err is None else str(err),
                        "maps_differ": not exact(m)}
        # the give-up's cost per poll: the same stall at ten times the spin
        # limit; the slope extrapolates to the release build's kSlantSpinLimit
        os.environ["SGM_SLANT_SPIN_LIMIT"] = str(10 * args.spin_limit)
        t0 = time.perf_counter()
        frame()
        torch.cuda.synchronize(dev)
        t10 = time.perf_counter() - t0
        try:
            sgm.check()
        except SGMError:
            pass
        per_spin = max(t10 - out["stall"]["frame_s"], 0.0) / (9 * args.spin_limit)
        out["stall"]["frame_s_10x"] = round(t10, 4)
        out["stall"]["us_per_spin"] = round(per_spin * 1e6, 3)
        out["stall"]["release_give_up_s"] = round(per_spin * (1 << 22), 2)  # kSlantSpinLimit
        del os.environ["SGM_SLANT_STALL"], os.environ["SGM_SLANT_SPIN_LIMIT"]
        # 2. the next frame is valid again
        m = frame()
        rc_ok = True
        try:
            sgm.check()
        except SGMError:
            rc_ok = False
        out["recovery"] = {"exact": exact(m), "check_ok": rc_ok}
        # 3. the smallest grids
        out["grids"] = {}
        for g in (1, 2, 3):
            os.environ["SGM_SLANT_GRID"] = str(g)
            t0 = time.perf_counter()
            m = frame()
            sgm.check()
            out["grids"][str(g)] = {"exact": exact(m), "frame_s": round(time.perf_counter() - t0, 4)}
        del os.environ["SGM_SLANT_GRID"]
    out["ok"] = bool(out["baseline_exact"] and out["stall"]["code"] == 3
                     and "timed out" in (out["stall"]["message"] or "")
                     and out["recovery"]["exact"] and out["recovery"]["check_ok"]
                     and all(v["exact"] for v in out["grids"].values()))
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
