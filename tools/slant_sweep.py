"""Frame time of the slanted-tile schedule (at several top-down CU shares)
against the default non-slanted schedule (bands above the Infinity Cache,
whole-volume pairs below it), per frame size: sets sgm_capi.hip
slant_default and slant_down_grid_eighths.  Runs the -DSGM_SLANT_DEBUG build
(SGM_SLANT_DOWN_EIGHTHS); each size: one handle per variant, 2 warm-up frames,
6 timed frames on device-resident inputs, alternated REPS times, best kept.
Usage (GPU): python tools/slant_sweep.py "EIGHTHS" HxWxDxV ...   (EIGHTHS e.g. "4 6 8")"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SGM_HIP_LIB"] = os.path.join(ROOT, "stereo_matching_amd", "libsgm_hip_slantdbg.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

torch.cuda.init()
from stereo_matching_amd import SGM, synthetic  # noqa: E402

REPS = int(os.environ.get("REPS", "2"))
NFR = int(os.environ.get("NFR", "6"))  # timed frames per handle
eighths = [int(x) for x in sys.argv[1].split()]
sizes = [tuple(int(x) for x in a.split("x")) for a in sys.argv[2:]]
dev = torch.device("cuda", 0)
cus = torch.cuda.get_device_properties(0).multi_processor_count
for (h, w, D, V) in sizes:
    left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
    dl, dr = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
    out = torch.empty((h, w), dtype=torch.float32, device=dev)
    variants = [("base", "0", None)] + [(f"slant{e}", "1", str(e)) for e in eighths]
    res = {}
    for rep in range(REPS):
        for name, sl, e in variants:
            os.environ["SGM_SLANT"] = sl
            if e is None:
                os.environ.pop("SGM_SLANT_DOWN_EIGHTHS", None)
            else:
                os.environ["SGM_SLANT_DOWN_EIGHTHS"] = e
            with SGM(h, w, 1, D, views=V, device=0) as sgm:
                for _ in range(2):
                    sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(NFR):
                    sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
                torch.cuda.synchronize()
                res.setdefault(name, []).append((time.perf_counter() - t0) / NFR * 1e3)
                sgm.check()
                if os.environ.get("PROF") and rep == 0:
                    sgm.set_profiling(True)
                    for _ in range(NFR):
                        sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
                    torch.cuda.synchronize()
                    prof = sgm.get_profile()
                    sgm.set_profiling(False)
                    print(f"  {name}: " + " ".join(f"{k}={v[1] / v[0] * 1e3:.0f}" for k, v in prof.items()),
                          flush=True)
    b = min(res["base"])
    best = min((min(v), k) for k, v in res.items() if k != "base")
    parts = " ".join(f"{k} {min(v):.3f}" for k, v in res.items())
    print(f"{h}x{w} D={D} V={V} ({h * w * D * 4 / 2**20:.0f} MB/view, views*W/(14*CUs) "
          f"{V * w / (14 * cus):.2f}): {parts} ms; best slanted {best[1]} {(best[0] / b - 1) * 100:+.1f}% vs base",
          flush=True)
