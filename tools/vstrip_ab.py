"""Paired A/B of the slanted schedule's cost stage: checkpoints + strip pass
(sgm_vstrip.hip, the default) against cost_h + vfwd_l3 (SGM_VSTRIP=0), per
frame size: one handle per variant, 2 warm-up frames, NFR timed frames on
device-resident inputs, alternated REPS times, best kept; then one profiled
pass per variant (per-class microseconds per frame).
Usage (GPU): python tools/vstrip_ab.py HxWxDxV ..."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

torch.cuda.init()
from stereo_matching_amd import SGM, synthetic  # noqa: E402

REPS = int(os.environ.get("REPS", "3"))
NFR = int(os.environ.get("NFR", "6"))
sizes = [tuple(int(x) for x in a.split("x")) for a in sys.argv[1:]]
dev = torch.device("cuda", 0)
os.environ["SGM_SLANT"] = "1"
for (h, w, D, V) in sizes:
    left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
    dl, dr = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
    out = {k: torch.empty((h, w), dtype=torch.float32, device=dev) for k in ("strips", "twopass")}
    res, prof = {}, {}
    for rep in range(REPS):
        for name, env in (("strips", "1"), ("twopass", "0")):
            os.environ["SGM_VSTRIP"] = env
            with SGM(h, w, 1, D, views=V, device=0) as sgm:
                o = out[name]
                for _ in range(2):
                    sgm.process_device(dl.data_ptr(), dr.data_ptr(), o.data_ptr())
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(NFR):
                    sgm.process_device(dl.data_ptr(), dr.data_ptr(), o.data_ptr())
                torch.cuda.synchronize()
                res.setdefault(name, []).append((time.perf_counter() - t0) / NFR * 1e3)
                sgm.check()
                if rep == 0:
                    sgm.set_profiling(True)
                    for _ in range(3):
                        sgm.process_device(dl.data_ptr(), dr.data_ptr(), o.data_ptr())
                    torch.cuda.synchronize()
                    prof[name] = sgm.get_profile()
                    sgm.set_profiling(False)
    same = bool(torch.equal(out["strips"].view(torch.int32), out["twopass"].view(torch.int32)))
    a, b = min(res["strips"]), min(res["twopass"])
    print(f"{w}x{h} D={D} V={V}: strips {a:.3f} ms  twopass {b:.3f} ms  ({(a / b - 1) * 100:+.1f}%)  "
          f"maps identical {same}", flush=True)
    for name, p in prof.items():
        print(f"  {name}: " + " ".join(f"{k}={v[1] / v[0] * 1e3:.0f}" for k, v in p.items()), flush=True)
