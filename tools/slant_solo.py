"""The concurrent region's two launches alone and in sequence (debug build,
SGM_SLANT_SOLO; the maps are wrong in these probes): per launch, its time and
its algorithmic bytes' rate.  Usage (GPU): python tools/slant_solo.py H W D V"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SGM_HIP_LIB"] = os.path.join(ROOT, "stereo_matching_amd", "libsgm_hip_slantdbg.so")
os.environ["SGM_SLANT"] = "1"
sys.path.insert(0, ROOT)
import torch  # noqa: E402

torch.cuda.init()
import bench  # noqa: E402
from stereo_matching_amd import SGM, synthetic  # noqa: E402

h, w, D, V = (int(x) for x in sys.argv[1:5])
left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
dev = torch.device("cuda", 0)
dl, dr = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
out = torch.empty((h, w), dtype=torch.float32, device=dev)
torch.cuda.synchronize()
with SGM(h, w, 1, D, views=V, device=0) as sgm:
    for mode in ("", "down", "hpair", "seq"):
        if mode:
            os.environ["SGM_SLANT_SOLO"] = mode
        else:
            os.environ.pop("SGM_SLANT_SOLO", None)
        for _ in range(2):
            sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
        torch.cuda.synchronize()
        sgm.set_profiling(True)
        for _ in range(4):
            sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
        prof = sgm.get_profile()
        sgm.set_profiling(False)
        parts = []
        for k in ("slant_down_hpair", "slant_down", "stage_a_h", "slant_up"):
            if k in prof:
                n, tot, el = prof[k]
                us = tot / n * 1e3
                parts.append(f"{k} {us:8.1f} us ({bench.algorithmic_bytes(k, el, D) / us / 1e6:.2f} TB/s)")
        print(f"{w}x{h} D={D} V={V} [{mode or 'concurrent'}]: " + ", ".join(parts), flush=True)
