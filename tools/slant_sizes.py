"""Frame time of the slanted-tile schedule against the bands over frame sizes
above the Infinity Cache (sets sgm_capi.hip slant_default).  Each size: a
handle per schedule (SGM_SLANT read at create), 2 warm-up frames, then 6
timed frames on device-resident inputs, alternated twice.
Usage: python tools/slant_sizes.py [HxWxDxV ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from stereo_matching_amd import SGM, synthetic  # noqa: E402

sizes = [(1080, 1920, 256, 1), (2160, 3840, 256, 1), (512, 1056, 128, 2), (720, 1280, 256, 2),
         (1080, 1920, 128, 2), (1080, 1920, 64, 2), (2160, 3840, 128, 2), (1080, 1920, 256, 2)]
if len(sys.argv) > 1:
    sizes = [tuple(int(x) for x in a.split("x")) for a in sys.argv[1:]]
dev = torch.device("cuda", 0)
for (h, w, D, V) in sizes:
    left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
    dl, dr = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
    out = torch.empty((h, w), dtype=torch.float32, device=dev)
    res = {}
    for rep in range(2):
        for m in ("0", "1"):
            os.environ["SGM_SLANT"] = m
            with SGM(h, w, 1, D, views=V, device=0) as sgm:
                for _ in range(2):
                    sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(6):
                    sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
                torch.cuda.synchronize()
                res.setdefault(m, []).append((time.perf_counter() - t0) / 6 * 1e3)
    b, s = min(res["0"]), min(res["1"])
    tiles_per_wg = V * w * h / (14 * 256) / h
    print(f"{h}x{w} D={D} V={V} ({h * w * D * 4 / 2**20:.0f} MB/view, {tiles_per_wg:.2f} tiles/WG): "
          f"bands {b:.3f} ms, slant {s:.3f} ms ({(s / b - 1) * 100:+.1f}%)", flush=True)
