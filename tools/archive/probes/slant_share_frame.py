"""Top-down share sweep on any frame size (debug build, SGM_SLANT_DOWN_EIGHTHS):
ms per frame of sgm_process_device, best of 2 x 6 frames per share, shares
interleaved.  Usage (GPU): python tools/slant_share_frame.py H W D V "4 5 6 7"."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SGM_HIP_LIB"] = os.path.join(ROOT, "stereo_matching_amd", "libsgm_hip_slantdbg.so")
os.environ["SGM_SLANT"] = "1"
sys.path.insert(0, ROOT)
import torch  # noqa: E402

torch.cuda.init()
from stereo_matching_amd import SGM, synthetic  # noqa: E402

h, w, D, V = (int(x) for x in sys.argv[1:5])
shares = [int(x) for x in sys.argv[5].split()]
left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
dev = torch.device("cuda", 0)
dl, dr = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
out = torch.empty((h, w), dtype=torch.float32, device=dev)
torch.cuda.synchronize()
best = {e: 1e9 for e in shares}
with SGM(h, w, 1, D, views=V, device=0) as sgm:
    for rep in range(2):
        for e in shares:
            os.environ["SGM_SLANT_DOWN_EIGHTHS"] = str(e)
            sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
            sgm.check()
            t0 = time.perf_counter()
            for _ in range(6):
                sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
            sgm.check()
            best[e] = min(best[e], (time.perf_counter() - t0) / 6 * 1e3)
print(f"{w}x{h} D={D} V={V}: " + "  ".join(f"{e}/8 {best[e]:.3f} ms" for e in shares), flush=True)
