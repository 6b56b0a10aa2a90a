"""Barrier-wait breakdown of the split pair kernels (library built with
-DSGM_STAMPS).  Runs a few K128 frames and prints, per wave role, the mean
work and barrier-wait cycles per wave.  Usage: stamps.py [H W D]."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from stereo_matching_amd import SGM, synthetic, _capi  # noqa: E402

h, w, D = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (375, 1242, 128)
left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
dev = torch.device("cuda", 0)
dl, dr = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
out = torch.empty((h, w), dtype=torch.float32, device=dev)
sgm = SGM(h, w, 1, D, views=1, device=0)
lib = _capi.lib()
for f in (lib.sgm_debug_stamps_pair, lib.sgm_debug_stamps_sweep):
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
b1 = (ctypes.c_ulonglong * 48)()
b2 = (ctypes.c_ulonglong * 48)()
for it in range(4):
    sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    lib.sgm_debug_stamps_pair(b1, 1)
    lib.sgm_debug_stamps_sweep(b2, 1)
buf = [x + y for x, y in zip(b1, b2)]
names = ["final producer", "final consumer", "final WTA", "H producer (B)", "H consumer (B)",
         "H fwd (A)", "D6 fwd (A)", "V fwd", "L5 sweep (A)", "L8 sweep", "other sweep",
         "D2 bwd (B)", "-", "H bwd 1-wave", "V bwd 1-wave", "-"]
for r in range(16):
    work, wait, n = buf[3 * r], buf[3 * r + 1], buf[3 * r + 2]
    if n:
        print(f"{names[r]:16s} waves {n:5d}  work {work / n / 1e3:8.1f} kcyc  wait {wait / n / 1e3:8.1f} kcyc")
