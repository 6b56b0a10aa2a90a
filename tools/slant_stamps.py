"""Where the slanted bottom-up pass spends its time (library built with
-DSGM_SLANT_STAMPS: bash tools/variant.sh slantst -DSGM_SLANT_STAMPS, loaded
with SGM_HIP_LIB=build/slantst/libsgm_hip.so).  Usage: slant_stamps.py [H W D V]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SGM_SLANT"] = "1"
import torch  # noqa: E402
from stereo_matching_amd import SGM, synthetic, _capi  # noqa: E402

h, w, D, V = (int(x) for x in sys.argv[1:5]) if len(sys.argv) > 4 else (1080, 1920, 256, 2)
left, right = synthetic.stereo_pair(h, w, D, pair_index=0)
dev = torch.device("cuda", 0)
dl, dr = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
out = torch.empty((h, w), dtype=torch.float32, device=dev)
sgm = SGM(h, w, 1, D, views=V, device=0)
lib = _capi.lib()
lib.sgm_debug_slant_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
b = (ctypes.c_ulonglong * 32)()
for it in range(3):
    sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    lib.sgm_debug_slant_stamps(b, 1)
sgm.set_profiling(True)
sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr())
torch.cuda.synchronize()
prof = sgm.get_profile()
lib.sgm_debug_slant_stamps(b, 1)
xa = list(b)
print(f"{h}x{w} D={D} V={V}: slant_up {prof['slant_up'][1]:.3f} ms, slant_down {prof['slant_down'][1]:.3f} ms")
for name, x, ms in (("down", xa[:16], prof['slant_down'][1]), ("up", xa[16:], prof['slant_up'][1])):
    steps = max(x[0], 1)
    wg = max(x[8], 1)
    rate = x[7] / wg / (ms * 1e3)  # ticks per us (inside-tile ticks per WG over the launch)
    print(f"  {name}: workgroups {x[8]}, tiles {x[9]}, tile-steps {x[0]} ({x[0] / wg:.0f} per WG), "
          f"{ms * 1e3 / (x[0] / wg):.2f} us per step, ~{rate:.0f} ticks/us")
    print(f"    compute wave 0 per step: work {x[4] / steps:.0f}  barrier {x[5] / steps:.0f} ticks")
    print(f"    receiver per phase: work {x[10] / steps:.0f}  barrier {x[11] / steps:.0f}; "
          f"publisher per phase: work {x[12] / steps:.0f}  barrier {x[13] / steps:.0f} ticks")
    print(f"    re-polled phases {x[1]} ({x[1] / steps * 100:.1f}%), re-polls {x[2]}, "
          f"ticks in re-polls per phase {x[3] / steps:.0f}")
    print("    raw:", x[:14])
