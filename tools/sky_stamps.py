"""Phase breakdown of the sky detector's column kernel (library built with
-DSGM_STAMPS, loaded through SGM_HIP_LIB): mean cycles per workgroup for the
strip staging, the per-(row, column) threshold counts and the column walk."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from stereo_matching_amd import SGM, synthetic, _capi  # noqa: E402

for h, w in ((375, 1242), (2160, 3840)):
    img = synthetic.noise_image(h, w, 7)
    img[: h // 3] = 200  # a bright band for a sky
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(img).to(dev)
    d_mask = torch.empty((h, w), dtype=torch.uint8, device=dev)
    sgm = SGM(h, w, 1, 64, device=0, aux_only=True)
    lib = _capi.lib()
    lib.sgm_debug_stamps_sky.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 4)()
    for it in range(4):
        sgm.sky_detect_device(d_img.data_ptr(), d_mask.data_ptr())
        torch.cuda.synchronize()
        lib.sgm_debug_stamps_sky(buf, 1)
    n = buf[3]
    print(f"{w}x{h}: blocks {n}  staging {buf[0] / n / 1e3:.1f} kcyc  counts {buf[1] / n / 1e3:.1f} kcyc"
          f"  walk {buf[2] / n / 1e3:.1f} kcyc")
    sgm.close()
