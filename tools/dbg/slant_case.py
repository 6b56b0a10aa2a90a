"""Debug: one fuzz case of tests/test_gpu_fuzz.py under SGM_SLANT=1, repeated."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
os.environ["SGM_SLANT"] = "1"
import numpy as np
import oracle
from stereo_matching_amd import SGM, synthetic
import test_gpu_fuzz as tf

want_id = sys.argv[1] if len(sys.argv) > 1 else "51x80_D32"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
for c in tf.CASES:
    cid = f"{c['h']}x{c['w']}_D{c['D']}"
    if cid != want_id:
        continue
    print(c)
    h, w, D, s = c["h"], c["w"], c["D"], c["s"]
    left, right = synthetic.stereo_pair(h, w, D, pair_index=100 + c["seed"], kind=c["kind"])
    H, W = h // s, w // s
    sky = synthetic.sky_mask(H, W) if c["sky"] else None
    ref = oracle.process(left, right, D, scale=s, sky_l=sky, sky_r=sky, P1=c["p1"], P2=c["p2"],
                         uniq=c["uniq"], lr_dis=c["lr"], blur=c["blur"], views=c["views"])
    with SGM(h, w, s, D, blur=c["blur"], views=c["views"], p1=c["p1"], p2=c["p2"],
             uniqueness=c["uniq"], lr_max_diff=c["lr"]) as sgm:
        for rep in range(reps):
            sgm.process(left, right, sky, sky)
            raw = sgm.get_raw_disp().astype(np.int64)
            diff = np.argwhere(raw != ref["disp"].astype(np.int64))
            err = ""
            if os.environ.get("SGM_HIP_LIB", "").startswith("build/dbg"):
                import ctypes
                from stereo_matching_amd import _capi
                lib = _capi.lib()
                lib.sgm_debug_slant_err.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_uint)]
                dn, up = ctypes.c_uint(), ctypes.c_uint()
                lib.sgm_debug_slant_err(sgm._h, ctypes.byref(dn), ctypes.byref(up))
                err = f" timeouts down {dn.value} up {up.value}"
            print(rep, "mismatches", len(diff), diff[:6].tolist(), err, flush=True)
