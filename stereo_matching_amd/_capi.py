"""ctypes binding of libsgm_hip.so (include/sgm_hip.h).

The library is the product: there is no CPU fallback.  If the shared object
is missing or cannot be loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_PKG = os.path.dirname(os.path.abspath(__file__))
# SGM_HIP_LIB points the loader at another build of the same library (the
# instrumented -DSGM_STAMPS build of tools/stamps.py); default: the in-tree one
LIB_PATH = os.environ.get("SGM_HIP_LIB") or os.path.join(_PKG, "libsgm_hip.so")
CSRC = os.path.join(_PKG, "csrc")

SGM_OK = 0
SGM_ERR_INVALID_ARG = 1
SGM_ERR_OUT_OF_MEMORY = 2
SGM_ERR_HIP = 3
SGM_ERR_NO_DEVICE = 4
SGM_SOLVER_SGM = 0
SGM_SOLVER_BM = 1
SGM_VIEW_LEFT = 0
SGM_VIEW_RIGHT = 1

# Every symbol include/sgm_hip.h declares.
EXPORTS = (
    "sgm_default_params", "sgm_create", "sgm_destroy", "sgm_last_error", "sgm_get_size",
    "sgm_device_bytes", "sgm_process", "sgm_process_device",
    "sgm_post_filter_device", "sgm_stage_census", "sgm_stage_cost", "sgm_stage_path",
    "sgm_stage_aggregate", "sgm_stage_lr", "sgm_stage_post_filter", "sgm_set_profiling",
    "sgm_get_profile", "sgm_lk_refine_device", "sgm_stage_lk_refine", "sgm_sky_detect_device",
    "sgm_stage_sky_detect", "sgm_colormap_device", "sgm_point_cloud_device", "sgm_stage_colormap",
    "sgm_stage_point_cloud", "sgm_lr_check_device", "sgm_get_stream", "sgm_check",
    "sgm_comm_create", "sgm_comm_unique_id", "sgm_comm_create_rank", "sgm_comm_destroy",
    "sgm_comm_last_error", "sgm_comm_info", "sgm_batch_gather", "sgm_batch_gather_all",
)
SGM_COMM_ID_BYTES = 128


class SGMError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"libsgm_hip error {code}: {msg}")
        self.code = code


class Params(ctypes.Structure):
    _fields_ = [
        ("height", ctypes.c_int), ("width", ctypes.c_int), ("scale", ctypes.c_int),
        ("max_disp", ctypes.c_int), ("p1", ctypes.c_int), ("p2", ctypes.c_int),
        ("uniqueness", ctypes.c_float), ("lr_max_diff", ctypes.c_float),
        ("blur", ctypes.c_int), ("views", ctypes.c_int), ("post_filter", ctypes.c_int),
        ("lk_refine", ctypes.c_int), ("sky_detect", ctypes.c_int),
        ("solver", ctypes.c_int), ("aux_only", ctypes.c_int),
        ("view", ctypes.c_int),
    ]


class Camera(ctypes.Structure):
    """sgm_camera: CamIntrinsics (inc/utils.h:14-20) + node.cpp:122-123."""
    _fields_ = [("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float),
                ("cy", ctypes.c_float), ("baseline", ctypes.c_double),
                ("max_range", ctypes.c_float)]


class KernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_int),
                ("total_ms", ctypes.c_double), ("elems", ctypes.c_double)]


# the -DSGM_SLANT_DEBUG build (csrc/Makefile `make dbg`): test infrastructure
# for the hang-guard tests and the share sweeps, never the product
DBG_LIB_PATH = os.path.join(_PKG, "libsgm_hip_slantdbg.so")


def build(force: bool = False, jobs: int = 2, debug: bool = False) -> str:
    """Compile libsgm_hip.so for gfx950 with hipcc (csrc/Makefile); debug=True
    builds the slanted passes' debug library (`make dbg`) instead."""
    if force:
        subprocess.run(["make", "-s", "-C", CSRC, "clean"], check=True)
    subprocess.run(["make", "-s", "-C", CSRC, f"-j{jobs}"] + (["dbg"] if debug else []), check=True)
    return DBG_LIB_PATH if debug else LIB_PATH


_lib = None


def hip_runtimes() -> list:
    """The libamdhip64 files mapped into this process (/proc/self/maps)."""
    found = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.split()[-1] if len(line.split()) >= 6 else ""
                if "libamdhip64.so" in os.path.basename(path) and path not in found:
                    found.append(path)
    except OSError:
        pass
    return found


def _bind_hip_runtime() -> None:
    """Load PyTorch's HIP runtime before libsgm_hip.so, whatever the caller
    imported first (INTEGRATION.md "One HIP runtime per process").

    torch's bundled libamdhip64.so and /opt/rocm's libamdhip64.so.7 carry
    the same soname, so the dynamic loader binds the library's NEEDED entry
    to whichever copy is already in the process.  With torch loaded first
    the library and torch share torch's runtime; loaded the other way round,
    torch's own HIP libraries run beside /opt/rocm's runtime and torch finds
    no GPU.  Importing torch here (it loads its runtime, it does not
    initialise a device) makes the order the same for every caller.  Without
    torch the library binds /opt/rocm's runtime, its RUNPATH."""
    if os.environ.get("SGM_HIP_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401  (loads torch's libamdhip64.so)
    except ImportError:
        return


def lib():
    """Load libsgm_hip.so (raises if absent: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SGMError(SGM_ERR_NO_DEVICE,
                       f"{LIB_PATH} is missing; build it with stereo_matching_amd._capi.build()")
    _bind_hip_runtime()
    L = ctypes.CDLL(LIB_PATH)
    rts = hip_runtimes()
    if len(rts) > 1:
        raise SGMError(SGM_ERR_NO_DEVICE,
                       "two HIP runtimes are mapped in this process (" + ", ".join(rts) + "): load "
                       "PyTorch before anything that links /opt/rocm's libamdhip64 "
                       "(INTEGRATION.md \"One HIP runtime per process\")")
    P = ctypes.c_void_p
    I = ctypes.c_int
    PP = ctypes.POINTER(Params)
    L.sgm_default_params.argtypes = [PP, I, I, I, I]
    L.sgm_create.argtypes = [PP, I, ctypes.POINTER(P)]
    L.sgm_destroy.argtypes = [P]
    L.sgm_last_error.argtypes = [P]
    L.sgm_last_error.restype = ctypes.c_char_p
    L.sgm_get_size.argtypes = [P, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I)]
    L.sgm_device_bytes.argtypes = [P]
    L.sgm_device_bytes.restype = ctypes.c_size_t
    L.sgm_get_stream.argtypes = [P]
    L.sgm_get_stream.restype = ctypes.c_void_p
    L.sgm_process.argtypes = [P, P, P, I, P, P, I, P, I, P]
    L.sgm_process_device.argtypes = [P, P, P, I, P, P, I, P, I, P, P]
    L.sgm_check.argtypes = [P]
    L.sgm_post_filter_device.argtypes = [P, P, I, P]
    L.sgm_lr_check_device.argtypes = [P, P, I, P, I, P, I, P]
    L.sgm_stage_post_filter.argtypes = [P, P]
    L.sgm_lk_refine_device.argtypes = [P, P, P, I, P, I, P]
    L.sgm_stage_lk_refine.argtypes = [P, P, P, I, P]
    L.sgm_sky_detect_device.argtypes = [P, P, I, P, I, P]
    L.sgm_stage_sky_detect.argtypes = [P, P, I, P]
    CP = ctypes.POINTER(Camera)
    L.sgm_colormap_device.argtypes = [P, P, I, P, I, P]
    L.sgm_point_cloud_device.argtypes = [P, P, I, P, I, CP, P, P, P, P]
    L.sgm_stage_colormap.argtypes = [P, P, P]
    L.sgm_stage_point_cloud.argtypes = [P, P, P, I, CP, P, P, P]
    L.sgm_stage_census.argtypes = [P, P, I, P]
    L.sgm_stage_cost.argtypes = [P, P, P, P, I, I, P]
    L.sgm_stage_path.argtypes = [P, I, P, P, P]
    L.sgm_stage_aggregate.argtypes = [P, P, P, P]
    L.sgm_stage_lr.argtypes = [P, P, P, P]
    L.sgm_set_profiling.argtypes = [P, I]
    L.sgm_get_profile.argtypes = [P, ctypes.POINTER(KernelStat), I, ctypes.POINTER(I)]
    L.sgm_comm_create.argtypes = [ctypes.POINTER(I), I, ctypes.POINTER(P)]
    L.sgm_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.sgm_comm_create_rank.argtypes = [ctypes.c_char_p, I, I, I, ctypes.POINTER(P)]
    L.sgm_comm_destroy.argtypes = [P]
    L.sgm_comm_last_error.argtypes = [P]
    L.sgm_comm_last_error.restype = ctypes.c_char_p
    L.sgm_comm_info.argtypes = [P, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I)]
    L.sgm_batch_gather.argtypes = [P, I, P, I, I, I, P, P]
    L.sgm_batch_gather_all.argtypes = [P, ctypes.POINTER(P), I, I, I, P, ctypes.POINTER(P)]
    for name in EXPORTS:
        if name not in ("sgm_last_error", "sgm_device_bytes", "sgm_get_stream", "sgm_comm_last_error"):
            getattr(L, name).restype = I
    _lib = L
    return L


def check(rc: int, handle=None) -> None:
    if rc != SGM_OK:
        msg = ""
        if handle is not None and _lib is not None:
            raw = _lib.sgm_last_error(handle)
            msg = raw.decode() if raw else ""
        raise SGMError(rc, msg)


def default_params(h: int, w: int, s: int, d: int) -> Params:
    p = Params()
    check(lib().sgm_default_params(ctypes.byref(p), h, w, s, d))
    return p
