"""Python mirror of the reference's Solver/SGM class surface.

Reference: inc/Solver.h:23-70 and inc/SGM.h:10-26 (constructor SGM(h, w, s, d),
process(l, r[, sky, sky_beta]), get_disp()).  Every call goes through the
C-ABI of libsgm_hip.so; nothing here computes disparities itself.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _capi
from ._capi import check, lib


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


# hipStreamLegacy (hip_runtime_api.h): the legacy default ("null") stream
_HIP_STREAM_LEGACY = 1


def _stream(stream):
    """The hipStream_t the C-ABI gets: None -> NULL, the handle's own stream
    (non-blocking: NOT ordered with the null stream); 0 -> hipStreamLegacy,
    the legacy default stream (torch's default stream reports cuda_stream 0,
    so passing torch.cuda.current_stream().cuda_stream orders the call with
    torch's work either way); anything else is a hipStream_t handle."""
    if stream is None:
        return ctypes.c_void_p(None)
    return ctypes.c_void_p(_HIP_STREAM_LEGACY if stream == 0 else stream)


def _u8(a, shape, what):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    if a.shape != shape:
        raise ValueError(f"{what}: expected shape {shape}, got {a.shape}")
    return a


class SGM:
    """Semi-global matcher on one MI355X (HIP device `device`).

    Mirrors ``SGM(int h, int w, int s, int d)`` (src/SGM.cpp:4-29).  The
    reference asserts s in {1, 2} and d in {32, 64, 128} (Solver.cpp:6-10);
    here d = 256 is also accepted and invalid arguments raise SGMError.
    """

    def __init__(self, h: int, w: int, s: int = 1, d: int = 128, *, device: int = 0,
                 blur: bool = True, views: int = 2, p1: int = 10, p2: int = 100,
                 uniqueness: float = 0.7, lr_max_diff: float = 1.0, post_filter: bool = False,
                 lk_refine: bool = False, sky_detect: bool = False,
                 aux_only: bool = False, view: str = "left", _solver: int = _capi.SGM_SOLVER_SGM):
        self._lib = lib()
        p = _capi.default_params(h, w, s, d)
        p.blur = int(bool(blur))
        p.views = views
        # post_filter: process_device's output is post_filter()ed on the GPU
        # (SGM.cpp:821); process() keeps the LR map and get_disp() filters it
        p.post_filter = int(bool(post_filter))
        # lk_refine: ... then LKRefine (SGM.cpp:824, commented out in the reference)
        p.lk_refine = int(bool(lk_refine))
        # sky_detect: masks from SkyAreaDetector::detect on the GPU (node.cpp:80-93)
        p.sky_detect = int(bool(sky_detect))
        p.solver = _solver
        # aux_only: side stages only (sky, post_filter, LKRefine, colormap, cloud)
        p.aux_only = int(bool(aux_only))
        # view ("left" | "right", views=1 only): the right view alone (SGM.cpp:448-801),
        # for a pair split over two GPUs that meet in lr_check_device
        if view not in ("left", "right"):
            raise ValueError(f"view must be 'left' or 'right', got {view!r}")
        p.view = _capi.SGM_VIEW_RIGHT if view == "right" else _capi.SGM_VIEW_LEFT
        p.p1, p.p2 = p1, p2
        p.uniqueness, p.lr_max_diff = uniqueness, lr_max_diff
        self.params = p
        self.h, self.w, self.scale, self.max_disp = h, w, s, d
        self.rows, self.cols = h // s, w // s
        self.invalid_disp = d + 1
        handle = ctypes.c_void_p()
        check(self._lib.sgm_create(ctypes.byref(p), device, ctypes.byref(handle)))
        self._h = handle
        self.device = device
        self._lr = np.full((self.rows, self.cols), self.invalid_disp, np.float32)
        self._raw = np.zeros((self.rows, self.cols), np.uint16)
        self._final = None

    # ---------------------------------------------------------- lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.sgm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def device_bytes(self) -> int:
        return int(self._lib.sgm_device_bytes(self._h))

    @property
    def stream(self) -> int:
        """The handle's own stream (sgm_get_stream), as an integer hipStream_t
        for torch.cuda.ExternalStream: work on it is ordered with the calls
        made with stream=None, and those calls record no events."""
        return int(self._lib.sgm_get_stream(self._h) or 0)

    # ------------------------------------------------------------ process
    def process(self, img_l, img_r, sky_mask=None, sky_mask_beta=None) -> None:
        """SGM::process (src/SGM.cpp:32-826, sky overload :829-834)."""
        l = _u8(img_l, (self.h, self.w), "img_l")
        r = _u8(img_r, (self.h, self.w), "img_r")
        sl = None if sky_mask is None or np.size(sky_mask) == 0 else \
            _u8(sky_mask, (self.rows, self.cols), "sky_mask")
        sr = None if sky_mask_beta is None or np.size(sky_mask_beta) == 0 else \
            _u8(sky_mask_beta, (self.rows, self.cols), "sky_mask_beta")
        # Fresh output maps per frame: the arrays handed out by get_disp() /
        # get_lr_disp() / get_raw_disp() for one frame are never overwritten
        # by the next (the reference's get_disp() reference is valid until the
        # next process(), inc/Solver.h:36; a copy-free handle-owned buffer
        # would alias the previous frame's result).
        out = np.empty((self.rows, self.cols), np.float32)
        raw = np.empty((self.rows, self.cols), np.uint16)
        check(self._lib.sgm_process(self._h, _ptr(l), _ptr(r), self.w, _ptr(sl), _ptr(sr),
                                    self.cols, _ptr(out), self.cols, _ptr(raw)),
              self._h)
        self._raw = raw
        if self.params.post_filter or self.params.lk_refine:  # sgm_process returned the final map
            self._final, self._lr = out, None
        else:
            self._final, self._lr = None, out

    def process_device(self, d_left: int, d_right: int, d_out: int, *, pitch: int | None = None,
                       d_sky_l: int = 0, d_sky_r: int = 0, sky_pitch: int | None = None,
                       out_pitch: int | None = None, d_raw: int = 0, stream: int | None = None) -> None:
        """Device-pointer variant (sgm_process_device): enqueue on `stream`
        (None: the handle's own stream; a torch stream's `cuda_stream`,
        including 0 for torch's default stream: that stream)."""
        check(self._lib.sgm_process_device(
            self._h, ctypes.c_void_p(d_left), ctypes.c_void_p(d_right), pitch or self.w,
            ctypes.c_void_p(d_sky_l or None), ctypes.c_void_p(d_sky_r or None),
            sky_pitch or self.cols, ctypes.c_void_p(d_out), out_pitch or self.cols,
            ctypes.c_void_p(d_raw or None), _stream(stream)), self._h)

    def check(self) -> None:
        """sgm_check: wait for the frames enqueued so far and raise SGMError
        (SGM_ERR_HIP) if a slanted-pass hand-off gave up in any of them since
        the last report (their maps are invalid).  Call it after
        synchronising and before gathering or timing device maps."""
        check(self._lib.sgm_check(self._h), self._h)

    def get_disp(self) -> np.ndarray:
        """Post-filtered disparity (inc/Solver.h:36: filtered_disp after
        post_filter, Solver.cpp:600-649), computed on the GPU; invalid = D+1."""
        if self._final is None:
            self._final = self.post_filter(self._lr)
        return self._final

    def get_lr_disp(self) -> np.ndarray:
        """Sub-pixel disparity after the LR check (SGM.cpp:803-818)."""
        if self._lr is None:
            raise RuntimeError("constructed with post_filter=True: only get_disp() is kept")
        return self._lr

    def lr_check_device(self, d_fl: int, d_fr: int, d_out: int, *, fl_pitch: int | None = None,
                        fr_pitch: int | None = None, out_pitch: int | None = None,
                        stream: int | None = None) -> None:
        """The LR check (SGM.cpp:803-818) of two device sub-pixel maps, e.g.
        the left and right views computed on two GPUs (sgm_lr_check_device);
        d_out may be d_fl."""
        check(self._lib.sgm_lr_check_device(
            self._h, ctypes.c_void_p(d_fl), fl_pitch or self.cols, ctypes.c_void_p(d_fr),
            fr_pitch or self.cols, ctypes.c_void_p(d_out), out_pitch or self.cols,
            _stream(stream)), self._h)

    def post_filter(self, disp) -> np.ndarray:
        """post_filter() (Solver.cpp:600-649) of a rows x cols map on the GPU
        (sgm_stage_post_filter); returns a filtered copy."""
        f = np.array(disp, dtype=np.float32, copy=True, order="C")
        if f.shape != (self.rows, self.cols):
            raise ValueError(f"disp: expected shape {(self.rows, self.cols)}, got {f.shape}")
        check(self._lib.sgm_stage_post_filter(self._h, _ptr(f)), self._h)
        return f

    def post_filter_device(self, d_disp: int, *, pitch: int | None = None, stream: int | None = None) -> None:
        """In place on a device map (sgm_post_filter_device)."""
        check(self._lib.sgm_post_filter_device(self._h, ctypes.c_void_p(d_disp),
                                               pitch or self.cols,
                                               _stream(stream)), self._h)

    def lk_refine(self, img_l, img_r, disp) -> np.ndarray:
        """LKSubPixel::LKRefine(img_l, img_r, disp_float) (LKSubPixelImpl.cpp:
        13-235) on the GPU: full-size images, working-grid map; returns a
        refined copy (sgm_stage_lk_refine)."""
        l = _u8(img_l, (self.h, self.w), "img_l")
        r = _u8(img_r, (self.h, self.w), "img_r")
        f = np.array(disp, dtype=np.float32, copy=True, order="C")
        if f.shape != (self.rows, self.cols):
            raise ValueError(f"disp: expected shape {(self.rows, self.cols)}, got {f.shape}")
        check(self._lib.sgm_stage_lk_refine(self._h, _ptr(l), _ptr(r), self.w, _ptr(f)), self._h)
        return f

    def lk_refine_device(self, d_left: int, d_right: int, d_disp: int, *, pitch: int | None = None,
                         disp_pitch: int | None = None, stream: int | None = None) -> None:
        """In place on a device map (sgm_lk_refine_device)."""
        check(self._lib.sgm_lk_refine_device(
            self._h, ctypes.c_void_p(d_left), ctypes.c_void_p(d_right), pitch or self.w,
            ctypes.c_void_p(d_disp), disp_pitch or self.cols, _stream(stream)),
            self._h)

    def sky_detect(self, img) -> np.ndarray:
        """SkyAreaDetector::detect(img, ..., scale) (imageSkyDetector.cpp:166-208)
        on the GPU: u8 mask on the working grid, 255 = sky."""
        img = _u8(img, (self.h, self.w), "img")
        mask = np.empty((self.rows, self.cols), np.uint8)
        check(self._lib.sgm_stage_sky_detect(self._h, _ptr(img), self.w, _ptr(mask)), self._h)
        return mask

    def sky_detect_device(self, d_img: int, d_mask: int, *, pitch: int | None = None,
                          mask_pitch: int | None = None, stream: int | None = None) -> None:
        check(self._lib.sgm_sky_detect_device(self._h, ctypes.c_void_p(d_img), pitch or self.w,
                                              ctypes.c_void_p(d_mask), mask_pitch or self.cols,
                                              _stream(stream)), self._h)

    def colormap(self, disp) -> np.ndarray:
        """Solver::colormap (Solver.cpp:652-707) on the GPU: rows x cols x 3 BGR."""
        f = np.ascontiguousarray(disp, dtype=np.float32)
        if f.shape != (self.rows, self.cols):
            raise ValueError(f"disp: expected shape {(self.rows, self.cols)}, got {f.shape}")
        out = np.empty((self.rows, self.cols, 3), np.uint8)
        check(self._lib.sgm_stage_colormap(self._h, _ptr(f), _ptr(out)), self._h)
        return out

    def point_cloud(self, disp, img, fx, fy, cx, cy, baseline=0.5, max_range=100.0):
        """node.cpp:119-143 on the GPU: (N x 3 float64 points, N u8 gray values)
        in row-major order; img is the node's full-size image."""
        f = np.ascontiguousarray(disp, dtype=np.float32)
        im = np.ascontiguousarray(img, dtype=np.uint8)
        if f.shape != (self.rows, self.cols) or im.shape[0] < self.rows or im.shape[1] < self.cols:
            raise ValueError("disp must be rows x cols and img at least that large")
        cam = _capi.Camera(fx, fy, cx, cy, baseline, max_range)
        xyz = np.empty((self.rows * self.cols, 3), np.float64)
        pix = np.empty(self.rows * self.cols, np.uint8)
        n = ctypes.c_int()
        check(self._lib.sgm_stage_point_cloud(self._h, _ptr(f), _ptr(im), im.shape[1],
                                              ctypes.byref(cam), _ptr(xyz), _ptr(pix),
                                              ctypes.byref(n)), self._h)
        return xyz[:n.value].copy(), pix[:n.value].copy()

    def get_raw_disp(self) -> np.ndarray:
        """Left WTA disparity (SGM.cpp:411-415; disp_beta, :755-795, for a
        right-view handle), uint16, invalid = D+1."""
        return self._raw

    # ---------------------------------------------------------- profiling
    def set_profiling(self, enable: bool) -> None:
        check(self._lib.sgm_set_profiling(self._h, int(bool(enable))), self._h)

    def get_profile(self) -> dict:
        """{kernel class: (launches, total_ms, elements per launch)}; resets."""
        buf = (_capi.KernelStat * 64)()
        n = ctypes.c_int()
        check(self._lib.sgm_get_profile(self._h, buf, 64, ctypes.byref(n)), self._h)
        return {buf[k].name.decode(): (buf[k].launches, buf[k].total_ms, buf[k].elems)
                for k in range(n.value)}

    # ------------------------------------------------------------- stages
    def stage_census(self, img) -> np.ndarray:
        img = _u8(img, (self.h, self.w), "img")
        out = np.empty((self.rows, self.cols), np.uint64)
        check(self._lib.sgm_stage_census(self._h, _ptr(img), self.w, _ptr(out)), self._h)
        return out

    def stage_cost(self, ctl, ctr, view=0, sky=None, filters=3) -> np.ndarray:
        ctl = np.ascontiguousarray(ctl, np.uint64)
        ctr = np.ascontiguousarray(ctr, np.uint64)
        sky = None if sky is None else _u8(sky, (self.rows, self.cols), "sky")
        out = np.empty((self.rows, self.cols, self.max_disp), np.float32)
        check(self._lib.sgm_stage_cost(self._h, _ptr(ctl), _ptr(ctr), _ptr(sky), view, filters,
                                       _ptr(out)), self._h)
        return out

    def stage_path(self, direction: int, cost):
        cost = np.ascontiguousarray(cost, np.float32)
        L = np.empty_like(cost)
        m = np.empty((self.rows, self.cols), np.float32)
        check(self._lib.sgm_stage_path(self._h, direction, _ptr(cost), _ptr(L), _ptr(m)),
              self._h)
        return L, m

    def stage_aggregate(self, cost):
        cost = np.ascontiguousarray(cost, np.float32)
        d = np.empty((self.rows, self.cols), np.uint16)
        f = np.empty((self.rows, self.cols), np.float32)
        check(self._lib.sgm_stage_aggregate(self._h, _ptr(cost), _ptr(d), _ptr(f)), self._h)
        return d, f

    def stage_lr(self, fl, fr) -> np.ndarray:
        fl = np.ascontiguousarray(fl, np.float32)
        fr = np.ascontiguousarray(fr, np.float32)
        out = np.empty_like(fl)
        check(self._lib.sgm_stage_lr(self._h, _ptr(fl), _ptr(fr), _ptr(out)), self._h)
        return out


class BM(SGM):
    """Block matcher on one MI355X: mirrors ``BM(int h, int w, int s, int d)``
    (inc/BM.h:6-19, src/BM.cpp:4-97): census cost + the two cost filters and a
    winner-take-all on the filtered cost (uniqueness |d1 - d2| > 2), then
    post_filter().  get_disp() is the post-filtered integer disparity (the
    reference's BM never writes filtered_disp); get_raw_disp() the
    WTA result."""

    def __init__(self, h: int, w: int, s: int = 1, d: int = 128, *, device: int = 0,
                 blur: bool = True, uniqueness: float = 0.7, sky_detect: bool = False):
        super().__init__(h, w, s, d, device=device, blur=blur, views=1, uniqueness=uniqueness,
                         post_filter=True, sky_detect=sky_detect, _solver=_capi.SGM_SOLVER_BM)


class GPU_SGM(SGM):
    """Mirrors the reference's CUDA backend class ``GPU_SGM(int h, int w, int s,
    int d)`` (gpu_sgm/inc/SGM.cuh:23-62; node.cpp:50 holds its commented-out
    call site): process(l, r) runs the LEFT view only -- SGM, WTA, sub-pixel,
    then post_filter (gpu_sgm/src/SGM.cu:105-232) -- and get_disp() returns
    that post-filtered map.  Results follow the reference's CPU path bit for bit
    (src/SGM.cpp:32-443, Solver.cpp:569-649), not the CUDA tree's
    approximations."""

    def __init__(self, h: int, w: int, s: int = 1, d: int = 128, *, device: int = 0):
        super().__init__(h, w, s, d, device=device, views=1, post_filter=True)
