"""CPU checks of the C-ABI library: it is built for gfx950, loads, exports
every entry point include/sgm_hip.h declares, and validates arguments the way
the reference's asserts do -- without running any kernel."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest

from stereo_matching_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sgm_hip.h")


def header_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(sgm_[a-z_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_capi.LIB_PATH):
        _capi.build()
    return _capi.lib()


def test_header_and_binding_agree():
    assert header_symbols() == sorted(_capi.EXPORTS)


def test_library_exports_every_symbol(lib):
    for name in header_symbols():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for name in header_symbols():
        assert re.search(rf"\bT {name}$", out, re.M), name


def test_library_carries_gfx950_code_object():
    # the embedded HIP fat binary names its offload targets
    data = open(_capi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_default_params_are_the_reference_constants(lib):
    p = _capi.default_params(375, 1242, 1, 128)
    assert (p.p1, p.p2) == (10, 100)                # src/SGM.cpp:27-28
    assert abs(p.uniqueness - 0.7) < 1e-7           # inc/Solver.h:14
    assert p.lr_max_diff == 1.0                     # inc/Solver.h:16
    assert p.blur == 1 and p.views == 2 and p.scale == 1 and p.max_disp == 128
    assert p.view == _capi.SGM_VIEW_LEFT and p.post_filter == 0 and p.aux_only == 0


@pytest.mark.parametrize("h,w,s,d", [(375, 1242, 3, 128), (375, 1242, 1, 96), (0, 10, 1, 32),
                                     (2, 100, 1, 32), (100, 4, 1, 32)])
def test_invalid_arguments_rejected(lib, h, w, s, d):
    # the reference asserts (Solver.cpp:6-10); the C-ABI returns SGM_ERR_INVALID_ARG
    p = _capi.Params()
    lib.sgm_default_params(ctypes.byref(p), h, w, s, d)
    handle = ctypes.c_void_p()
    rc = lib.sgm_create(ctypes.byref(p), 0, ctypes.byref(handle))
    assert rc == _capi.SGM_ERR_INVALID_ARG
    assert not handle.value


@pytest.mark.parametrize("fields", [{"solver": 7}, {"sky_detect": 1, "width": 9000, "height": 100},
                                    {"sky_detect": 1, "height": 5000, "width": 100}, {"views": 3},
                                    {"view": 2}, {"view": 1},                      # views == 2
                                    {"view": 1, "views": 1, "post_filter": 1},
                                    {"view": 1, "views": 1, "lk_refine": 1},
                                    {"view": 1, "views": 1, "solver": 1},
                                    # uniqueness ratios at which SGM.cpp:392-408 reads the
                                    # previous pixel's sec_min_d: 0, negative,
                                    # below 8 (P2 + 999999) / FLT_MAX
                                    {"uniqueness": 0.0}, {"uniqueness": -0.5},
                                    {"uniqueness": 1e-33}, {"uniqueness": float("nan")}])
def test_invalid_stage_parameters_rejected(lib, fields):
    # parameters of the section-8f stages and of the view split are checked
    # at sgm_create, before any device work (sky detector limits: sgm_sky.hip)
    p = _capi.Params()
    lib.sgm_default_params(ctypes.byref(p), 375, 1242, 1, 64)
    for field, value in fields.items():
        setattr(p, field, value)
    handle = ctypes.c_void_p()
    assert lib.sgm_create(ctypes.byref(p), 0, ctypes.byref(handle)) == _capi.SGM_ERR_INVALID_ARG
    assert not handle.value


def test_stage_entry_points_reject_null(lib):
    for fn, nargs in (("sgm_post_filter_device", 4), ("sgm_lk_refine_device", 7),
                      ("sgm_sky_detect_device", 6), ("sgm_colormap_device", 6),
                      ("sgm_point_cloud_device", 10), ("sgm_stage_post_filter", 2),
                      ("sgm_stage_lk_refine", 5), ("sgm_stage_sky_detect", 4),
                      ("sgm_stage_colormap", 3), ("sgm_stage_point_cloud", 8),
                      ("sgm_lr_check_device", 8)):
        f = getattr(lib, fn)
        assert len(f.argtypes) == nargs, fn
        args = [0 if t is ctypes.c_int else None for t in f.argtypes]
        assert f(*args) == _capi.SGM_ERR_INVALID_ARG, fn


def test_null_arguments_rejected(lib):
    assert lib.sgm_create(None, 0, None) == _capi.SGM_ERR_INVALID_ARG
    assert lib.sgm_destroy(None) == _capi.SGM_ERR_INVALID_ARG
    assert lib.sgm_process(None, None, None, 0, None, None, 0, None, 0, None) == \
        _capi.SGM_ERR_INVALID_ARG


def test_no_silent_fallback_without_gpu(lib):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    from stereo_matching_amd import SGM, SGMError
    with pytest.raises(SGMError):
        SGM(375, 1242, 1, 128)


def test_check_and_comm_reject_null(lib):
    # sgm_check and the multi-GPU exchange validate before touching a device
    assert lib.sgm_check(None) == _capi.SGM_ERR_INVALID_ARG
    h = ctypes.c_void_p()
    assert lib.sgm_comm_create(None, 1, ctypes.byref(h)) == _capi.SGM_ERR_INVALID_ARG
    assert lib.sgm_comm_create((ctypes.c_int * 1)(0), 0, ctypes.byref(h)) == _capi.SGM_ERR_INVALID_ARG
    assert lib.sgm_comm_create((ctypes.c_int * 1)(0), 1, None) == _capi.SGM_ERR_INVALID_ARG
    assert not h.value
    assert lib.sgm_comm_create_rank(None, 1, 0, 0, ctypes.byref(h)) == _capi.SGM_ERR_INVALID_ARG
    uid = b"\0" * _capi.SGM_COMM_ID_BYTES
    assert lib.sgm_comm_create_rank(uid, 2, 2, 0, ctypes.byref(h)) == _capi.SGM_ERR_INVALID_ARG
    assert b"nranks or rank" in lib.sgm_comm_last_error(None)
    assert lib.sgm_comm_create_rank(uid, 0, 0, 0, ctypes.byref(h)) == _capi.SGM_ERR_INVALID_ARG
    assert lib.sgm_comm_unique_id(None) == _capi.SGM_ERR_INVALID_ARG
    assert lib.sgm_comm_destroy(None) == _capi.SGM_ERR_INVALID_ARG
    assert lib.sgm_comm_info(None, None, None, None) == _capi.SGM_ERR_INVALID_ARG
    assert lib.sgm_batch_gather(None, 0, None, 1, 1, 1, None, None) == _capi.SGM_ERR_INVALID_ARG
    assert lib.sgm_batch_gather_all(None, None, 1, 1, 1, None, None) == _capi.SGM_ERR_INVALID_ARG


def test_comm_without_gpu(lib):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    # (a duplicated device list: no device, or refused as a duplicate)
    rc = lib.sgm_comm_create((ctypes.c_int * 2)(0, 0), 2, ctypes.byref(h))
    assert rc in (_capi.SGM_ERR_NO_DEVICE, _capi.SGM_ERR_INVALID_ARG)
    assert lib.sgm_comm_create((ctypes.c_int * 1)(0), 1, ctypes.byref(h)) == _capi.SGM_ERR_NO_DEVICE
    assert b"no HIP device" in lib.sgm_comm_last_error(None)
    assert not h.value
