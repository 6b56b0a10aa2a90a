"""stereo_matching_amd -- MI355X-native semi-global stereo matcher.

Drop-in for hilbertw/stereo_matching's SGM hot path (census + Hamming cost,
8-path DP, WTA/uniqueness/sub-pixel, LR check) as hand-written gfx950 HIP
kernels behind the C-ABI of libsgm_hip.so (include/sgm_hip.h), plus the
stages around it: post_filter, LKRefine, the sky detector and the BM solver.
"""
from ._capi import LIB_PATH, SGMError, build, lib  # noqa: F401
from .solver import BM, GPU_SGM, SGM  # noqa: F401
from . import synthetic  # noqa: F401

DIRECTIONS = ("L1", "L2", "L3", "L4", "L5", "L6", "L7", "L8")
