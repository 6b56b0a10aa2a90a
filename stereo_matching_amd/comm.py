"""The C-ABI multi-GPU exchange (include/sgm_hip.h "multi-GPU"): an RCCL
communicator over the devices that hold one stereo pair each, and the gather
of their disparity maps to rank 0 (ncclGather over xGMI).

Python mirror of sgm_comm_* / sgm_batch_gather*, for tests and for callers
that drive several devices from one process; bench.py's torchrun layout uses
torch.distributed (stereo_matching_amd.distributed) instead.  Every call goes
through libsgm_hip.so."""
from __future__ import annotations

import ctypes
from typing import Sequence

from . import _capi
from ._capi import SGMError, lib


def _check(rc: int, comm=None) -> None:
    if rc != _capi.SGM_OK:
        raw = lib().sgm_comm_last_error(comm)
        raise SGMError(rc, raw.decode() if raw else "")


def unique_id() -> bytes:
    """sgm_comm_unique_id: rank 0's id for create_rank (ncclGetUniqueId)."""
    buf = ctypes.create_string_buffer(_capi.SGM_COMM_ID_BYTES)
    _check(lib().sgm_comm_unique_id(buf))
    return buf.raw


class Comm:
    """A communicator: `Comm(devices=[...])` drives every device from this
    process (ncclCommInitAll, ranks = list order); `Comm(uid=..., nranks=,
    rank=, device=)` joins one rank of a multi-process job."""

    def __init__(self, devices: Sequence[int] | None = None, *, uid: bytes | None = None,
                 nranks: int | None = None, rank: int | None = None, device: int | None = None):
        self._lib = lib()
        h = ctypes.c_void_p()
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            _check(self._lib.sgm_comm_create(arr, len(devices), ctypes.byref(h)))
        else:
            if uid is None or len(uid) != _capi.SGM_COMM_ID_BYTES:
                raise ValueError("uid must be the 128 bytes unique_id() returned")
            _check(self._lib.sgm_comm_create_rank(uid, nranks, rank, device, ctypes.byref(h)))
        self._h = h
        n, first, local = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(self._lib.sgm_comm_info(h, ctypes.byref(n), ctypes.byref(first), ctypes.byref(local)), h)
        self.nranks, self.first_rank, self.nlocal = n.value, first.value, local.value

    def gather(self, rank: int, d_map: int, rows: int, cols: int, d_root_out: int = 0, *,
               pitch: int | None = None, stream: int = 0) -> None:
        """sgm_batch_gather: rank `rank`'s device map (pitch in floats) into
        d_root_out[rank] on rank 0; enqueued on `stream` (0: default)."""
        _check(self._lib.sgm_batch_gather(self._h, rank, ctypes.c_void_p(d_map), rows, cols,
                                          pitch or cols, ctypes.c_void_p(d_root_out or None),
                                          ctypes.c_void_p(stream or None)), self._h)

    def gather_all(self, d_maps: Sequence[int], rows: int, cols: int, d_root_out: int, *,
                   pitch: int | None = None, streams: Sequence[int] | None = None) -> None:
        """sgm_batch_gather_all: every local rank's map, one RCCL group."""
        maps = (ctypes.c_void_p * len(d_maps))(*d_maps)
        sts = (ctypes.c_void_p * len(streams))(*[s or None for s in streams]) if streams else None
        _check(self._lib.sgm_batch_gather_all(self._h, maps, rows, cols, pitch or cols,
                                              ctypes.c_void_p(d_root_out), sts), self._h)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.sgm_comm_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
