"""HBM-resident batch API over dssg_*_device (torch is plumbing only: device
allocations and the stream handle; every computation is a HIP kernel).

Used by bench.py: inputs are uploaded once, then each step covers a batch of
query footprints and joins it against a resident EntityIndex without any
host round trip of the data.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib


def _torch():
    import torch  # plumbing only
    return torch


@dataclass
class DeviceFootprints:
    n: int
    kind: object   # torch int32 [n]
    voff: object   # torch int64 [n+1]
    lat: object    # torch float64
    lng: object
    radius_m: object  # torch float32 [n]

    @classmethod
    def upload(cls, fp, device="cuda"):
        t = _torch()
        return cls(int(len(fp.kind)), t.as_tensor(fp.kind, device=device), t.as_tensor(fp.voff, device=device),
                   t.as_tensor(fp.lat, device=device), t.as_tensor(fp.lng, device=device),
                   t.as_tensor(fp.radius_m, device=device))


def _ptr(x):
    return C.c_void_p(int(x.data_ptr()))


def _stream_ptr():
    t = _torch()
    return C.c_void_p(int(t.cuda.current_stream().cuda_stream))


def cover(ctx: _lib.Context, fp: DeviceFootprints) -> _lib.Cells:
    """dssg_cover_batch_device; the returned device pointers stay valid until
    the next cover() on the same context."""
    out = _lib.Cells()
    ctx.check(ctx.L.dssg_cover_batch_device(ctx.h, fp.n, _ptr(fp.kind), _ptr(fp.voff), _ptr(fp.lat), _ptr(fp.lng),
                                            _ptr(fp.radius_m), _stream_ptr(), C.byref(out)))
    return out


def build_index(ctx: _lib.Context, cells: _lib.Cells, alt_lo, alt_hi, t0, t1, owner=None,
                cell_range=None) -> C.c_void_p:
    """dssg_index_build_device from a device covering (entities = footprints);
    cell_range=(lo, hi): a cell-range shard (dssg_index_build_range_device)."""
    h = C.c_void_p()
    lo, hi = cell_range if cell_range is not None else (0, 2**64 - 1)
    ctx.check(ctx.L.dssg_index_build_range_device(ctx.h, cells.n, C.c_void_p(cells.offs), C.c_void_p(cells.cells),
                                                  _ptr(alt_lo), _ptr(alt_hi), _ptr(t0), _ptr(t1),
                                                  _ptr(owner) if owner is not None else C.c_void_p(0), int(lo),
                                                  int(hi), _stream_ptr(), C.byref(h)))
    return h


def search(ctx: _lib.Context, index: C.c_void_p, cells: _lib.Cells, alt_lo, alt_hi, tlo, thi, owner=None) -> _lib.Pairs:
    out = _lib.Pairs()
    ctx.check(ctx.L.dssg_search_device(ctx.h, index, cells.n, C.c_void_p(cells.offs), C.c_void_p(cells.cells),
                                       _ptr(alt_lo), _ptr(alt_hi), _ptr(tlo), _ptr(thi),
                                       _ptr(owner) if owner is not None else C.c_void_p(0), _stream_ptr(),
                                       C.byref(out)))
    return out


def copy_back(ctx: _lib.Context, ptr: int, n: int, dtype) -> np.ndarray:
    """Device -> host copy of an engine-owned buffer (dssg_copy_to_host)."""
    dst = np.empty(n, dtype=dtype)
    if n:
        ctx.check(ctx.L.dssg_copy_to_host(ctx.h, dst.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), dst.nbytes))
    return dst
