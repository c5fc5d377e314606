"""Host-resident encode / rebuild through the pinned-buffer pipeline
(include/redset_hip.h, "streaming pipeline"): cells live in host memory or in
files with redset's logical-file layout and stream through HBM."""
from __future__ import annotations

import ctypes
from ctypes import c_char_p, c_int, c_ulonglong, c_void_p
from typing import List, Optional, Sequence, Tuple

from . import _lib


class HostIO:
    """Cells in host memory, laid out like the device set layout."""

    def __init__(self, ranks: int, lofi_ptrs: Sequence[int], parity_ptrs: Sequence[int], cell_stride: int,
                 keepalive=(), pinned: bool = False):
        self.io = _lib.StreamIO()
        h = c_void_p()
        _lib.check(_lib.load().redset_hip_hostio_create(
            ranks, _lib.ptr_array(lofi_ptrs), _lib.ptr_array(parity_ptrs), cell_stride, int(pinned),
            ctypes.byref(self.io), ctypes.byref(h)), "hostio_create")
        self._h = h
        self._keep = keepalive

    def close(self):
        if self._h:
            _lib.load().redset_hip_hostio_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        self.close()


class FileIO:
    """Member r's logical file = concatenation of files[r] = [(path, size), ...];
    parity at redundancy[r] + header[r] + slot * chunk (redset's layout)."""

    def __init__(self, files: Sequence[Sequence[Tuple[str, int]]], redundancy: Sequence[str],
                 headers: Optional[Sequence[int]], chunk: int, writable: Optional[Sequence[bool]] = None):
        p = len(files)
        nfiles = (c_int * p)(*[len(f) for f in files])
        flat = [x for f in files for x in f]
        paths = (c_char_p * max(1, len(flat)))(*[x[0].encode() for x in flat])
        sizes = (c_ulonglong * max(1, len(flat)))(*[int(x[1]) for x in flat])
        reds = (c_char_p * p)(*[x.encode() for x in redundancy])
        hdr = (c_ulonglong * p)(*([int(h) for h in headers] if headers else [0] * p))
        wr = (c_int * p)(*([1 if w else 0 for w in writable] if writable else [0] * p))
        self.io = _lib.StreamIO()
        h = c_void_p()
        _lib.check(_lib.load().redset_hip_fileio_create(
            p, nfiles, paths, sizes, reds, hdr, chunk, wr, ctypes.byref(self.io), ctypes.byref(h)),
            "fileio_create")
        self._h = h

    def close(self):
        if self._h:
            _lib.load().redset_hip_fileio_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        self.close()


def _run(fn, *args) -> dict:
    st = _lib.StreamStats()
    _lib.check(fn(*args, ctypes.byref(st)), fn.__name__)
    return st.as_dict()


def rs_encode_stream(codec, chunk: int, io, first: int = 0, nstripes: int = 0, slice_bytes: int = 0,
                     io_threads: int = 0) -> dict:
    return _run(_lib.load().redset_hip_rs_encode_stream, codec._h, chunk, first, nstripes, slice_bytes,
                io_threads, ctypes.byref(io.io))


def rs_rebuild_stream(codec, lost: Sequence[int], chunk: int, io, first: int = 0, nstripes: int = 0,
                      slice_bytes: int = 0, io_threads: int = 0) -> dict:
    r = sorted(lost)
    arr = (c_int * len(r))(*r)
    return _run(_lib.load().redset_hip_rs_rebuild_stream, codec._h, len(r), arr, chunk, first, nstripes,
                slice_bytes, io_threads, ctypes.byref(io.io))


def xor_encode_stream(ranks: int, chunk: int, io, first: int = 0, nstripes: int = 0, slice_bytes: int = 0,
                      io_threads: int = 0) -> dict:
    return _run(_lib.load().redset_hip_xor_encode_stream, ranks, chunk, first, nstripes, slice_bytes,
                io_threads, ctypes.byref(io.io))


def xor_rebuild_stream(ranks: int, root: int, chunk: int, io, first: int = 0, nstripes: int = 0,
                       slice_bytes: int = 0, io_threads: int = 0) -> dict:
    return _run(_lib.load().redset_hip_xor_rebuild_stream, ranks, root, chunk, first, nstripes, slice_bytes,
                io_threads, ctypes.byref(io.io))


def chunk_size_for(max_bytes: int, data_cells: int) -> int:
    """redset_apply_rs / redset_apply_xor chunk size: ceil(max / data cells),
    at least 1 (src/redset_reedsolomon.c:485-493, src/redset_xor.c:362-370)."""
    c = max_bytes // data_cells
    if c * data_cells < max_bytes:
        c += 1
    return max(1, c)
