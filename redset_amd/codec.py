"""Python face of the HIP codec, for tests, bench and the multi-GPU driver.

The codec itself is the C ABI in ``include/redset_hip.h`` (host C++ planner +
gfx950 kernels). This module only passes device pointers through ctypes;
PyTorch provides device memory and streams. Names follow redset's domain:
a *set* of ``ranks`` members, each with a logical file of data *cells* and a
redundancy region of parity cells; a *stripe* is the row of cells, one per
member, that one parity computation covers.
"""
from __future__ import annotations

import ctypes
from ctypes import c_int, c_ubyte, c_void_p
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib

CELL_ALIGN = 256  # cell_stride rounding in SetLayout (16 B is the kernel's minimum)


def _stream_handle(stream) -> Optional[int]:
    if stream is None:
        try:
            import torch

            if torch.cuda.is_available():
                return torch.cuda.current_stream().cuda_stream
        except Exception:  # pragma: no cover
            pass
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _ptr(x) -> int:
    return x if isinstance(x, int) else x.data_ptr()


class Plan:
    """Prepared kernel launches for one whole-set operation."""

    def __init__(self, handle: c_void_p, keepalive=()):
        self._h = handle
        self._keep = keepalive
        info = _lib.PlanInfo()
        _lib.check(_lib.load().redset_hip_plan_get_info(self._h, ctypes.byref(info)), "plan_get_info")
        self.info = info

    def execute(self, stream=None) -> None:
        _lib.check(_lib.load().redset_hip_plan_execute(self._h, _stream_handle(stream)), "plan_execute")

    @property
    def bytes_read(self) -> int:
        return int(self.info.bytes_read)

    @property
    def bytes_written(self) -> int:
        return int(self.info.bytes_written)

    @property
    def launches(self) -> int:
        """Kernel launches one execute() issues (one per stripe when the
        plan runs its jobs one after another)."""
        return int(self.info.launches)

    def close(self) -> None:
        if self._h:
            _lib.load().redset_hip_plan_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - finaliser
        try:
            self.close()
        except Exception:
            pass


class RSCodec:
    """GF(2^8) tables + encoding matrix for a set of ``ranks`` members with
    ``encoding`` parity cells per stripe (redset_construct_rs,
    src/redset_reedsolomon.c:80-188)."""

    def __init__(self, ranks: int, encoding: int):
        lib = _lib.load()
        h = c_void_p()
        _lib.check(lib.redset_hip_rs_create(ranks, encoding, ctypes.byref(h)), "rs_create")
        self._h = h
        self.ranks = ranks
        self.encoding = encoding

    @property
    def data_cells(self) -> int:
        return self.ranks - self.encoding

    def matrix(self) -> np.ndarray:
        p, e = self.ranks, self.encoding
        buf = (c_ubyte * ((p + e) * p))()
        _lib.check(_lib.load().redset_hip_rs_matrix(self._h, buf), "rs_matrix")
        return np.frombuffer(bytes(buf), dtype=np.uint8).reshape(p + e, p).copy()

    def decode_matrix(self, rebuild_ranks: Sequence[int], chunk_id: int) -> np.ndarray:
        m = len(rebuild_ranks)
        ranks = (c_int * m)(*sorted(rebuild_ranks))
        buf = (c_ubyte * (m * self.ranks))()
        _lib.check(
            _lib.load().redset_hip_rs_decode_matrix(self._h, m, ranks, chunk_id, buf), "rs_decode_matrix"
        )
        return np.frombuffer(bytes(buf), dtype=np.uint8).reshape(m, self.ranks).copy()

    def encoding_id(self, rank: int, chunk_id: int) -> int:
        return _lib.load().redset_hip_rs_get_encoding_id(self.ranks, self.encoding, rank, chunk_id)

    def data_id(self, rank: int, chunk_id: int) -> int:
        return _lib.load().redset_hip_rs_get_data_id(self.ranks, self.encoding, rank, chunk_id)

    def plan_encode(self, lofi, parity, chunk_size: int, cell_stride: Optional[int] = None) -> Plan:
        stride = chunk_size if cell_stride is None else cell_stride
        a, b = _lib.ptr_array([_ptr(x) for x in lofi]), _lib.ptr_array([_ptr(x) for x in parity])
        h = c_void_p()
        _lib.check(
            _lib.load().redset_hip_rs_plan_encode(self._h, a, b, chunk_size, stride, ctypes.byref(h)),
            "rs_plan_encode",
        )
        return Plan(h, (self, lofi, parity))

    def plan_rebuild(self, rebuild_ranks: Sequence[int], lofi, parity, chunk_size: int,
                     cell_stride: Optional[int] = None) -> Plan:
        stride = chunk_size if cell_stride is None else cell_stride
        ranks = sorted(rebuild_ranks)
        r = (c_int * max(1, len(ranks)))(*ranks)
        a, b = _lib.ptr_array([_ptr(x) for x in lofi]), _lib.ptr_array([_ptr(x) for x in parity])
        h = c_void_p()
        _lib.check(
            _lib.load().redset_hip_rs_plan_rebuild(
                self._h, len(ranks), r, a, b, chunk_size, stride, ctypes.byref(h)
            ),
            "rs_plan_rebuild",
        )
        return Plan(h, (self, lofi, parity))

    def close(self) -> None:
        if self._h:
            _lib.load().redset_hip_rs_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def xor_plan_encode(ranks: int, lofi, xorc, chunk_size: int, cell_stride: Optional[int] = None) -> Plan:
    stride = chunk_size if cell_stride is None else cell_stride
    a, b = _lib.ptr_array([_ptr(x) for x in lofi]), _lib.ptr_array([_ptr(x) for x in xorc])
    h = c_void_p()
    _lib.check(
        _lib.load().redset_hip_xor_plan_encode(ranks, a, b, chunk_size, stride, ctypes.byref(h)),
        "xor_plan_encode",
    )
    return Plan(h, (lofi, xorc))


def xor_plan_rebuild(ranks: int, root: int, lofi, xorc, chunk_size: int,
                     cell_stride: Optional[int] = None) -> Plan:
    stride = chunk_size if cell_stride is None else cell_stride
    a, b = _lib.ptr_array([_ptr(x) for x in lofi]), _lib.ptr_array([_ptr(x) for x in xorc])
    h = c_void_p()
    _lib.check(
        _lib.load().redset_hip_xor_plan_rebuild(ranks, root, a, b, chunk_size, stride, ctypes.byref(h)),
        "xor_plan_rebuild",
    )
    return Plan(h, (lofi, xorc))


def gf_combine(inputs, outputs, coeffs: np.ndarray, nbytes: int, accumulate: bool = False, stream=None) -> None:
    """outputs[j] (^)= sum_i coeffs[j, i] * inputs[i] over GF(2^8) (device buffers)."""
    coeffs = np.ascontiguousarray(coeffs, dtype=np.uint8)
    nout, nin = coeffs.shape
    assert len(inputs) == nin and len(outputs) == nout
    c = (c_ubyte * coeffs.size).from_buffer_copy(coeffs.tobytes())
    _lib.check(
        _lib.load().redset_hip_gf_combine(
            _lib.ptr_array([_ptr(x) for x in inputs]), nin,
            _lib.ptr_array([_ptr(x) for x in outputs]), nout,
            c, nbytes, int(accumulate), _stream_handle(stream),
        ),
        "gf_combine",
    )


def xor_combine(inputs, output, nbytes: int, accumulate: bool = False, stream=None) -> None:
    _lib.check(
        _lib.load().redset_hip_xor_combine(
            _lib.ptr_array([_ptr(x) for x in inputs]), len(inputs), _ptr(output), nbytes,
            int(accumulate), _stream_handle(stream),
        ),
        "xor_combine",
    )


@dataclass
class SetLayout:
    """Device-resident layout of one redundancy set (see include/redset_hip.h).

    Member r's logical file = ``data_cells`` cells and its redundancy region =
    ``parity_cells`` cells, every cell ``cell_stride`` bytes apart (chunk_size
    rounded up to CELL_ALIGN). One allocation holds the whole set.
    """

    ranks: int
    data_cells: int
    parity_cells: int
    chunk_size: int
    cell_stride: int
    storage: object  # torch.uint8 tensor

    @classmethod
    def allocate(cls, ranks: int, data_cells: int, parity_cells: int, chunk_size: int, device="cuda",
                 pad: int = 0):
        """``pad`` extra bytes after every cell (rounded to CELL_ALIGN): moves
        the cells of a stripe relative to each other in HBM."""
        import torch

        stride = max(CELL_ALIGN, -(-chunk_size // CELL_ALIGN) * CELL_ALIGN)
        stride += -(-pad // CELL_ALIGN) * CELL_ALIGN
        per = (data_cells + parity_cells) * stride
        storage = torch.empty(ranks * per, dtype=torch.uint8, device=device)
        return cls(ranks, data_cells, parity_cells, chunk_size, stride, storage)

    @property
    def member_bytes(self) -> int:
        return (self.data_cells + self.parity_cells) * self.cell_stride

    def lofi(self, r: int):
        base = r * self.member_bytes
        return self.storage[base: base + self.data_cells * self.cell_stride]

    def parity(self, r: int):
        base = r * self.member_bytes + self.data_cells * self.cell_stride
        return self.storage[base: base + self.parity_cells * self.cell_stride]

    def data_cell(self, r: int, s: int):
        return self.lofi(r)[s * self.cell_stride: s * self.cell_stride + self.chunk_size]

    def parity_cell(self, r: int, i: int):
        return self.parity(r)[i * self.cell_stride: i * self.cell_stride + self.chunk_size]

    def lofi_ptrs(self):
        return [self.lofi(r).data_ptr() for r in range(self.ranks)]

    def parity_ptrs(self):
        return [self.parity(r).data_ptr() for r in range(self.ranks)]


def cell_stride(chunk_size: int) -> int:
    """The library's recommended cell stride for a set held in one
    allocation (include/redset_hip.h redset_hip_cell_stride)."""
    return int(_lib.load().redset_hip_cell_stride(chunk_size))


def ring_faults(clear: bool = True) -> int:
    """Capped loader-ring handshake spins on the current device since the
    last clearing read (include/redset_hip.h redset_hip_ring_faults). Outputs
    are correct either way -- a capped spin falls back to direct HBM loads --
    so this is a stall counter: 0 means every launch's ring handshake
    completed in time. Synchronises the device."""
    from ctypes import c_uint

    n = c_uint(0)
    _lib.check(_lib.load().redset_hip_ring_faults(ctypes.byref(n), int(clear)), "ring_faults")
    return int(n.value)


def hang_faults(clear: bool = True, stream=None) -> int:
    """Capped HANG waits on the current device since the last clearing read
    (include/redset_hip.h redset_hip_hang_faults): waits with no fallback
    that gave up, so some launch's outputs are wrong. 0 on every healthy
    run. Read in order on `stream` (default: the library's own stream, after
    nothing -- synchronise the work to be counted first)."""
    from ctypes import c_uint

    n = c_uint(0)
    h = None if stream is None else _stream_handle(stream)
    _lib.check(_lib.load().redset_hip_hang_faults(h, ctypes.byref(n), int(clear)), "hang_faults")
    return int(n.value)
