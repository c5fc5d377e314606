"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use this as the checker / baseline; the product path never
does. Buffers are numpy uint8 arrays.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_size_t, c_uint, c_uint32, c_void_p

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return ORACLE_SO


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        build()
    L = ctypes.CDLL(ORACLE_SO)
    PP = POINTER(c_void_p)
    L.ro_rs_new.restype = c_void_p
    L.ro_rs_new.argtypes = [c_int, c_int]
    L.ro_rs_delete.argtypes = [c_void_p]
    L.ro_rs_matrix.restype = POINTER(c_uint)
    L.ro_rs_matrix.argtypes = [c_void_p]
    L.ro_gf_tables.argtypes = [POINTER(c_uint)] * 3
    L.ro_gf_mult.restype = c_uint
    L.ro_gf_mult.argtypes = [c_void_p, c_uint, c_uint]
    L.ro_rs_get_encoding_id.argtypes = [c_int] * 4
    L.ro_rs_get_data_id.argtypes = [c_int] * 4
    L.ro_rs_multadd.argtypes = [c_void_p, c_size_t, c_void_p, c_uint, c_void_p]
    L.ro_rs_identify_rows.argtypes = [c_void_p, c_int, POINTER(c_int), POINTER(c_uint), POINTER(c_int)]
    L.ro_rs_gaussian_solve.argtypes = [c_void_p, POINTER(c_uint), c_int, c_size_t, PP]
    L.ro_rs_encode_set.argtypes = [c_void_p, c_size_t, PP, PP, c_size_t]
    L.ro_rs_rebuild_set.restype = c_int
    L.ro_rs_rebuild_set.argtypes = [c_void_p, c_size_t, c_int, POINTER(c_int), PP, PP, c_size_t]
    L.ro_xor_encode_set.argtypes = [c_int, c_size_t, PP, PP, c_size_t]
    L.ro_xor_rebuild_set.argtypes = [c_int, c_size_t, c_int, PP, PP, c_size_t]
    L.ro_rs_encode_pthreads.restype = c_int
    L.ro_rs_encode_pthreads.argtypes = [c_void_p, c_size_t, PP, PP, c_size_t, c_int, c_int, c_int]
    L.ro_xor_encode_pthreads.restype = c_int
    L.ro_xor_encode_pthreads.argtypes = [c_int, c_size_t, PP, PP, c_size_t, c_int, c_int, c_int]
    L.ro_crc32.restype = c_uint32
    L.ro_crc32.argtypes = [c_uint32, c_void_p, c_size_t]
    _lib = L
    return L


def _pp(arrs):
    out = (c_void_p * len(arrs))()
    for i, a in enumerate(arrs):
        assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
        out[i] = a.ctypes.data
    return out


def gf_tables():
    L = load()
    lg, ex, im = (c_uint * 256)(), (c_uint * 256)(), (c_uint * 256)()
    L.ro_gf_tables(lg, ex, im)
    return np.array(lg[:], np.uint32), np.array(ex[:], np.uint32), np.array(im[:], np.uint32)


class OracleRS:
    """Oracle state for (ranks, encoding)."""

    def __init__(self, ranks: int, encoding: int):
        self.L = load()
        self.h = self.L.ro_rs_new(ranks, encoding)
        if not self.h:
            raise ValueError(f"invalid RS parameters ranks={ranks} encoding={encoding}")
        self.ranks, self.encoding = ranks, encoding

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ro_rs_delete(self.h)
            self.h = None

    def matrix(self) -> np.ndarray:
        p, e = self.ranks, self.encoding
        m = np.ctypeslib.as_array(self.L.ro_rs_matrix(self.h), shape=((p + e) * p,))
        return m.astype(np.uint32).reshape(p + e, p).copy()

    def mult(self, a: int, b: int) -> int:
        return self.L.ro_gf_mult(self.h, a, b)

    def encoding_id(self, rank, chunk):
        return self.L.ro_rs_get_encoding_id(self.ranks, self.encoding, rank, chunk)

    def data_id(self, rank, chunk):
        return self.L.ro_rs_get_data_id(self.ranks, self.encoding, rank, chunk)

    def multadd(self, buf: np.ndarray, coeff: int, data: np.ndarray):
        if data.size < buf.size:
            raise ValueError(f"multadd: {data.size} B of data for {buf.size} B of buffer")
        self.L.ro_rs_multadd(self.h, buf.size, buf.ctypes.data, coeff, data.ctypes.data)

    def encode_set(self, lofi, parity, chunk_size: int, slice_bytes: int = 1 << 20):
        self.L.ro_rs_encode_set(self.h, chunk_size, _pp(lofi), _pp(parity), slice_bytes)

    def rebuild_set(self, rebuild_ranks, lofi, parity, chunk_size: int, slice_bytes: int = 1 << 20) -> int:
        r = sorted(rebuild_ranks)
        arr = (c_int * max(1, len(r)))(*r)
        return self.L.ro_rs_rebuild_set(self.h, chunk_size, len(r), arr, _pp(lofi), _pp(parity), slice_bytes)

    def encode_pthreads(self, lofi, parity, chunk_size, slice_bytes=1 << 20, nthreads=0, lo=0, hi=None) -> int:
        hi = self.ranks if hi is None else hi
        return self.L.ro_rs_encode_pthreads(
            self.h, chunk_size, _pp(lofi), _pp(parity), slice_bytes, nthreads, lo, hi
        )

    def identify_rows(self, unknowns):
        m = len(unknowns)
        u = (c_int * m)(*unknowns)
        mat = (c_uint * (m * m))()
        rows = (c_int * m)()
        self.L.ro_rs_identify_rows(self.h, m, u, mat, rows)
        return np.array(mat[:], np.uint32).reshape(m, m), list(rows[:])


def xor_encode_set(ranks, lofi, xorc, chunk_size, slice_bytes=1 << 20):
    load().ro_xor_encode_set(ranks, chunk_size, _pp(lofi), _pp(xorc), slice_bytes)


def xor_rebuild_set(ranks, root, lofi, xorc, chunk_size, slice_bytes=1 << 20):
    load().ro_xor_rebuild_set(ranks, chunk_size, root, _pp(lofi), _pp(xorc), slice_bytes)


def xor_encode_pthreads(ranks, lofi, xorc, chunk_size, slice_bytes=1 << 20, nthreads=0, lo=0, hi=None) -> int:
    hi = ranks if hi is None else hi
    return load().ro_xor_encode_pthreads(ranks, chunk_size, _pp(lofi), _pp(xorc), slice_bytes, nthreads, lo, hi)


def crc32(buf: np.ndarray, crc: int = 0) -> int:
    return load().ro_crc32(crc, buf.ctypes.data, buf.size)


def random_set(ranks: int, data_cells: int, parity_cells: int, chunk_size: int, seed: int):
    """Per-member logical files (data_cells * chunk) of random bytes + zeroed parity."""
    rng = np.random.default_rng(seed)
    lofi = [rng.integers(0, 256, size=data_cells * chunk_size, dtype=np.uint8) for _ in range(ranks)]
    parity = [np.zeros(parity_cells * chunk_size, dtype=np.uint8) for _ in range(ranks)]
    return lofi, parity
