"""ctypes binding of the in-tree HIP codec library (redset_amd/lib/libredset_hip.so).

The library is the product: every codec call below goes through it. There is
no CPU fallback -- if the shared object is missing or fails to load, importing
:mod:`redset_amd` still works (so CPU-only tooling can inspect the package),
but the first call raises :class:`RedsetHipUnavailable` loudly.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_size_t, c_ubyte, c_uint, c_ulonglong, c_void_p

# REDSET_HIP_LIBRARY points at another build of the same library (the test
# twin redset_amd/lib_test/, whose planner honours the test knobs)
LIB_PATH = os.environ.get("REDSET_HIP_LIBRARY") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "lib", "libredset_hip.so")

REDSET_SUCCESS = 0
REDSET_FAILURE = 1

PLAN_RS_ENCODE = 1
PLAN_RS_REBUILD = 2
PLAN_XOR_ENCODE = 3
PLAN_XOR_REBUILD = 4

# every symbol include/redset_hip.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = (
    "redset_hip_rs_create",
    "redset_hip_rs_destroy",
    "redset_hip_rs_matrix",
    "redset_hip_rs_shape",
    "redset_hip_rs_get_encoding_id",
    "redset_hip_rs_get_data_id",
    "redset_hip_cell_stride",
    "redset_hip_rs_plan_encode",
    "redset_hip_rs_plan_rebuild",
    "redset_hip_xor_plan_encode",
    "redset_hip_xor_plan_rebuild",
    "redset_hip_plan_execute",
    "redset_hip_plan_get_info",
    "redset_hip_plan_destroy",
    "redset_hip_gf_combine",
    "redset_hip_xor_combine",
    "redset_hip_rs_decode_matrix",
    "redset_hip_ring_faults",
    "redset_hip_hang_faults",
    "redset_hip_test_build",
    "redset_hip_last_error",
    "redset_hip_record_error",
    "redset_hip_version",
    "redset_hip_rs_encode_stream",
    "redset_hip_rs_rebuild_stream",
    "redset_hip_xor_encode_stream",
    "redset_hip_xor_rebuild_stream",
    "redset_hip_hostio_create",
    "redset_hip_hostio_destroy",
    "redset_hip_release_scratch",
    "redset_hip_fileio_create",
    "redset_hip_fileio_destroy",
    "redset_hip_shard_slice_bytes",
    "redset_hip_rs_sharded_plan",
    "redset_hip_xor_sharded_plan",
    "redset_hip_rs_sharded_plan_on",
    "redset_hip_xor_sharded_plan_on",
    "redset_hip_sharded_execute",
    "redset_hip_sharded_execute_phase",
    "redset_hip_sharded_get_info",
    "redset_hip_sharded_destroy",
    "redset_hip_rccl_available",
    "redset_hip_rccl_unique_id",
    "redset_hip_rccl_transport_create",
    "redset_hip_rccl_transport_destroy",
    "redset_hip_plan_combine",
    "redset_hip_rs_sharded_plan_ex",
    "redset_hip_xor_sharded_plan_ex",
    "redset_hip_sharded_get_shape",
    "redset_hip_abi_version",
)

# include/redset_hip.h REDSET_HIP_ABI_VERSION: the struct layouts below
ABI_VERSION = 6

PHASE_GATHER = 0
PHASE_COMPUTE = 1
PHASE_RETURN = 2
PHASE_ACCUMULATE = 3
# every phase of one execute, in order (either shape)
PHASES = (PHASE_GATHER, PHASE_COMPUTE, PHASE_RETURN, PHASE_ACCUMULATE)

SHAPE_AUTO = 0
SHAPE_GATHER = 1
SHAPE_REDUCE = 2
SHAPE_NAMES = {SHAPE_AUTO: "auto", SHAPE_GATHER: "gather", SHAPE_REDUCE: "reduce"}


class RedsetHipUnavailable(RuntimeError):
    """The HIP codec library could not be loaded."""


class RedsetHipError(RuntimeError):
    """A codec call returned REDSET_FAILURE."""


class PlanInfo(ctypes.Structure):
    _fields_ = [
        ("kind", c_int),
        ("ranks", c_int),
        ("encoding", c_int),
        ("missing", c_int),
        ("launches", c_int),
        ("jobs", c_int),
        ("chunk_size", c_size_t),
        ("bytes_read", c_ulonglong),
        ("bytes_written", c_ulonglong),
    ]


class StreamIO(ctypes.Structure):
    """redset_hip_io: read/write callbacks + context (opaque here)."""

    _fields_ = [("read", c_void_p), ("write", c_void_p), ("map", c_void_p), ("ctx", c_void_p)]


class StreamStats(ctypes.Structure):
    _fields_ = [
        ("seconds", ctypes.c_double),
        ("bytes_read", c_ulonglong),
        ("bytes_written", c_ulonglong),
        ("units", c_ulonglong),
        ("read_seconds", ctypes.c_double),
        ("write_seconds", ctypes.c_double),
        ("gpu_seconds", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Xfer(ctypes.Structure):
    """redset_hip_xfer: one message (or half of a local copy) of an exchange."""

    _fields_ = [("peer", c_int), ("send", c_int), ("buf", c_void_p), ("len", c_size_t)]


EXCHANGE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, POINTER(Xfer), c_int, c_void_p)
COMPUTE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_int, c_int, POINTER(c_int), POINTER(c_void_p), POINTER(c_void_p),
                              c_size_t, c_size_t, c_void_p)


class CombineJob(ctypes.Structure):
    """redset_hip_combine_job: out[j] = (out[j] ^) sum_i coef[j*nin+i] * in[i]."""

    _fields_ = [("nin", c_int), ("nout", c_int), ("inp", POINTER(c_void_p)), ("out", POINTER(c_void_p)),
                ("coef", POINTER(c_ubyte)), ("accumulate", c_int)]


COMBINE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, POINTER(CombineJob), c_int, c_size_t, c_void_p)


class Transport(ctypes.Structure):
    _fields_ = [("world", c_int), ("rank", c_int), ("exchange", c_void_p), ("ctx", c_void_p)]


class Compute(ctypes.Structure):
    _fields_ = [("run", c_void_p), ("ctx", c_void_p)]


class ShardedOpts(ctypes.Structure):
    _fields_ = [("struct_size", c_size_t), ("shape", c_int), ("compute_on", POINTER(c_int)),
                ("compute", POINTER(Compute)), ("combine", c_void_p), ("combine_ctx", c_void_p)]


class ShapeInfo(ctypes.Structure):
    _fields_ = [
        ("struct_size", c_size_t),
        ("shape", c_int),
        ("reduce_possible", c_int),
        ("gather_busiest_bytes", c_ulonglong),
        ("reduce_busiest_bytes", c_ulonglong),
        ("gather_bytes_sent", c_ulonglong),
        ("gather_bytes_recv", c_ulonglong),
        ("reduce_bytes_sent", c_ulonglong),
        ("reduce_bytes_recv", c_ulonglong),
        ("scratch_bytes_needed", c_ulonglong),
        ("scratch_bytes", c_ulonglong),
        ("reduce_messages", c_int),
        ("reduce_recv_messages", c_int),
        ("reduce_fused", c_int),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "struct_size"}
        d["shape"] = SHAPE_NAMES.get(d["shape"], d["shape"])
        return d


class ShardLayout(ctypes.Structure):
    _fields_ = [
        ("nsets", c_int),
        ("host", POINTER(c_int)),
        ("slot", POINTER(c_int)),
        ("max_hosted", c_int),
        ("chunk_size", c_size_t),
        ("slice_bytes", c_size_t),
        ("hosted_data", c_void_p),
        ("hosted_parity", c_void_p),
        ("gathered_data", c_void_p),
        ("gathered_parity", c_void_p),
    ]


class ShardedInfo(ctypes.Structure):
    _fields_ = [
        ("kind", c_int),
        ("world", c_int),
        ("rank", c_int),
        ("nsets", c_int),
        ("missing", c_int),
        ("my_slice_len", c_size_t),
        ("gather_messages", c_int),
        ("return_messages", c_int),
        ("gather_bytes_sent", c_ulonglong),
        ("gather_bytes_recv", c_ulonglong),
        ("return_bytes_sent", c_ulonglong),
        ("return_bytes_recv", c_ulonglong),
        ("local_bytes", c_ulonglong),
        ("compute_bytes", c_ulonglong),
        ("gather_msg_max", c_ulonglong),
        ("gather_msg_min", c_ulonglong),
        ("return_msg_max", c_ulonglong),
        ("return_msg_min", c_ulonglong),
        ("gather_recv_messages", c_int),
        ("return_recv_messages", c_int),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_PP = POINTER(c_void_p)
_IOP = POINTER(StreamIO)
_STP = POINTER(StreamStats)

_SIGNATURES = {
    "redset_hip_rs_create": (c_int, [c_int, c_int, POINTER(c_void_p)]),
    "redset_hip_rs_destroy": (None, [c_void_p]),
    "redset_hip_rs_matrix": (c_int, [c_void_p, POINTER(c_ubyte)]),
    "redset_hip_rs_shape": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int)]),
    "redset_hip_rs_get_encoding_id": (c_int, [c_int, c_int, c_int, c_int]),
    "redset_hip_rs_get_data_id": (c_int, [c_int, c_int, c_int, c_int]),
    "redset_hip_cell_stride": (c_size_t, [c_size_t]),
    "redset_hip_rs_plan_encode": (c_int, [c_void_p, _PP, _PP, c_size_t, c_size_t, POINTER(c_void_p)]),
    "redset_hip_rs_plan_rebuild": (
        c_int,
        [c_void_p, c_int, POINTER(c_int), _PP, _PP, c_size_t, c_size_t, POINTER(c_void_p)],
    ),
    "redset_hip_xor_plan_encode": (c_int, [c_int, _PP, _PP, c_size_t, c_size_t, POINTER(c_void_p)]),
    "redset_hip_xor_plan_rebuild": (c_int, [c_int, c_int, _PP, _PP, c_size_t, c_size_t, POINTER(c_void_p)]),
    "redset_hip_plan_execute": (c_int, [c_void_p, c_void_p]),
    "redset_hip_plan_get_info": (c_int, [c_void_p, POINTER(PlanInfo)]),
    "redset_hip_plan_destroy": (None, [c_void_p]),
    "redset_hip_gf_combine": (c_int, [_PP, c_int, _PP, c_int, POINTER(c_ubyte), c_size_t, c_int, c_void_p]),
    "redset_hip_xor_combine": (c_int, [_PP, c_int, c_void_p, c_size_t, c_int, c_void_p]),
    "redset_hip_rs_decode_matrix": (c_int, [c_void_p, c_int, POINTER(c_int), c_int, POINTER(c_ubyte)]),
    "redset_hip_rs_encode_stream": (c_int, [c_void_p, c_size_t, c_int, c_int, c_size_t, c_int, _IOP, _STP]),
    "redset_hip_rs_rebuild_stream": (
        c_int, [c_void_p, c_int, POINTER(c_int), c_size_t, c_int, c_int, c_size_t, c_int, _IOP, _STP]),
    "redset_hip_xor_encode_stream": (c_int, [c_int, c_size_t, c_int, c_int, c_size_t, c_int, _IOP, _STP]),
    "redset_hip_xor_rebuild_stream": (c_int, [c_int, c_int, c_size_t, c_int, c_int, c_size_t, c_int, _IOP, _STP]),
    "redset_hip_hostio_create": (c_int, [c_int, _PP, _PP, c_size_t, c_int, _IOP, POINTER(c_void_p)]),
    "redset_hip_hostio_destroy": (None, [c_void_p]),
    "redset_hip_release_scratch": (None, []),
    "redset_hip_fileio_create": (
        c_int,
        [c_int, POINTER(c_int), POINTER(c_char_p), POINTER(c_ulonglong), POINTER(c_char_p), POINTER(c_ulonglong),
         c_size_t, POINTER(c_int), _IOP, POINTER(c_void_p)],
    ),
    "redset_hip_fileio_destroy": (None, [c_void_p]),
    "redset_hip_shard_slice_bytes": (c_size_t, [c_size_t, c_int]),
    "redset_hip_rs_sharded_plan": (
        c_int, [c_void_p, c_int, c_int, POINTER(c_int), POINTER(ShardLayout), POINTER(Transport), POINTER(Compute),
                POINTER(c_void_p)]),
    "redset_hip_xor_sharded_plan": (
        c_int, [c_int, c_int, c_int, POINTER(ShardLayout), POINTER(Transport), POINTER(Compute), POINTER(c_void_p)]),
    "redset_hip_rs_sharded_plan_on": (
        c_int, [c_void_p, c_int, c_int, POINTER(c_int), POINTER(ShardLayout), POINTER(c_int), POINTER(Transport),
                POINTER(Compute), POINTER(c_void_p)]),
    "redset_hip_xor_sharded_plan_on": (
        c_int, [c_int, c_int, c_int, POINTER(ShardLayout), POINTER(c_int), POINTER(Transport), POINTER(Compute),
                POINTER(c_void_p)]),
    "redset_hip_sharded_execute": (c_int, [c_void_p, c_void_p]),
    "redset_hip_sharded_execute_phase": (c_int, [c_void_p, c_int, c_void_p]),
    "redset_hip_sharded_get_info": (c_int, [c_void_p, POINTER(ShardedInfo)]),
    "redset_hip_sharded_destroy": (None, [c_void_p]),
    "redset_hip_plan_combine": (c_int, [POINTER(CombineJob), c_int, c_size_t, POINTER(c_void_p)]),
    "redset_hip_rs_sharded_plan_ex": (
        c_int, [c_void_p, c_int, c_int, POINTER(c_int), POINTER(ShardLayout), POINTER(Transport), POINTER(ShardedOpts),
                POINTER(c_void_p)]),
    "redset_hip_xor_sharded_plan_ex": (
        c_int, [c_int, c_int, c_int, POINTER(ShardLayout), POINTER(Transport), POINTER(ShardedOpts),
                POINTER(c_void_p)]),
    "redset_hip_sharded_get_shape": (c_int, [c_void_p, POINTER(ShapeInfo), c_size_t]),
    "redset_hip_abi_version": (c_int, []),
    "redset_hip_rccl_available": (c_int, []),
    "redset_hip_rccl_unique_id": (c_int, [POINTER(c_ubyte)]),
    "redset_hip_rccl_transport_create": (c_int, [POINTER(c_ubyte), c_int, c_int, POINTER(Transport), POINTER(c_void_p)]),
    "redset_hip_rccl_transport_destroy": (None, [c_void_p]),
    "redset_hip_ring_faults": (c_int, [POINTER(c_uint), c_int]),
    "redset_hip_hang_faults": (c_int, [c_void_p, POINTER(c_uint), c_int]),
    "redset_hip_test_build": (c_int, []),
    "redset_hip_last_error": (c_char_p, []),
    "redset_hip_record_error": (c_int, [c_char_p]),
    "redset_hip_version": (c_char_p, []),
}

_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and return the codec library; raise if it is unavailable."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    lib = open_library(path)
    if path == LIB_PATH:
        _lib = lib
    return lib


def open_library(path: str) -> ctypes.CDLL:
    """Open the library at ``path`` and bind its signatures (no caching)."""
    if not os.path.exists(path):
        raise RedsetHipUnavailable(
            f"HIP codec library not built: {path} is missing "
            "(run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C redset_amd/csrc`)"
        )
    try:
        lib = ctypes.CDLL(path)
    except OSError as exc:  # pragma: no cover - depends on the box
        raise RedsetHipUnavailable(f"cannot load {path}: {exc}") from exc
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    got = lib.redset_hip_abi_version()
    if got != ABI_VERSION:
        # the struct layouts bound above belong to another header revision:
        # fail loudly instead of reading or writing past a struct
        raise RedsetHipUnavailable(f"{path} has ABI version {got}, this binding expects {ABI_VERSION} "
                                   "(rebuild: make -C redset_amd/csrc)")
    return lib


def check(rc: int, what: str) -> None:
    if rc != REDSET_SUCCESS:
        msg = load().redset_hip_last_error().decode(errors="replace")
        raise RedsetHipError(f"{what} failed: {msg}")


def ptr_array(ptrs) -> ctypes.Array:
    """Host array of device pointers (ints) for the C ABI."""
    arr = (c_void_p * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = int(p)
    return arr
