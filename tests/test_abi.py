"""CPU tests of the C-ABI library: it loads, exports every symbol declared in
include/redset_hip.h, and its host-side math (matrix, layout maps, decode
maps, argument checks) agrees with the oracle. No kernel runs here."""
import ctypes
import itertools
import os
import re

import numpy as np
import pytest

import np_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "redset_hip.h")


@pytest.fixture(scope="module")
def hiplib():
    import redset_amd
    from redset_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build_library()
    return redset_amd


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(redset_hip_\w+)\s*\(", text)))


def test_header_declares_what_binding_expects():
    from redset_amd import _lib

    assert declared_symbols() == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(hiplib):
    lib = ctypes.CDLL(hiplib.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert b"gfx950" in hiplib.load().redset_hip_version()


def test_mpi_library_exports_every_declared_symbol(hiplib):
    """include/redset_hip_mpi.h's per-rank backends are exported by
    libredset_hip_mpi.so (built where MPICH is present, as in this image).
    Checked with nm: dlopen would need libmpi on the loader path."""
    import shutil
    import subprocess

    mpi_h = os.path.join(ROOT, "include", "redset_hip_mpi.h")
    mpi_so = os.path.join(ROOT, "redset_amd", "lib", "libredset_hip_mpi.so")
    if not os.path.exists(mpi_so) or not shutil.which("nm"):
        pytest.skip("libredset_hip_mpi.so not built (no MPICH) or nm missing")
    text = re.sub(r"/\*.*?\*/", "", open(mpi_h).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(redset_hip_\w+)\s*\(", text)))
    assert declared == ["redset_hip_mpi_transport_create", "redset_hip_mpi_transport_destroy",
                        "redset_hip_mpi_transport_reserve",
                        "redset_hip_rank_last_exchange", "redset_hip_rank_last_stats",
                        "redset_hip_rank_scratch_release",
                        "redset_hip_rank_set_exchange", "redset_hip_rs_decode_rank", "redset_hip_rs_encode_rank",
                        "redset_hip_xor_decode_rank", "redset_hip_xor_encode_rank"]
    out = subprocess.run(["nm", "-D", "--defined-only", mpi_so], capture_output=True, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    for name in declared:
        assert name in exported, name


def test_missing_library_fails_loudly(tmp_path):
    from redset_amd import _lib

    with pytest.raises(_lib.RedsetHipUnavailable):
        _lib.open_library(str(tmp_path / "nope.so"))


@pytest.mark.parametrize("p,e", [(4, 2), (8, 1), (11, 3), (20, 4), (24, 8), (64, 16)])
def test_matrix_matches_oracle(hiplib, oracle, p, e):
    m = hiplib.RSCodec(p, e).matrix()
    assert np.array_equal(m.astype(np.uint32), oracle.OracleRS(p, e).matrix())


def test_doc_known_answer(hiplib):
    m = hiplib.RSCodec(4, 2).matrix()
    assert m[4:].tolist() == [[27, 28, 18, 20], [28, 27, 20, 18]]


def test_layout_maps(hiplib, oracle):
    for p, e in [(4, 2), (11, 3), (20, 4), (7, 6)]:
        c = hiplib.RSCodec(p, e)
        o = oracle.OracleRS(p, e)
        for r in range(p):
            for k in range(p):
                assert c.encoding_id(r, k) == o.encoding_id(r, k)
                assert c.data_id(r, k) == o.data_id(r, k)


@pytest.mark.parametrize("p,e", [(1, 1), (257, 1), (10, 0), (10, 10), (250, 7)])
def test_invalid_parameters_rejected(hiplib, p, e):
    with pytest.raises(hiplib.RedsetHipError):
        hiplib.RSCodec(p, e)


def _apply(D, cells):
    out = np.zeros((D.shape[0], cells.shape[1]), np.uint8)
    for i in range(D.shape[0]):
        for s in range(D.shape[1]):
            if D[i, s]:
                out[i] ^= np_ref.MUL[D[i, s], cells[s]]
    return out


@pytest.mark.parametrize("p,e", [(4, 2), (6, 3), (11, 3), (20, 4)])
def test_decode_maps_reproduce_oracle_rebuild(hiplib, oracle, p, e):
    """The host decode map (identify_rows + symbolic elimination) applied to
    the surviving cells must equal the oracle's reduce_decode + Gaussian solve
    for every stripe -- this is exactly what the GPU rebuild computes."""
    chunk = 33
    codec = hiplib.RSCodec(p, e)
    st = oracle.OracleRS(p, e)
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=p + e)
    st.encode_set(lofi, parity, chunk)

    def cell(lf, pr, s, c):
        enc = np_ref.encoding_id(p, e, s, c)
        if enc < p:
            k = np_ref.data_id(p, e, s, c)
            return lf[s][k * chunk:(k + 1) * chunk]
        return pr[s][(enc - p) * chunk:(enc - p + 1) * chunk]

    patterns = [pat for m in range(1, e + 1) for pat in itertools.combinations(range(p), m)]
    if len(patterns) > 150:
        rng = np.random.default_rng(0)
        patterns = [patterns[i] for i in rng.choice(len(patterns), 150, replace=False)]
    for lost in patterns:
        lf = [x.copy() for x in lofi]
        pr = [x.copy() for x in parity]
        for r in lost:
            lf[r][:] = 0
            pr[r][:] = 0
        want_l = [x.copy() for x in lf]
        want_p = [x.copy() for x in pr]
        assert st.rebuild_set(lost, want_l, want_p, chunk) == 0
        for c in range(p):
            D = codec.decode_matrix(lost, c)
            assert not D[:, list(lost)].any()
            cells = np.stack([cell(lf, pr, s, c) for s in range(p)])
            got = _apply(D, cells)
            for i, r in enumerate(sorted(lost)):
                assert np.array_equal(got[i], cell(want_l, want_p, r, c)), (lost, c, r)


def test_shape_and_error_recording(hiplib):
    from ctypes import byref, c_int, c_void_p

    from redset_amd import _lib

    L = _lib.load()
    h = c_void_p()
    assert L.redset_hip_rs_create(20, 4, byref(h)) == 0
    p, e = c_int(), c_int()
    assert L.redset_hip_rs_shape(h, byref(p), byref(e)) == 0 and (p.value, e.value) == (20, 4)
    L.redset_hip_rs_destroy(h)
    assert L.redset_hip_record_error(b"per-rank backend: lofi read failed") == 1
    assert L.redset_hip_last_error() == b"per-rank backend: lofi read failed"


def test_bad_arguments_rejected_before_any_device_work(hiplib):
    """Argument checks of the C ABI fail with REDSET_FAILURE and a message
    before touching the device (runs on CPU): erasure lists out of range, not
    ascending, duplicated or longer than the parity count (src/redset_
    reedsolomon.c:1096), and malformed stripe-primitive calls."""
    from ctypes import POINTER, byref, c_int, c_ubyte, c_void_p

    from redset_amd import _lib

    L = _lib.load()
    h = c_void_p()
    assert L.redset_hip_rs_create(11, 3, byref(h)) == 0
    out = (c_ubyte * (4 * 11))()
    for ranks, msg in [([11], b"out of range"), ([-1], b"out of range"), ([2, 1], b"ascending"),
                       ([3, 3], b"ascending"), ([0, 1, 2, 3], b"cannot rebuild")]:
        arr = (c_int * len(ranks))(*ranks)
        assert L.redset_hip_rs_decode_matrix(h, len(ranks), arr, 0, out) == 1, ranks
        assert msg in L.redset_hip_last_error(), (ranks, L.redset_hip_last_error())
    L.redset_hip_rs_destroy(h)
    ptrs = (c_void_p * 2)(16, 32)
    nul = (c_void_p * 2)(16, None)
    coef = (c_ubyte * 4)(1, 2, 3, 4)
    PP = POINTER(c_void_p)
    as_pp = lambda a: ctypes.cast(a, PP)  # noqa: E731
    assert L.redset_hip_gf_combine(as_pp(ptrs), 0, as_pp(ptrs), 1, coef, 64, 0, None) == 1
    assert b"nin=0" in L.redset_hip_last_error()
    assert L.redset_hip_gf_combine(as_pp(ptrs), 257, as_pp(ptrs), 1, coef, 64, 0, None) == 1
    assert L.redset_hip_gf_combine(as_pp(nul), 2, as_pp(ptrs), 1, coef, 64, 0, None) == 1
    assert b"null input 1" in L.redset_hip_last_error()
    assert L.redset_hip_gf_combine(as_pp(ptrs), 2, as_pp(nul), 2, coef, 64, 0, None) == 1
    assert b"null output 1" in L.redset_hip_last_error()
    assert L.redset_hip_gf_combine(None, 2, as_pp(ptrs), 1, coef, 64, 0, None) == 1
    assert L.redset_hip_xor_combine(as_pp(ptrs), 0, 16, 64, 0, None) == 1
    assert L.redset_hip_xor_combine(as_pp(nul), 2, 16, 64, 0, None) == 1
    assert b"null input 1" in L.redset_hip_last_error()
    assert L.redset_hip_xor_combine(as_pp(ptrs), 2, None, 64, 0, None) == 1


def test_cell_stride_recommendation(hiplib):
    """redset_hip_cell_stride: 256-B aligned, >= chunk, and a 16 MiB stagger
    for 16 MiB-multiple cells (the bench's 64 MiB layout)."""
    f = hiplib.cell_stride
    MiB = 1 << 20
    assert f(0) == 256 and f(1) == 256 and f(256) == 256 and f(257) == 512
    assert f(5592406) == 5592576                      # configs[0]'s chunk: aligned, no pad
    assert f(64 * MiB) == 80 * MiB                    # configs[1]-[3]
    assert f(256 * MiB) == 272 * MiB                  # configs[4]
    assert f(16 * MiB) == 32 * MiB and f(16 * MiB + 1) == 16 * MiB + 256
    for c in (1, 4095, 3 * MiB + 7, 48 * MiB):
        assert f(c) >= c and f(c) % 256 == 0
