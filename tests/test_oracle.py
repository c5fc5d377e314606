"""CPU tests of the oracle: pinned against the reference's known answers and
cross-checked against the independent numpy restatement (tests/np_ref.py)."""
import itertools
import os

import numpy as np
import pytest

import np_ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# The reference's own known-answer test: doc/rst/schemes.rst:381-388 and
# src/redset_reedsolomon_common.c:684-694 (p = 4 ranks, 2 checksums).
DOC_MATRIX_P4_E2 = np.array(
    [[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1], [27, 28, 18, 20], [28, 27, 20, 18]], np.uint32
)


def test_matrix_matches_reference_doc(oracle):
    st = oracle.OracleRS(4, 2)
    assert np.array_equal(st.matrix(), DOC_MATRIX_P4_E2)


def test_gf_tables_are_field(oracle):
    lg, ex, im = oracle.gf_tables()
    # exp/log inverse on the 255 units, generator 2, poly 0x11D, reference
    # conventions exp[255] = 0, log[0] = 0 (src/redset_reedsolomon_common.c:110-117)
    assert ex[255] == 0 and lg[0] == 0 and lg[1] == 0 and ex[0] == 1
    assert sorted(ex[:255].tolist()) == list(range(1, 256))
    for i in range(255):
        assert lg[ex[i]] == i
    assert ex[8] == 0x1D  # 2^8 = x^4 + x^3 + x^2 + 1
    assert np.array_equal(ex[:255], np_ref.EXP[:255])
    st = oracle.OracleRS(4, 2)
    for a in range(1, 256):
        assert st.mult(a, int(im[a])) == 1
    rng = np.random.default_rng(1)
    for a, b in rng.integers(0, 256, size=(500, 2)):
        assert st.mult(int(a), int(b)) == np_ref.MUL[a, b]


@pytest.mark.parametrize("p,e", [(2, 1), (4, 1), (4, 2), (8, 1), (8, 3), (11, 3), (16, 4), (20, 4), (24, 8), (40, 6)])
def test_matrix_matches_numpy(oracle, p, e):
    assert np.array_equal(oracle.OracleRS(p, e).matrix(), np_ref.encoding_matrix(p, e).astype(np.uint32))


@pytest.mark.parametrize("p,e", [(4, 2), (11, 3), (20, 4), (9, 8)])
def test_layout_maps_match_numpy(oracle, p, e):
    st = oracle.OracleRS(p, e)
    for r in range(p):
        for c in range(p):
            assert st.encoding_id(r, c) == np_ref.encoding_id(p, e, r, c)
            if np_ref.encoding_id(p, e, r, c) < p:
                assert st.data_id(r, c) == np_ref.data_id(p, e, r, c)
    # every stripe has exactly e parity holders and each member's d data
    # segments are a permutation of 0..d-1
    d = p - e
    for c in range(p):
        assert sum(np_ref.encoding_id(p, e, r, c) >= p for r in range(p)) == e
    for r in range(p):
        segs = [np_ref.data_id(p, e, r, c) for c in range(p) if np_ref.encoding_id(p, e, r, c) < p]
        assert sorted(segs) == list(range(d))


def test_parity_slot_is_stripe_r_plus_i(oracle):
    # src/redset_reedsolomon.c:347-375: member r's slot i holds stripe (r+i)%p, row p+i
    p, e = 11, 3
    for r in range(p):
        for i in range(e):
            assert np_ref.encoding_id(p, e, r, (r + i) % p) == p + i


@pytest.mark.parametrize("p,e,chunk", [(4, 2, 1000), (11, 3, 777), (20, 4, 256), (5, 1, 333)])
def test_encode_matches_numpy(oracle, p, e, chunk):
    st = oracle.OracleRS(p, e)
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=p * 100 + e)
    st.encode_set(lofi, parity, chunk, slice_bytes=300)
    ref = np_ref.rs_encode_set(p, e, lofi, chunk)
    for r in range(p):
        assert np.array_equal(parity[r], ref[r]), r


def test_slicing_does_not_change_parity(oracle):
    p, e, chunk = 11, 3, 5000
    st = oracle.OracleRS(p, e)
    lofi, par_a = oracle.random_set(p, p - e, e, chunk, seed=7)
    par_b = [x.copy() for x in par_a]
    st.encode_set(lofi, par_a, chunk, slice_bytes=chunk)
    st.encode_set(lofi, par_b, chunk, slice_bytes=129)
    assert all(np.array_equal(a, b) for a, b in zip(par_a, par_b))


@pytest.mark.parametrize("p,e", [(4, 2), (6, 3), (11, 3)])
def test_rebuild_every_pattern(oracle, p, e):
    chunk = 97
    st = oracle.OracleRS(p, e)
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=11)
    st.encode_set(lofi, parity, chunk)
    for m in range(1, e + 1):
        for lost in itertools.combinations(range(p), m):
            lf = [x.copy() for x in lofi]
            pr = [x.copy() for x in parity]
            for r in lost:
                lf[r][:] = 0xA5
                pr[r][:] = 0x5A
            assert st.rebuild_set(lost, lf, pr, chunk, slice_bytes=50) == 0
            for r in range(p):
                assert np.array_equal(lf[r], lofi[r]) and np.array_equal(pr[r], parity[r]), (lost, r)


def test_rebuild_too_many_fails(oracle):
    p, e, chunk = 6, 2, 10
    st = oracle.OracleRS(p, e)
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=3)
    assert st.rebuild_set([0, 1, 2], lofi, parity, chunk) == 1


def test_rebuild_matches_numpy_solver(oracle):
    p, e, chunk = 11, 3, 64
    st = oracle.OracleRS(p, e)
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=5)
    st.encode_set(lofi, parity, chunk)
    lost = [1, 2, 9]
    lf = [x.copy() if r not in lost else np.zeros_like(x) for r, x in enumerate(lofi)]
    pr = [x.copy() if r not in lost else np.zeros_like(x) for r, x in enumerate(parity)]
    nl, npar = np_ref.rs_rebuild_set(p, e, lost, lf, pr, chunk)
    st.rebuild_set(lost, lf, pr, chunk)
    for r in range(p):
        assert np.array_equal(lf[r], nl[r]) and np.array_equal(pr[r], npar[r])


@pytest.mark.parametrize("p,chunk", [(2, 100), (4, 5593), (8, 1024)])
def test_xor_encode_and_rebuild(oracle, p, chunk):
    lofi, xorc = oracle.random_set(p, p - 1, 1, chunk, seed=p)
    oracle.xor_encode_set(p, lofi, xorc, chunk, slice_bytes=1000)
    ref = np_ref.xor_encode_set(p, lofi, chunk)
    for r in range(p):
        assert np.array_equal(xorc[r], ref[r])
    for root in range(p):
        lf = [x.copy() for x in lofi]
        xc = [x.copy() for x in xorc]
        lf[root][:] = 0
        xc[root][:] = 0
        oracle.xor_rebuild_set(p, root, lf, xc, chunk, slice_bytes=777)
        assert np.array_equal(lf[root], lofi[root]) and np.array_equal(xc[root], xorc[root])


def test_pthreads_baseline_matches_serial(oracle):
    p, e, chunk = 11, 3, 3000
    st = oracle.OracleRS(p, e)
    lofi, par_a = oracle.random_set(p, p - e, e, chunk, seed=9)
    par_b = [x.copy() for x in par_a]
    st.encode_set(lofi, par_a, chunk, slice_bytes=1024)
    n = st.encode_pthreads(lofi, par_b, chunk, slice_bytes=1024, nthreads=4)
    assert n == 4
    assert all(np.array_equal(a, b) for a, b in zip(par_a, par_b))
    lx, xa = oracle.random_set(8, 7, 1, chunk, seed=2)
    xb = [x.copy() for x in xa]
    oracle.xor_encode_set(8, lx, xa, chunk)
    oracle.xor_encode_pthreads(8, lx, xb, chunk, nthreads=3)
    assert all(np.array_equal(a, b) for a, b in zip(xa, xb))


def test_crc32_matches_zlib(oracle):
    import zlib

    buf = np.random.default_rng(0).integers(0, 256, 10000, dtype=np.uint8)
    assert oracle.crc32(buf) == zlib.crc32(buf.tobytes())


def _golden_files():
    # doc_*.npz: the documented worked examples, checked by tests/test_doc_examples.py
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz") and not f.startswith("doc_")) \
        if os.path.isdir(GOLDEN) else []


@pytest.mark.parametrize("name", _golden_files())
def test_oracle_reproduces_golden(oracle, name):
    z = np.load(os.path.join(GOLDEN, name))
    kind = str(z["kind"])
    p, e, chunk = int(z["ranks"]), int(z["encoding"]), int(z["chunk"])
    if kind == "matrix":
        assert np.array_equal(oracle.OracleRS(p, e).matrix(), z["matrix"].astype(np.uint32))
        return
    lofi = [np.ascontiguousarray(x) for x in z["lofi"]]
    if kind == "rs":
        st = oracle.OracleRS(p, e)
        parity = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
        st.encode_set(lofi, parity, chunk)
        assert np.array_equal(np.stack(parity), z["parity"])
    elif kind == "xor":
        xorc = [np.zeros(chunk, np.uint8) for _ in range(p)]
        oracle.xor_encode_set(p, lofi, xorc, chunk)
        assert np.array_equal(np.stack(xorc), z["parity"])


@pytest.mark.parametrize("name", ["rs_p11_e3_c64MiB", "xor_p8_c64MiB"])
def test_full_size_inputs_regenerate(name):
    """The full-size digest fixture (tests/golden/full_size_digests.json) is
    usable: member 0's regenerated input hashes as recorded, and the recorded
    case matches tests/full_size.py."""
    import json

    import full_size

    with open(os.path.join(GOLDEN, "full_size_digests.json")) as f:
        want = json.load(f)[name]
    case = full_size.CASES[name]
    assert all(want[k] == v for k, v in case.items())
    assert len(want["parity_sha256"]) == case["ranks"]
    assert full_size.sha256(full_size.member_lofi(case, 0)) == want["lofi_sha256"][0]
