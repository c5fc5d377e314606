"""Randomised parity of the C ABI's host maps against the oracle (CPU): for
random set shapes (p, e) and erasure patterns, the decode map of every stripe
(redset_hip_rs_decode_matrix, what the GPU rebuild applies) reproduces the
oracle's reduce_decode + Gaussian solve (src/redset_reedsolomon_common.c:
855-899, :570-630), and the encoding maps reproduce the oracle's encode."""
import numpy as np
import pytest

import np_ref

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402


@pytest.fixture(scope="module")
def rd():
    import redset_amd

    return redset_amd


def _apply(D, cells):
    out = np.zeros((D.shape[0], cells.shape[1]), np.uint8)
    for i in range(D.shape[0]):
        for s in range(D.shape[1]):
            if D[i, s]:
                out[i] ^= np_ref.MUL[D[i, s], cells[s]]
    return out


@st.composite
def shapes(draw):
    p = draw(st.integers(2, 40))
    e = draw(st.integers(1, min(p - 1, 8)))
    m = draw(st.integers(1, e))
    lost = sorted(draw(st.lists(st.integers(0, p - 1), min_size=m, max_size=m, unique=True)))
    seed = draw(st.integers(0, 2 ** 31))
    return p, e, lost, seed


@settings(max_examples=60, deadline=None)
@given(shapes())
def test_decode_maps_match_oracle_rebuild(rd, oracle, shape):
    p, e, lost, seed = shape
    chunk = 7
    codec = rd.RSCodec(p, e)
    ost = oracle.OracleRS(p, e)
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=seed)
    ost.encode_set(lofi, parity, chunk)
    lf = [x.copy() for x in lofi]
    pr = [x.copy() for x in parity]
    for r in lost:
        lf[r][:] = 0
        pr[r][:] = 0
    wl = [x.copy() for x in lf]
    wp = [x.copy() for x in pr]
    assert ost.rebuild_set(lost, wl, wp, chunk) == 0

    def cell(L, P, s, c):
        enc = codec.encoding_id(s, c)
        if enc < p:
            k = codec.data_id(s, c)
            return L[s][k * chunk:(k + 1) * chunk]
        return P[s][(enc - p) * chunk:(enc - p + 1) * chunk]

    for c in range(p):
        D = codec.decode_matrix(lost, c)
        assert not D[:, lost].any()
        got = _apply(D, np.stack([cell(lf, pr, s, c) for s in range(p)]))
        for i, r in enumerate(lost):
            assert np.array_equal(got[i], cell(wl, wp, r, c)), (p, e, lost, c, r)
            assert np.array_equal(got[i], cell(lofi, parity, r, c))  # and it is the original
