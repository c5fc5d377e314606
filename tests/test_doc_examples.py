"""The reference's own worked Reed-Solomon examples, p = 4 processes, k = 2
checksums (doc/rst/schemes.rst:449-500 encode, :650-693 rebuild), checked
against the oracle, the C ABI's host maps and (``-m gpu``) the HIP plans.

The expected bytes in tests/golden/doc_p4_e2_*.npz come from the doc's
formulas and the chunk placement drawn in doc/rst/fig/rs_encode.png alone
(tests/golden/make_doc_examples.py evaluates them with its own GF(2^8)
multiply), so these tests pin what the matrix known-answer test cannot: which
segment of which process lands in which row of chunks, which coefficient each
sender gets, and which equations the rebuild selects.
"""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


ENC = _load("doc_p4_e2_encode.npz")
REB = _load("doc_p4_e2_rebuild.npz")
P, E, C = int(ENC["ranks"]), int(ENC["encoding"]), int(ENC["chunk"])


FIG = [[str(x) for x in row] for row in ENC["figure_columns"]]  # fig/rs_encode.png a)


def doc_row_of_segment(s, j):
    """Row of chunks holding segment j of process s in the figure."""
    return FIG[s].index(f"{s}:{j}")


def doc_checksum_holder(row, i):
    """Process storing checksum c_i of a row in the figure (process 0 holds
    c0 of the first row and c1 of the second, schemes.rst:449; process 1 c0
    of the second, :656)."""
    return next(s for s in range(P) if FIG[s][row] == f"C{i}")


def _sets():
    lofi = [ENC["lofi"][r].copy() for r in range(P)]
    parity = [np.zeros(E * C, np.uint8) for _ in range(P)]
    return lofi, parity


# --------------------------------------------------------------------------
# host side: oracle and C-ABI maps
# --------------------------------------------------------------------------

def test_layout_maps_follow_the_documented_ring(oracle):
    st = oracle.OracleRS(P, E)
    for s in range(P):
        for j in range(P - E):
            row = doc_row_of_segment(s, j)
            assert st.encoding_id(s, row) == s, (s, j)  # a data contributor of that row
            assert st.data_id(s, row) == j, (s, j)
    for row in range(P):
        for i in range(E):
            assert st.encoding_id(doc_checksum_holder(row, i), row) == P + i


def test_codec_layout_maps_follow_the_documented_ring(hiplib_cpu):
    c = hiplib_cpu.RSCodec(P, E)
    for s in range(P):
        for j in range(P - E):
            assert c.data_id(s, doc_row_of_segment(s, j)) == j
    for row in range(P):
        for i in range(E):
            assert c.encoding_id(doc_checksum_holder(row, i), row) == P + i


def test_oracle_encode_matches_process0_example(oracle):
    lofi, parity = _sets()
    oracle.OracleRS(P, E).encode_set(lofi, parity, C)
    assert np.array_equal(parity[0], ENC["process0_parity"])


def test_oracle_rebuild_matches_documented_solution(oracle):
    st = oracle.OracleRS(P, E)
    lofi, parity = _sets()
    st.encode_set(lofi, parity, C)
    # the doc's knowns for the second row: d3 = seg(3, 0), c1 on process 0
    assert np.array_equal(lofi[3][:C], REB["d3"])
    assert np.array_equal(parity[0][C:2 * C], REB["c1"])
    lost = [int(x) for x in REB["lost"]]
    for r in lost:
        lofi[r][:] = 0
        parity[r][:] = 0
    assert st.rebuild_set(lost, lofi, parity, C) == 0
    assert np.array_equal(lofi[2][C:2 * C], REB["d2"])   # d2 = seg(2, 1)
    assert np.array_equal(parity[1][:C], REB["c0"])      # process 1's c0 of row 1


def test_identify_rows_selects_the_documented_system(oracle):
    """redset_reedsolomon_decode lists the unknowns of row 1 by lost rank
    (src/redset_reedsolomon.c:607-611): process 1 -> c0 (id p+0), process 2 ->
    d2 (id 2). identify_rows (src/redset_reedsolomon_common.c:425-564) must
    pick both checksum rows, giving the doc's A with its columns in that
    order (the doc writes x = (d2, c0))."""
    st = oracle.OracleRS(P, E)
    unknowns = [P + 0, 2]
    assert [st.encoding_id(r, int(REB["row"])) for r in REB["lost"]] == unknowns
    m, rows = st.identify_rows(unknowns)
    assert sorted(rows) == [0, 1]
    A = REB["A"]
    assert np.array_equal(m[np.argsort(rows)], A[:, [1, 0]])


def test_codec_decode_map_matches_documented_solution(hiplib_cpu):
    """The C ABI's decode map for row 1 reads only the doc's knowns (d3 on
    process 3, c1 on process 0) with the coefficients of the doc's solution."""
    c = hiplib_cpu.RSCodec(P, E)
    D = c.decode_matrix([int(x) for x in REB["lost"]], int(REB["row"]))
    M = REB["map_known_d3_c1"]  # rows (d2, c0), columns (d3, c1)
    # rows of D: lost ranks ascending -> process 1 (c0), process 2 (d2)
    want = np.zeros((2, P), np.uint8)
    want[0, 3], want[0, 0] = M[1]
    want[1, 3], want[1, 0] = M[0]
    assert np.array_equal(D, want)


@pytest.fixture(scope="module")
def hiplib_cpu():
    import redset_amd
    from redset_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build_library()
    return redset_amd


# --------------------------------------------------------------------------
# device: the HIP plans on the documented set
# --------------------------------------------------------------------------

@pytest.mark.gpu
def test_gpu_encode_and_rebuild_match_documented_examples():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import redset_amd as rd

    for padded in (True, False):
        if padded:
            lay = rd.SetLayout.allocate(P, P - E, E, C)
        else:
            lay = rd.SetLayout(P, P - E, E, C, C, torch.empty(P * P * C, dtype=torch.uint8, device="cuda"))
        lay.storage.fill_(0x5A)
        for r in range(P):
            for s in range(P - E):
                lay.data_cell(r, s).copy_(torch.from_numpy(ENC["lofi"][r][s * C:(s + 1) * C].copy()))
        codec = rd.RSCodec(P, E)
        codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), C, lay.cell_stride).execute()
        torch.cuda.synchronize()
        got = np.concatenate([lay.parity_cell(0, i).cpu().numpy() for i in range(E)])
        assert np.array_equal(got, ENC["process0_parity"]), padded
        lost = [int(x) for x in REB["lost"]]
        for r in lost:
            lay.lofi(r).fill_(0xEE)
            lay.parity(r).fill_(0xEE)
        codec.plan_rebuild(lost, lay.lofi_ptrs(), lay.parity_ptrs(), C, lay.cell_stride).execute()
        torch.cuda.synchronize()
        assert np.array_equal(lay.data_cell(2, 1).cpu().numpy(), REB["d2"]), padded
        assert np.array_equal(lay.parity_cell(1, 0).cpu().numpy(), REB["c0"]), padded
        for r in range(P):
            assert np.array_equal(lay.lofi(r).cpu().numpy().reshape(P - E, -1)[:, :C].reshape(-1),
                                  ENC["lofi"][r]), (padded, r)


# --------------------------------------------------------------------------
# XOR: doc/rst/fig/xor.png (4 processes, PAD at row r of process r, XOR:c on
# process c)
# --------------------------------------------------------------------------

XOR = _load("doc_xor_p4.npz")
XC = int(XOR["chunk"])


def test_xor_figure_layout_is_the_reference_rule():
    """The figure's columns follow src/redset_xor.c:251-266: process t's
    chunk in row c is segment c for c < t and c - 1 for c > t."""
    fig = [[str(x) for x in row] for row in XOR["figure_columns"]]
    for t in range(4):
        for c in range(4):
            want = "PAD" if c == t else f"{t}:{c if c < t else c - 1}"
            assert fig[t][c] == want


def test_oracle_xor_encode_and_rebuild_match_figure(oracle):
    lofi = [XOR["lofi"][r].copy() for r in range(4)]
    xorc = [np.zeros(XC, np.uint8) for _ in range(4)]
    oracle.xor_encode_set(4, lofi, xorc, XC)
    for r in range(4):
        assert np.array_equal(xorc[r], XOR["xor_of_process"][r]), r
    for root in range(4):
        lf = [x.copy() for x in lofi]
        xc = [x.copy() for x in xorc]
        lf[root][:] = 0
        xc[root][:] = 0
        oracle.xor_rebuild_set(4, root, lf, xc, XC)
        assert np.array_equal(lf[root], XOR["lofi"][root]) and np.array_equal(xc[root], XOR["xor_of_process"][root])


@pytest.mark.gpu
def test_gpu_xor_encode_and_rebuild_match_figure():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import redset_amd as rd

    lay = rd.SetLayout.allocate(4, 3, 1, XC)
    lay.storage.fill_(0x5A)
    for r in range(4):
        for s in range(3):
            lay.data_cell(r, s).copy_(torch.from_numpy(XOR["lofi"][r][s * XC:(s + 1) * XC].copy()))
    rd.xor_plan_encode(4, lay.lofi_ptrs(), lay.parity_ptrs(), XC, lay.cell_stride).execute()
    torch.cuda.synchronize()
    for r in range(4):
        assert np.array_equal(lay.parity_cell(r, 0).cpu().numpy(), XOR["xor_of_process"][r]), r
    for root in range(4):
        lay.lofi(root).fill_(0xEE)
        lay.parity(root).fill_(0xEE)
        rd.xor_plan_rebuild(4, root, lay.lofi_ptrs(), lay.parity_ptrs(), XC, lay.cell_stride).execute()
        torch.cuda.synchronize()
        got = np.concatenate([lay.data_cell(root, s).cpu().numpy() for s in range(3)])
        assert np.array_equal(got, XOR["lofi"][root]), root
        assert np.array_equal(lay.parity_cell(root, 0).cpu().numpy(), XOR["xor_of_process"][root]), root
