"""Regenerate tests/golden/doc_p4_e2_{encode,rebuild}.npz: the reference's
own worked Reed-Solomon examples, p = 4 processes, k = 2 checksums
(run from the repo root: ``python tests/golden/make_doc_examples.py``).

Provenance: the expected bytes come ONLY from the formulas printed in the
reference's documentation, evaluated with the GF(2^8) arithmetic the same
document defines (bytes, XOR addition, the 0x11D field whose p=4, k=2 matrix
is printed at doc/rst/schemes.rst:381-388). Neither the oracle nor the
product library is used here, so these fixtures pin both of them.

* Placement of chunks, doc/rst/fig/rs_encode.png panel a) (also
  fig/rs_general.png panel d): the column of each process, rows of chunks
  top to bottom, "s:j" = segment j of process s's logical file, C0/C1 its
  checksum chunks -- transcribed as FIGURE_COLUMNS below.
* Encode, doc/rst/schemes.rst:449-500. Process 0 stores c0 of the first row
  of chunks and c1 of the second (:449). Its ring steps (:482-497, and
  rs_encode.png panels b, c): step 1 receives from processes 1 and 2
  (``c0 += 28*d1``, ``c1 += 20*d2``), step 2 from processes 2 and 3
  (``c0 += 18*d2``, ``c1 += 18*d3``), where d_s is process s's chunk in that
  row. With the figure's placement:
      c0 (row 0) = 28 * seg(1, 0) + 18 * seg(2, 0)
      c1 (row 1) = 20 * seg(2, 1) + 18 * seg(3, 0)
* XOR, doc/rst/fig/xor.png (schemes.rst:185-200, "Logically insert alternating
  zero-padded chunk and reduce"; "Scatter XOR chunks among the different
  ranks"): with N = 4 processes each logical file splits into N-1 chunks,
  process r's column has a zero PAD chunk at row r, and XOR:c -- the XOR of
  row c over all processes -- is stored by process c (XOR_FIGURE_COLUMNS).
* Rebuild, doc/rst/schemes.rst:650-693: processes 1 and 2 lost, second row
  of chunks. Unknowns x = (d2, c0), d2 = seg(2, 1), c0 = process 1's first
  checksum chunk; A = [[18, 1], [20, 0]], b = (20*d3, 18*d3 + c1) with
  d3 = seg(3, 0) and c1 = process 0's second checksum chunk. Solved here:
      d2 = (18*d3 + c1) / 20,   c0 = 20*d3 + 18*d2.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CHUNK = 32
SEED = 449
# doc/rst/fig/rs_encode.png a): FIGURE_COLUMNS[process][row of chunks]
FIGURE_COLUMNS = [
    ["C0", "C1", "0:0", "0:1"],
    ["1:0", "C0", "C1", "1:1"],
    ["2:0", "2:1", "C0", "C1"],
    ["C1", "3:0", "3:1", "C0"],
]


# doc/rst/fig/xor.png, middle panel: XOR_FIGURE_COLUMNS[process][row]
XOR_FIGURE_COLUMNS = [
    ["PAD", "0:0", "0:1", "0:2"],
    ["1:0", "PAD", "1:1", "1:2"],
    ["2:0", "2:1", "PAD", "2:2"],
    ["3:0", "3:1", "3:2", "PAD"],
]


def gf_mul(a: int, b: int) -> int:
    """Shift-and-add multiply in GF(2^8) mod x^8+x^4+x^3+x^2+1 (0x11D)."""
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
    return r


def gf_inv(a: int) -> int:
    return next(x for x in range(1, 256) if gf_mul(a, x) == 1)


def mul(c: int, v: np.ndarray) -> np.ndarray:
    return np.array([gf_mul(c, int(x)) for x in v], np.uint8)


def main():
    rng = np.random.default_rng(SEED)
    # logical files of the 4 processes, (p - k) = 2 segments each
    lofi = rng.integers(0, 256, size=(4, 2 * CHUNK), dtype=np.uint8)
    seg = lambda s, j: lofi[s, j * CHUNK:(j + 1) * CHUNK]  # noqa: E731
    cell = lambda s, row: seg(*map(int, FIGURE_COLUMNS[s][row].split(":")))  # noqa: E731
    assert FIGURE_COLUMNS[0][:2] == ["C0", "C1"]  # process 0: c0 of row 0, c1 of row 1
    c0 = mul(28, cell(1, 0)) ^ mul(18, cell(2, 0))
    c1 = mul(20, cell(2, 1)) ^ mul(18, cell(3, 1))
    assert np.array_equal(c0, mul(28, seg(1, 0)) ^ mul(18, seg(2, 0)))
    assert np.array_equal(c1, mul(20, seg(2, 1)) ^ mul(18, seg(3, 0)))
    # the same checksums as the doc's step-by-step accumulation (:489-497)
    acc0 = mul(28, cell(1, 0))
    acc1 = mul(20, cell(2, 1))
    acc0 ^= mul(18, cell(2, 0))
    acc1 ^= mul(18, cell(3, 1))
    assert np.array_equal(acc0, c0) and np.array_equal(acc1, c1)
    np.savez_compressed(os.path.join(HERE, "doc_p4_e2_encode.npz"), ranks=4, encoding=2, chunk=CHUNK,
                        lofi=lofi, process0_parity=np.concatenate([c0, c1]),
                        figure_columns=np.array(FIGURE_COLUMNS))

    # rebuild of the second row with processes 1 and 2 lost
    assert FIGURE_COLUMNS[1][1] == "C0" and FIGURE_COLUMNS[0][1] == "C1"
    d3 = cell(3, 1)
    b0 = mul(20, d3)
    b1 = mul(18, d3) ^ c1
    inv20 = gf_inv(20)
    d2 = mul(inv20, b1)
    c0_row1 = b0 ^ mul(18, d2)
    assert np.array_equal(d2, cell(2, 1))  # the solution is the lost data
    A = np.array([[18, 1], [20, 0]], np.uint8)
    # A x = b holds for x = (d2, c0)
    for i in range(2):
        lhs = mul(int(A[i, 0]), d2) ^ mul(int(A[i, 1]), c0_row1)
        assert np.array_equal(lhs, (b0, b1)[i])
    # the same unknowns as a linear map of the known cells (d3, c1)
    D = np.array([[gf_mul(inv20, 18), inv20],                                   # d2
                  [gf_mul(20, 1) ^ gf_mul(18, gf_mul(inv20, 18)), gf_mul(18, inv20)]],  # c0
                 np.uint8)
    np.savez_compressed(os.path.join(HERE, "doc_p4_e2_rebuild.npz"), ranks=4, encoding=2, chunk=CHUNK,
                        lost=np.array([1, 2]), row=1, A=A, d3=d3, c1=c1, b=np.stack([b0, b1]),
                        d2=d2, c0=c0_row1, map_known_d3_c1=D)
    # XOR set of the figure: 4 processes, 3 chunks each
    xlofi = rng.integers(0, 256, size=(4, 3 * CHUNK), dtype=np.uint8)
    xseg = lambda s, j: xlofi[s, j * CHUNK:(j + 1) * CHUNK]  # noqa: E731
    xor_cells = np.zeros((4, CHUNK), np.uint8)
    for row in range(4):
        for s in range(4):
            label = XOR_FIGURE_COLUMNS[s][row]
            if label != "PAD":
                xor_cells[row] ^= xseg(*map(int, label.split(":")))
    np.savez_compressed(os.path.join(HERE, "doc_xor_p4.npz"), ranks=4, chunk=CHUNK, lofi=xlofi,
                        xor_of_process=xor_cells, figure_columns=np.array(XOR_FIGURE_COLUMNS))
    print("wrote doc_p4_e2_encode.npz, doc_p4_e2_rebuild.npz, doc_xor_p4.npz")


if __name__ == "__main__":
    main()
