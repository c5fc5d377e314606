"""Regenerate the golden fixtures in tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

Provenance. The reference (ECP-VeloC/redset) cannot be built or run in this
image (it needs a cmake-generated config.h and the un-vendored KVTree
library; see DESIGN.md "Oracle"), and its tests hold no parity vectors. So:
  * matrix_p4_e2.npz is the reference's own known answer, transcribed from
    doc/rst/schemes.rst:381-388 (= src/redset_reedsolomon_common.c:684-694);
  * every other fixture is produced by the CPU oracle (oracle/redset_oracle.c)
    AFTER it has been checked against that known answer and against the
    independent numpy restatement (tests/np_ref.py). They freeze the oracle's
    behaviour so a later change to it cannot silently move the target.
Inputs come from numpy's PCG64 with the seeds below.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_lib  # noqa: E402
import np_ref  # noqa: E402


def save(name, **kw):
    np.savez_compressed(os.path.join(HERE, name), **kw)
    print("wrote", name)


def main():
    oracle_lib.build()
    doc = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1],
                    [27, 28, 18, 20], [28, 27, 20, 18]], np.uint8)
    save("matrix_p4_e2.npz", kind="matrix", ranks=4, encoding=2, chunk=0, matrix=doc)
    for p, e in [(11, 3), (20, 4), (8, 1)]:
        m = oracle_lib.OracleRS(p, e).matrix().astype(np.uint8)
        assert np.array_equal(m, np_ref.encoding_matrix(p, e))
        save(f"matrix_p{p}_e{e}.npz", kind="matrix", ranks=p, encoding=e, chunk=0, matrix=m)
    for p, e, chunk, seed in [(4, 2, 64, 101), (11, 3, 48, 102), (20, 4, 40, 103)]:
        st = oracle_lib.OracleRS(p, e)
        lofi, parity = oracle_lib.random_set(p, p - e, e, chunk, seed)
        st.encode_set(lofi, parity, chunk)
        ref = np_ref.rs_encode_set(p, e, lofi, chunk)
        assert all(np.array_equal(a, b) for a, b in zip(parity, ref))
        save(f"rs_p{p}_e{e}_c{chunk}.npz", kind="rs", ranks=p, encoding=e, chunk=chunk,
             lofi=np.stack(lofi), parity=np.stack(parity))
    for p, chunk, seed in [(4, 37, 201), (8, 64, 202)]:
        lofi, xorc = oracle_lib.random_set(p, p - 1, 1, chunk, seed)
        oracle_lib.xor_encode_set(p, lofi, xorc, chunk)
        save(f"xor_p{p}_c{chunk}.npz", kind="xor", ranks=p, encoding=1, chunk=chunk,
             lofi=np.stack(lofi), parity=np.stack(xorc))


if __name__ == "__main__":
    main()
