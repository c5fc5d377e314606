"""Independent numpy restatement of redset's GF(2^8) codec (test-only).

Written separately from oracle/redset_oracle.c so the two cross-check each
other: tables come from a different construction (repeated doubling of a
vector), the matrix is built by matrix algebra (V * inv(top of V)), and
encode/rebuild use vectorised table lookups. The normalisation of
src/redset_reedsolomon_common.c:634-682 is column elimination, i.e. right
multiplication of the Vandermonde matrix V by inv(V_top); any such
normalisation of a full-rank V gives the same unique matrix with I on top.
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D


def tables():
    exp = np.zeros(512, np.int64)
    log = np.zeros(256, np.int64)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= POLY
    exp[255:510] = exp[:255]
    return exp, log


EXP, LOG = tables()
# full 256x256 product table
_A = np.arange(256)
MUL = np.zeros((256, 256), np.uint8)
MUL[1:, 1:] = EXP[(LOG[1:, None] + LOG[None, 1:]) % 255].astype(np.uint8)


def inv(a: int) -> int:
    return int(EXP[(255 - LOG[a]) % 255])


def mat_mul(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    A = np.asarray(A, np.uint8)
    B = np.asarray(B, np.uint8)
    out = np.zeros((A.shape[0], B.shape[1]), np.uint8)
    for k in range(A.shape[1]):
        out ^= MUL[A[:, k][:, None], B[k, :][None, :]]
    return out


def mat_inv(A: np.ndarray) -> np.ndarray:
    n = A.shape[0]
    M = np.concatenate([np.asarray(A, np.uint8), np.eye(n, dtype=np.uint8)], axis=1)
    for c in range(n):
        r = next(r for r in range(c, n) if M[r, c])
        M[[c, r]] = M[[r, c]]
        M[c] = MUL[inv(int(M[c, c])), M[c]]
        for r2 in range(n):
            if r2 != c and M[r2, c]:
                M[r2] ^= MUL[int(M[r2, c]), M[c]]
    return M[:, n:]


def encoding_matrix(p: int, e: int) -> np.ndarray:
    # V[r, c] = r^c with 0^0 = 1
    V = np.zeros((p + e, p), np.uint8)
    for r in range(p + e):
        acc = 1
        for c in range(p):
            V[r, c] = acc
            acc = int(MUL[acc, r])
    return mat_mul(V, mat_inv(V[:p]))


def encoding_id(p, e, rank, chunk):
    d = p - e
    i = (d - rank + p + chunk) % p
    return rank if i < d else p + (i - d)


def data_id(p, e, rank, chunk):
    i = chunk - e if chunk > rank else chunk
    lead = rank + e - p
    return i - lead if lead > 0 else i


def rs_encode_set(p, e, lofi, chunk):
    """parity[r][i] = sum_s mat[p+i, s] * data cell of s in stripe (r+i)%p."""
    M = encoding_matrix(p, e)
    parity = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    for c in range(p):
        for r in range(p):
            row = encoding_id(p, e, r, c)
            if row < p:
                continue
            acc = np.zeros(chunk, np.uint8)
            for s in range(p):
                if encoding_id(p, e, s, c) < p:
                    seg = data_id(p, e, s, c)
                    acc ^= MUL[M[row, s], lofi[s][seg * chunk:(seg + 1) * chunk]]
            parity[r][(row - p) * chunk:(row - p + 1) * chunk] = acc
    return parity


def rs_rebuild_set(p, e, missing, lofi, parity, chunk):
    """Rebuild erased members by solving each stripe with the MDS property
    (any d = p - e surviving cells determine the stripe's data)."""
    M = encoding_matrix(p, e)
    d = p - e
    lofi = [x.copy() for x in lofi]
    parity = [x.copy() for x in parity]
    erased = set(missing)
    for c in range(p):
        # rows of M (one per member cell) and the member order of the data vector
        data_members = [s for s in range(p) if encoding_id(p, e, s, c) < p]
        surv = [s for s in range(p) if s not in erased][:d]
        G = np.zeros((d, d), np.uint8)
        rhs = np.zeros((d, chunk), np.uint8)
        for k, s in enumerate(surv):
            row = encoding_id(p, e, s, c)
            if row < p:
                seg = data_id(p, e, s, c)
                rhs[k] = lofi[s][seg * chunk:(seg + 1) * chunk]
                G[k, data_members.index(s)] = 1
            else:
                rhs[k] = parity[s][(row - p) * chunk:(row - p + 1) * chunk]
                G[k] = [M[row, t] for t in data_members]
        data = mat_mul(mat_inv(G), rhs)
        for s in erased:
            row = encoding_id(p, e, s, c)
            if row < p:
                seg = data_id(p, e, s, c)
                lofi[s][seg * chunk:(seg + 1) * chunk] = data[data_members.index(s)]
            else:
                coef = np.array([[M[row, t] for t in data_members]], np.uint8)
                parity[s][(row - p) * chunk:(row - p + 1) * chunk] = mat_mul(coef, data)[0]
    return lofi, parity


def xor_encode_set(p, lofi, chunk):
    out = []
    for r in range(p):
        acc = np.zeros(chunk, np.uint8)
        for s in range(p):
            if s != r:
                seg = r if r < s else r - 1
                acc ^= lofi[s][seg * chunk:(seg + 1) * chunk]
        out.append(acc)
    return out
