"""The sharded plan's C ABI on CPU (no GPU, no process group): argument
checks, the slice width, and a world-1 plan whose transport and compute are
Python callbacks over host memory (the compute is the oracle), so the C
planner's placement and layout arithmetic are checked in-process."""
import ctypes
from ctypes import c_int, c_void_p

import numpy as np
import pytest


@pytest.fixture(scope="module")
def L():
    from redset_amd import _lib

    return _lib


def _layout(_lib, nsets, p, e, chunk, world, host, slot, mh, bufs):
    W = int(_lib.load().redset_hip_shard_slice_bytes(chunk, world))
    nm = nsets * p
    h = (c_int * nm)(*host)
    s = (c_int * nm)(*slot)
    lay = _lib.ShardLayout(nsets, h, s, mh, chunk, W, *[b.ctypes.data for b in bufs])
    return lay, W, (h, s)


def _plan(_lib, rs, kind, lost, lay, tr, comp=None):
    arr = (c_int * max(1, len(lost)))(*lost)
    out = c_void_p()
    rc = _lib.load().redset_hip_rs_sharded_plan(rs, kind, len(lost), arr, ctypes.byref(lay), ctypes.byref(tr),
                                                ctypes.byref(comp) if comp is not None else None, ctypes.byref(out))
    return rc, out


def test_slice_bytes(L):
    f = L.load().redset_hip_shard_slice_bytes
    assert f(64 << 20, 8) == 8 << 20
    assert f(1, 2) == 256
    assert f(1000, 3) == 512
    assert f(0, 4) == 0


def test_plan_argument_checks(L):
    lib = L.load()
    rs = c_void_p()
    assert lib.redset_hip_rs_create(6, 2, ctypes.byref(rs)) == 0
    p, e, chunk, world = 6, 2, 1000, 2
    mh = 6
    W = int(lib.redset_hip_shard_slice_bytes(chunk, world))
    bufs = [np.zeros(world * mh * (p - e) * W, np.uint8), np.zeros(world * mh * e * W, np.uint8)] * 2
    fn = L.EXCHANGE_FN(lambda ctx, x, n, s: 0)
    tr = L.Transport(world, 0, ctypes.cast(fn, c_void_p), None)
    cfn = L.COMPUTE_FN(lambda *a: 0)  # a compute callback: no HIP plan, no device needed
    comp = L.Compute(ctypes.cast(cfn, c_void_p), None)
    host = [m % world for m in range(2 * p)]
    slot = [m // world for m in range(2 * p)]
    lay, _, keep = _layout(L, 2, p, e, chunk, world, host, slot, mh, bufs)
    rc, h = _plan(L, rs, L.PLAN_RS_REBUILD, [1, 4], lay, tr, comp)
    assert rc == 0
    lib.redset_hip_sharded_destroy(h)
    for lost, msg in [([0, 1, 2], b"cannot rebuild"), ([3, 1], b"ascending"), ([6], b"ascending")]:
        rc, _ = _plan(L, rs, L.PLAN_RS_REBUILD, lost, lay, tr, comp)
        assert rc == 1 and msg in lib.redset_hip_last_error(), lost
    rc, _ = _plan(L, rs, L.PLAN_XOR_ENCODE, [], lay, tr, comp)
    assert rc == 1 and b"not RS" in lib.redset_hip_last_error()
    dup = list(slot)
    dup[1] = dup[3]  # members 1 and 3 both on process 1 at slot 1
    lay2, _, keep2 = _layout(L, 2, p, e, chunk, world, host, dup, mh, bufs)
    rc, _ = _plan(L, rs, L.PLAN_RS_ENCODE, [], lay2, tr, comp)
    assert rc == 1 and b"twice" in lib.redset_hip_last_error()
    bad = list(host)
    bad[0] = world
    lay3, _, keep3 = _layout(L, 2, p, e, chunk, world, bad, slot, mh, bufs)
    rc, _ = _plan(L, rs, L.PLAN_RS_ENCODE, [], lay3, tr, comp)
    assert rc == 1 and b"invalid" in lib.redset_hip_last_error()
    lay.slice_bytes = 256  # 2 x 256 < 1000
    rc, _ = _plan(L, rs, L.PLAN_RS_ENCODE, [], lay, tr, comp)
    assert rc == 1 and b"too small" in lib.redset_hip_last_error()
    lib.redset_hip_rs_destroy(rs)


@pytest.mark.parametrize("p,e,chunk,lost", [(11, 3, 3001, [1, 2]), (5, 2, 64, [0, 4]), (4, 1, 1, [3])])
def test_world1_plan_with_callbacks_matches_oracle(L, oracle, p, e, chunk, lost):
    """world 1, two sets on one process in slot order 1,0 (not member order):
    every exchange is a local copy; the compute callback runs the oracle on
    the gathered slices; hosted parity and rebuilt cells equal the oracle's."""
    lib = L.load()
    d, world, nsets = p - e, 1, 2
    mh = nsets * p
    W = int(lib.redset_hip_shard_slice_bytes(chunk, world))
    HD, HP = np.zeros((world, mh, d, W), np.uint8), np.zeros((world, mh, e, W), np.uint8)
    GD, GP = np.zeros_like(HD), np.zeros_like(HP)
    host = [0] * (nsets * p)
    slot = [(nsets * p - 1 - m) for m in range(nsets * p)]  # reversed placement
    rng = np.random.default_rng(p * chunk)
    lofi = [[rng.integers(0, 256, d * chunk, dtype=np.uint8) for _ in range(p)] for _ in range(nsets)]
    for k in range(nsets):
        for r in range(p):
            HD[0, slot[k * p + r], :, :chunk] = lofi[k][r].reshape(d, chunk)
    lay, W, keep = _layout(L, nsets, p, e, chunk, world, host, slot, mh, [HD, HP, GD, GP])
    spans = [(a.ctypes.data, a) for a in (HD, HP, GD, GP)]

    def view(addr, n):
        for base, a in spans:
            if base <= addr < base + a.nbytes:
                return a.reshape(-1)[addr - base: addr - base + n]
        raise AssertionError("address outside the buffers")

    def exchange(ctx, x, n, stream):
        i = 0
        while i < n:
            assert x[i].peer == 0 and x[i].send and not x[i + 1].send
            view(x[i + 1].buf, x[i + 1].len)[:] = view(x[i].buf, x[i].len)
            i += 2
        return 0

    st = oracle.OracleRS(p, e)

    def compute(ctx, kind, missing, ranks, lf, pr, n, stride, stream):
        lv = [view(lf[r], d * stride).reshape(d, stride) for r in range(p)]
        pv = [view(pr[r], e * stride).reshape(e, stride) for r in range(p)]
        a = [np.ascontiguousarray(v[:, :n]).reshape(-1) for v in lv]
        b = [np.ascontiguousarray(v[:, :n]).reshape(-1) for v in pv]
        if kind == L.PLAN_RS_ENCODE:
            st.encode_set(a, b, n)
        else:
            assert st.rebuild_set([ranks[i] for i in range(missing)], a, b, n) == 0
        for v, x in zip(lv, a):
            v[:, :n] = x.reshape(d, n)
        for v, x in zip(pv, b):
            v[:, :n] = x.reshape(e, n)
        return 0

    efn, cfn = L.EXCHANGE_FN(exchange), L.COMPUTE_FN(compute)
    tr = L.Transport(1, 0, ctypes.cast(efn, c_void_p), None)
    comp = L.Compute(ctypes.cast(cfn, c_void_p), None)
    rs = c_void_p()
    assert lib.redset_hip_rs_create(p, e, ctypes.byref(rs)) == 0
    rc, enc = _plan(L, rs, L.PLAN_RS_ENCODE, [], lay, tr, comp)
    assert rc == 0, lib.redset_hip_last_error()
    rc, reb = _plan(L, rs, L.PLAN_RS_REBUILD, lost, lay, tr, comp)
    assert rc == 0, lib.redset_hip_last_error()
    assert lib.redset_hip_sharded_execute(enc, None) == 0, lib.redset_hip_last_error()
    want = []
    for k in range(nsets):
        par = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
        st.encode_set(lofi[k], par, chunk)
        want.append(par)
        for r in range(p):
            assert np.array_equal(HP[0, slot[k * p + r], :, :chunk].reshape(-1), par[r]), (k, r)
    info = L.ShardedInfo()
    assert lib.redset_hip_sharded_get_info(reb, ctypes.byref(info)) == 0
    assert info.gather_bytes_sent == 0 and info.gather_messages == 0 and info.local_bytes == 0
    for k in range(nsets):
        for r in lost:
            HD[0, slot[k * p + r]] = 0xEE
            HP[0, slot[k * p + r]] = 0xEE
    GD[:] = 0xA5
    GP[:] = 0x5A
    assert lib.redset_hip_sharded_execute(reb, None) == 0, lib.redset_hip_last_error()
    for k in range(nsets):
        for r in range(p):
            assert np.array_equal(HD[0, slot[k * p + r], :, :chunk].reshape(-1), lofi[k][r]), (k, r)
            assert np.array_equal(HP[0, slot[k * p + r], :, :chunk].reshape(-1), want[k][r]), (k, r)
    lib.redset_hip_sharded_destroy(enc)
    lib.redset_hip_sharded_destroy(reb)
    lib.redset_hip_rs_destroy(rs)
