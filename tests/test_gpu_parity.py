"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle,
bit-exact, plus size-independent properties at BASELINE.json's full sizes."""
import itertools

import numpy as np
import pytest

import np_ref
from conftest import FALLBACK_RUN

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def rd():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import redset_amd

    redset_amd.load()
    return redset_amd


def upload_set(rd, lofi, parity, data_cells, parity_cells, chunk, padded=True):
    p = len(lofi)
    if padded:
        lay = rd.SetLayout.allocate(p, data_cells, parity_cells, chunk)
    else:  # cells packed back to back: unaligned whenever chunk % 16 != 0
        lay = rd.SetLayout(p, data_cells, parity_cells, chunk, chunk,
                           torch.empty(p * (data_cells + parity_cells) * chunk, dtype=torch.uint8, device="cuda"))
    for r in range(p):
        for s in range(data_cells):
            lay.data_cell(r, s).copy_(torch.from_numpy(lofi[r][s * chunk:(s + 1) * chunk]))
        for i in range(parity_cells):
            lay.parity_cell(r, i).copy_(torch.from_numpy(parity[r][i * chunk:(i + 1) * chunk]))
    torch.cuda.synchronize()
    return lay


def download_set(lay):
    lofi, parity = [], []
    for r in range(lay.ranks):
        lofi.append(np.concatenate([lay.data_cell(r, s).cpu().numpy() for s in range(lay.data_cells)]))
        parity.append(np.concatenate([lay.parity_cell(r, i).cpu().numpy() for i in range(lay.parity_cells)]))
    return lofi, parity


def gpu_bytes(arr: np.ndarray, offset=0):
    """device copy of arr starting `offset` bytes into a fresh allocation"""
    buf = torch.empty(arr.size + offset + 64, dtype=torch.uint8, device="cuda")
    view = buf[offset: offset + arr.size]
    view.copy_(torch.from_numpy(arr))
    return buf, view


# --------------------------------------------------------------------------
# stripe primitives
# --------------------------------------------------------------------------

@pytest.mark.parametrize("nin,nout", [(1, 1), (2, 3), (8, 3), (8, 4), (16, 4), (13, 2), (5, 1),
                                      (17, 1), (40, 6), (3, 9), (100, 5)])  # wider: split passes
@pytest.mark.parametrize("nbytes", [1, 15, 16, 17, 4096 + 7, (1 << 20) + 3])
def test_gf_combine_matches_numpy(rd, nin, nout, nbytes):
    rng = np.random.default_rng(nin * 100 + nout + nbytes)
    ins = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(nin)]
    coef = rng.integers(0, 256, (nout, nin), dtype=np.uint8)
    coef[0, 0] = 0  # zero coefficient
    if nin > 1:
        coef[-1, 1] = 1  # identity coefficient
    want = np.zeros((nout, nbytes), np.uint8)
    for j in range(nout):
        for i in range(nin):
            want[j] ^= np_ref.MUL[coef[j, i], ins[i]]
    d_in = [gpu_bytes(x)[1] for x in ins]
    d_out = [torch.zeros(nbytes, dtype=torch.uint8, device="cuda") for _ in range(nout)]
    rd.gf_combine(d_in, d_out, coef, nbytes)
    torch.cuda.synchronize()
    for j in range(nout):
        assert np.array_equal(d_out[j].cpu().numpy(), want[j]), j
    # accumulate: out ^= same sum -> zeros
    rd.gf_combine(d_in, d_out, coef, nbytes, accumulate=True)
    torch.cuda.synchronize()
    for j in range(nout):
        assert not d_out[j].any().item()


@pytest.mark.parametrize("offset", [1, 3, 8])
def test_gf_combine_unaligned(rd, offset):
    nbytes = 100_003
    rng = np.random.default_rng(offset)
    ins = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(4)]
    coef = rng.integers(1, 256, (3, 4), dtype=np.uint8)
    want = np.zeros((3, nbytes), np.uint8)
    for j in range(3):
        for i in range(4):
            want[j] ^= np_ref.MUL[coef[j, i], ins[i]]
    d_in = [gpu_bytes(x, offset)[1] for x in ins]
    outs = [gpu_bytes(np.zeros(nbytes, np.uint8), offset) for _ in range(3)]
    rd.gf_combine(d_in, [o[1] for o in outs], coef, nbytes)
    torch.cuda.synchronize()
    for j in range(3):
        assert np.array_equal(outs[j][1].cpu().numpy(), want[j])


@pytest.mark.parametrize("nin", [1, 2, 7, 16, 33])
@pytest.mark.parametrize("nbytes,offset", [(33, 0), (1 << 20, 0), (5592406, 0), (4099, 5)])
def test_xor_combine(rd, nin, nbytes, offset):
    rng = np.random.default_rng(nin + nbytes)
    ins = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(nin)]
    want = np.bitwise_xor.reduce(np.stack(ins), axis=0)
    d_in = [gpu_bytes(x, offset)[1] for x in ins]
    out = gpu_bytes(np.zeros(nbytes, np.uint8), offset)
    rd.xor_combine(d_in, out[1], nbytes)
    torch.cuda.synchronize()
    assert np.array_equal(out[1].cpu().numpy(), want)
    rd.xor_combine(d_in, out[1], nbytes, accumulate=True)
    torch.cuda.synchronize()
    assert not out[1].any().item()


# --------------------------------------------------------------------------
# whole-set RS / XOR against the oracle
# --------------------------------------------------------------------------

RS_CASES = [
    (4, 2, 4096),
    (11, 3, 65536),       # config 3 shape, small chunk
    (11, 3, 100_001),     # odd chunk: vector body + byte tail
    (20, 4, 32768),       # config 5 shape (d = 16)
    (8, 1, 20000),
    (12, 6, 8192),        # e > 4: two output groups
    (24, 4, 8192),        # d = 20 > 16: accumulate pass
    (2, 1, 1000),
    (16, 4, 1),           # smallest chunk redset makes (src/redset_reedsolomon.c:491-493)
]


@pytest.mark.parametrize("p,e,chunk", RS_CASES)
@pytest.mark.parametrize("padded", [True, False])
def test_rs_encode_set(rd, oracle, p, e, chunk, padded):
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=p * 1000 + e + chunk)
    lay = upload_set(rd, lofi, parity, p - e, e, chunk, padded=padded)
    codec = rd.RSCodec(p, e)
    plan = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    plan.execute()
    torch.cuda.synchronize()
    oracle.OracleRS(p, e).encode_set(lofi, parity, chunk)
    _, got = download_set(lay)
    for r in range(p):
        assert np.array_equal(got[r], parity[r]), f"member {r}"
    # each output group of <= 4 parity cells reads the stripe's inputs once;
    # stripes wider than 16 inputs take accumulate passes (read+write again)
    if p - e <= 16:
        assert plan.bytes_read == p * (p - e) * chunk * (-(-e // 4))
        assert plan.bytes_written == p * e * chunk


def _rebuild_case(rd, oracle, p, e, chunk, patterns, padded=True):
    st = oracle.OracleRS(p, e)
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=p + 7 * e + chunk)
    st.encode_set(lofi, parity, chunk)
    codec = rd.RSCodec(p, e)
    lay = upload_set(rd, lofi, parity, p - e, e, chunk, padded=padded)
    for lost in patterns:
        for r in lost:  # erase (the rebuild must not read these)
            lay.lofi(r).fill_(0xEE)
            lay.parity(r).fill_(0xEE)
        plan = codec.plan_rebuild(list(lost), lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
        plan.execute()
        torch.cuda.synchronize()
        # oracle: reference decode order on erased copies
        lf = [x.copy() for x in lofi]
        pr = [x.copy() for x in parity]
        for r in lost:
            lf[r][:] = 0
            pr[r][:] = 0
        assert st.rebuild_set(lost, lf, pr, chunk) == 0
        gl, gp = download_set(lay)
        for r in range(p):
            assert np.array_equal(gl[r], lf[r]), (lost, r)
            assert np.array_equal(gp[r], pr[r]), (lost, r)
            # and the oracle reproduces the original
            assert np.array_equal(lf[r], lofi[r]) and np.array_equal(pr[r], parity[r])


@pytest.mark.parametrize("p,e", [(4, 2), (6, 3)])
def test_rs_rebuild_every_pattern(rd, oracle, p, e):
    pats = [c for m in range(1, e + 1) for c in itertools.combinations(range(p), m)]
    _rebuild_case(rd, oracle, p, e, 4096 + 5, pats)


@pytest.mark.parametrize("p,e,chunk,n", [(11, 3, 65536, 40), (20, 4, 16384, 12), (12, 6, 4096, 8),
                                         (24, 4, 4096, 6)])
def test_rs_rebuild_sampled_patterns(rd, oracle, p, e, chunk, n):
    rng = np.random.default_rng(p * e)
    pats = [(1, 2)] + [tuple(sorted(rng.choice(p, size=int(rng.integers(1, e + 1)), replace=False).tolist()))
                       for _ in range(n)]
    _rebuild_case(rd, oracle, p, e, chunk, pats)


@pytest.mark.parametrize("p,e,chunk,lost", [(200, 56, 272, (0, 7, 55, 56, 100, 199)),
                                             (252, 4, 1027, (3, 4, 5, 251)),
                                             (128, 127, 48, tuple(range(1, 128)))])
def test_rs_largest_fields(rd, oracle, p, e, chunk, lost):
    """p + e up to 256, the GF(2^8) limit (src/redset_reedsolomon.c:174-185):
    d up to 248 inputs (16-input accumulate passes) and e up to 127 outputs
    (4-output groups); rebuild with as many erasures as some patterns allow."""
    if p + e > 256:
        pytest.skip("beyond the field")
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=p + e)
    lay = upload_set(rd, lofi, parity, p - e, e, chunk)
    codec = rd.RSCodec(p, e)
    codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).execute()
    torch.cuda.synchronize()
    oracle.OracleRS(p, e).encode_set(lofi, parity, chunk)
    _, got = download_set(lay)
    for r in range(p):
        assert np.array_equal(got[r], parity[r]), r
    _rebuild_case(rd, oracle, p, e, chunk, [tuple(lost[: min(len(lost), e)])])


def test_rs_rebuild_unpadded_odd_chunk(rd, oracle):
    _rebuild_case(rd, oracle, 11, 3, 5592406 // 64, [(0, 10), (3,), (2, 5, 7)], padded=False)


def test_rs_rebuild_too_many_fails(rd):
    codec = rd.RSCodec(6, 2)
    lay = rd.SetLayout.allocate(6, 4, 2, 1024)
    with pytest.raises(rd.RedsetHipError):
        codec.plan_rebuild([0, 1, 2], lay.lofi_ptrs(), lay.parity_ptrs(), 1024, lay.cell_stride)


@pytest.mark.parametrize("p,chunk,padded", [(4, 5592406, False), (4, 5592406, True), (8, 1 << 20, True),
                                            (20, 10007, True), (2, 77, False)])
def test_xor_encode_and_rebuild(rd, oracle, p, chunk, padded):
    lofi, xorc = oracle.random_set(p, p - 1, 1, chunk, seed=p * chunk)
    lay = upload_set(rd, lofi, xorc, p - 1, 1, chunk, padded=padded)
    plan = rd.xor_plan_encode(p, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    plan.execute()
    torch.cuda.synchronize()
    oracle.xor_encode_set(p, lofi, xorc, chunk)
    _, got = download_set(lay)
    for r in range(p):
        assert np.array_equal(got[r], xorc[r])
    for root in sorted({0, p - 1, p // 2}):
        lay.lofi(root).fill_(0x11)
        lay.parity(root).fill_(0x22)
        reb = rd.xor_plan_rebuild(p, root, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
        reb.execute()
        torch.cuda.synchronize()
        gl, gp = download_set(lay)
        assert np.array_equal(gl[root], lofi[root]) and np.array_equal(gp[root], xorc[root])


@pytest.mark.parametrize("mode,group,n_rs,n_xor", [("0", "1", 1, 1), ("1", "1", 11, 8), ("1", "3", 4, 3),
                                                   ("2", "1", 1, 1), ("3", "2", 6, 4), ("3", "0", 1, 1),
                                                   ("3", "1", 11, 8), ("4", "0", 1, 1), ("4", "3", 4, 3)])
@pytest.mark.knobs
def test_plan_job_order(rd, oracle, monkeypatch, mode, group, n_rs, n_xor):
    """A plan runs its stripes side by side in one launch (REDSET_HIP_SEQUENTIAL=0),
    one launch per stripe (=1, the default for cells >= 24 MiB but RS(8+3)'s; or
    per REDSET_HIP_STRIPES_PER_LAUNCH stripes), one launch whose blocks sweep the
    stripes in turn (=2), `group` stripes per launch streamed through one
    continuous ring (=3; REDSET_HIP_STREAM_JOBS, 0 = all) or the same with the
    items claimed at run time (=4, RS(8+3)'s default, all stripes in one
    launch, RS or XOR): same bytes."""
    monkeypatch.setenv("REDSET_HIP_SEQUENTIAL", mode)
    monkeypatch.setenv("REDSET_HIP_STRIPES_PER_LAUNCH", group)
    monkeypatch.setenv("REDSET_HIP_STREAM_JOBS", group)
    p, e, chunk, lost = 11, 3, 40_000, [0, 5, 9]
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=41)
    lay = upload_set(rd, lofi, parity, p - e, e, chunk)
    codec = rd.RSCodec(p, e)
    enc = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    assert enc.launches == n_rs
    enc.execute()
    torch.cuda.synchronize()
    oracle.OracleRS(p, e).encode_set(lofi, parity, chunk)
    _, got = download_set(lay)
    assert all(np.array_equal(a, b) for a, b in zip(got, parity))
    for r in lost:
        lay.lofi(r).fill_(0xEE)
        lay.parity(r).fill_(0xEE)
    reb = codec.plan_rebuild(lost, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    assert reb.launches == n_rs
    reb.execute()
    torch.cuda.synchronize()
    gl, gp = download_set(lay)
    assert all(np.array_equal(a, b) for a, b in zip(gl, lofi))
    assert all(np.array_equal(a, b) for a, b in zip(gp, parity))
    xl, xc = oracle.random_set(8, 7, 1, chunk, seed=42)
    xlay = upload_set(rd, xl, xc, 7, 1, chunk)
    xenc = rd.xor_plan_encode(8, xlay.lofi_ptrs(), xlay.parity_ptrs(), chunk, xlay.cell_stride)
    assert xenc.launches == n_xor
    xenc.execute()
    torch.cuda.synchronize()
    oracle.xor_encode_set(8, xl, xc, chunk)
    _, xgot = download_set(xlay)
    assert all(np.array_equal(a, b) for a, b in zip(xgot, xc))


@pytest.mark.parametrize("mode", ["2", "0", "1", "3", "4"])
@pytest.mark.knobs
def test_ring_jobs_back_to_back(rd, oracle, monkeypatch, mode):
    """The kernels' loader-wave ring is reused job after job inside one launch
    (REDSET_HIP_SEQUENTIAL=2: every block loops over the stripes) and launch
    after launch: repeated RS and XOR plans over small and ragged cells must
    stay bit-exact with no capped handshake poll (a loader that reset the next
    job's flags while consumers still polled the last one's hit the cap in
    round 2, profiles/r02s62_gpu_tests_ring_fault.log)."""
    monkeypatch.setenv("REDSET_HIP_SEQUENTIAL", mode)
    for chunk in (1_000, 65_536 + 48, 300_016):
        p, e = 11, 3
        lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=chunk)
        lay = upload_set(rd, lofi, parity, p - e, e, chunk)
        codec = rd.RSCodec(p, e)
        enc = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
        xl, xc = oracle.random_set(8, 7, 1, chunk, seed=chunk + 1)
        xlay = upload_set(rd, xl, xc, 7, 1, chunk)
        xenc = rd.xor_plan_encode(8, xlay.lofi_ptrs(), xlay.parity_ptrs(), chunk, xlay.cell_stride)
        for _ in range(20):
            enc.execute()
            xenc.execute()
        torch.cuda.synchronize()
        faults = rd.ring_faults()
        if not FALLBACK_RUN:
            assert faults == 0
        oracle.OracleRS(p, e).encode_set(lofi, parity, chunk)
        oracle.xor_encode_set(8, xl, xc, chunk)
        _, got = download_set(lay)
        _, xgot = download_set(xlay)
        assert all(np.array_equal(a, b) for a, b in zip(got, parity))
        assert all(np.array_equal(a, b) for a, b in zip(xgot, xc))


def _window_set(cells_of, p, ncell, chunk, lo, hi):
    """[lo, hi) of every cell of every member, cells back to back (what the
    oracle's set functions take, with chunk_size = hi - lo)"""
    return [np.concatenate([cells_of(r, s)[lo:hi].cpu().numpy() for s in range(ncell)]) for r in range(p)]


@pytest.mark.knobs
@pytest.mark.parametrize("chunk", [(4 << 20) + 5 * 1024 + 48, (4 << 20) + 7 * 1024])
def test_claimed_order_ragged_rows(rd, oracle, monkeypatch, chunk):
    """The claimed order (REDSET_HIP_SEQUENTIAL=4, RS(8+3)'s default encode
    for cells >= 24 MiB) at a size the fast suite can afford: >= 256 blocks,
    so the grid is a multiple of 8 and every XCD's queue is used, and a row
    count (4102 / 4103 rows of 1 KiB, the first with a 48-byte last row) that
    nq * batch = 32 does not divide, so queues end mid-batch and rows past
    the end are skipped. Encode and a 3-member rebuild, both
    claimed, against the oracle."""
    monkeypatch.setenv("REDSET_HIP_SEQUENTIAL", "4")
    p, e, lost = 11, 3, [2, 6, 7]
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=chunk % 1000)
    lay = upload_set(rd, lofi, parity, p - e, e, chunk)
    codec = rd.RSCodec(p, e)
    enc = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    assert enc.launches == 1
    for _ in range(3):  # repeated launches start from zeroed queues
        enc.execute()
    torch.cuda.synchronize()
    oracle.OracleRS(p, e).encode_set(lofi, parity, chunk)
    _, got = download_set(lay)
    assert all(np.array_equal(a, b) for a, b in zip(got, parity))
    for r in lost:
        lay.lofi(r).fill_(0x5A)
        lay.parity(r).fill_(0xA5)
    reb = codec.plan_rebuild(lost, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    assert reb.launches == 1
    reb.execute()
    torch.cuda.synchronize()
    gl, gp = download_set(lay)
    assert all(np.array_equal(a, b) for a, b in zip(gl, lofi))
    assert all(np.array_equal(a, b) for a, b in zip(gp, parity))
    # XOR sets through the same claimed kernel (claimed_sweep without tables)
    xl, xc = oracle.random_set(8, 7, 1, chunk, seed=chunk % 997)
    xlay = upload_set(rd, xl, xc, 7, 1, chunk)
    xenc = rd.xor_plan_encode(8, xlay.lofi_ptrs(), xlay.parity_ptrs(), chunk, xlay.cell_stride)
    assert xenc.launches == 1
    xenc.execute()
    xenc.execute()
    torch.cuda.synchronize()
    oracle.xor_encode_set(8, xl, xc, chunk)
    _, xgot = download_set(xlay)
    assert all(np.array_equal(a, b) for a, b in zip(xgot, xc))
    xlay.lofi(5).fill_(0x33)
    xlay.parity(5).fill_(0x44)
    xreb = rd.xor_plan_rebuild(8, 5, xlay.lofi_ptrs(), xlay.parity_ptrs(), chunk, xlay.cell_stride)
    assert xreb.launches == 1
    xreb.execute()
    torch.cuda.synchronize()
    gl, gp = download_set(xlay)
    assert np.array_equal(gl[5], xl[5]) and np.array_equal(gp[5], xc[5])


def test_claimed_encode_product_ragged_rows(rd, oracle):
    """The product library's own choice at a ragged big size: RS(8+3) with
    24 MiB + 5 KiB + 48 B cells encodes as ONE claimed launch (8 queues,
    24582 rows, not a multiple of 32) and rebuilds in streamed pairs. Cells
    are random on the device; three windows of every cell -- the start, the
    middle, and the ragged end -- are checked against the oracle, and the
    whole set by an encode -> erase -> rebuild round trip."""
    p, e, lost = 11, 3, [1, 4]
    d = p - e
    chunk = (24 << 20) + 5 * 1024 + 48
    lay = rd.SetLayout.allocate(p, d, e, chunk)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    lay.storage.copy_(torch.randint(0, 256, lay.storage.shape, dtype=torch.uint8, device="cuda", generator=g))
    codec = rd.RSCodec(p, e)
    enc = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    assert enc.launches == 1  # claimed: the whole set in one launch
    enc.execute()
    enc.execute()
    torch.cuda.synchronize()
    ref = lay.storage.clone()
    ora = oracle.OracleRS(p, e)
    for lo, hi in [(0, 65536), (chunk // 2 - 4096, chunk // 2 + 4096), (chunk - 70_000, chunk)]:
        wl = _window_set(lay.data_cell, p, d, chunk, lo, hi)
        wp = [np.zeros(e * (hi - lo), np.uint8) for _ in range(p)]
        ora.encode_set(wl, wp, hi - lo)
        got = _window_set(lay.parity_cell, p, e, chunk, lo, hi)
        assert all(np.array_equal(a, b) for a, b in zip(got, wp)), (lo, hi)
    for r in lost:  # the cells only: the pad bytes between them are no one's
        for s in range(d):
            lay.data_cell(r, s).fill_(0)
        for i in range(e):
            lay.parity_cell(r, i).fill_(0)
    reb = codec.plan_rebuild(lost, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    reb.execute()
    torch.cuda.synchronize()
    assert torch.equal(lay.storage, ref)


def test_zero_length_calls_are_noops(rd):
    """Zero-byte stripe primitives and zero-chunk plans succeed without
    touching their outputs (redset never makes a chunk smaller than 1 byte,
    src/redset_reedsolomon.c:491-493, but the ABI accepts 0)."""
    ins = [torch.full((64,), i + 1, dtype=torch.uint8, device="cuda") for i in range(3)]
    outs = [torch.full((64,), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(2)]
    rd.gf_combine(ins, outs, np.ones((2, 3), np.uint8), 0)
    rd.xor_combine(ins, outs[0], 0)
    lay = rd.SetLayout.allocate(6, 4, 2, 256)
    lay.storage.fill_(0xCD)
    codec = rd.RSCodec(6, 2)
    codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), 0, lay.cell_stride).execute()
    codec.plan_rebuild([1, 4], lay.lofi_ptrs(), lay.parity_ptrs(), 0, lay.cell_stride).execute()
    rd.xor_plan_encode(6, lay.lofi_ptrs(), lay.parity_ptrs(), 0, lay.cell_stride).execute()
    torch.cuda.synchronize()
    assert all(bool((o == 0xAB).all()) for o in outs)
    assert bool((lay.storage == 0xCD).all())


def test_plan_replays_in_cuda_graph(rd, oracle):
    p, e, chunk = 11, 3, 1 << 16
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=5)
    lay = upload_set(rd, lofi, parity, p - e, e, chunk)
    plan = rd.RSCodec(p, e).plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        plan.execute(s)  # warm-up outside capture
    torch.cuda.current_stream().wait_stream(s)
    for r in range(p):
        lay.parity(r).zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        plan.execute(torch.cuda.current_stream())
    g.replay()
    torch.cuda.synchronize()
    oracle.OracleRS(p, e).encode_set(lofi, parity, chunk)
    _, got = download_set(lay)
    assert all(np.array_equal(a, b) for a, b in zip(got, parity))


# --------------------------------------------------------------------------
# BASELINE.json full sizes: size-independent properties
# --------------------------------------------------------------------------

def _fill_random(lay, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    for r in range(lay.ranks):
        lay.lofi(r).copy_(torch.randint(0, 256, (lay.lofi(r).numel(),), dtype=torch.uint8, device="cuda",
                                        generator=g))


def _window_check(oracle, lay, p, e, windows, rng):
    """Parity is byte-wise: any byte window of the full-size parity must equal
    the oracle's parity of the same window of the inputs."""
    st = oracle.OracleRS(p, e)
    C = lay.chunk_size
    for _ in range(windows):
        w = int(rng.integers(1, 4096))
        off = int(rng.integers(0, C - w))
        lofi = [np.concatenate([lay.data_cell(r, s)[off:off + w].cpu().numpy() for s in range(p - e)])
                for r in range(p)]
        parity = [np.zeros(e * w, np.uint8) for _ in range(p)]
        st.encode_set(lofi, parity, w)
        for r in range(p):
            got = np.concatenate([lay.parity_cell(r, i)[off:off + w].cpu().numpy() for i in range(e)])
            assert np.array_equal(got, parity[r]), (r, off, w)


@pytest.mark.slow
@pytest.mark.parametrize("p,e,chunk", [(11, 3, 64 << 20), (20, 4, 64 << 20)])
def test_full_size_encode_windows_and_round_trip(rd, oracle, p, e, chunk):
    lay = rd.SetLayout.allocate(p, p - e, e, chunk)
    _fill_random(lay, seed=p * e)
    codec = rd.RSCodec(p, e)
    codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).execute()
    torch.cuda.synchronize()
    _window_check(oracle, lay, p, e, 12, np.random.default_rng(p))
    # checksum of checksums before erasure
    ref = lay.storage.clone()
    lost = [1, 2] if e < 4 else [0, 5, 13, 19]
    for r in lost:
        lay.lofi(r).fill_(0)
        lay.parity(r).fill_(0)
    codec.plan_rebuild(lost, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).execute()
    torch.cuda.synchronize()
    assert torch.equal(lay.storage, ref)


@pytest.mark.slow
def test_full_size_encode_is_linear(rd):
    p, e, chunk = 11, 3, 64 << 20
    codec = rd.RSCodec(p, e)
    A = rd.SetLayout.allocate(p, p - e, e, chunk)
    B = rd.SetLayout.allocate(p, p - e, e, chunk)
    _fill_random(A, 1)
    _fill_random(B, 2)
    for L in (A, B):
        codec.plan_encode(L.lofi_ptrs(), L.parity_ptrs(), chunk, L.cell_stride).execute()
    pa = torch.cat([A.parity(r) for r in range(p)]).clone()
    pb = torch.cat([B.parity(r) for r in range(p)]).clone()
    for r in range(p):
        A.lofi(r).bitwise_xor_(B.lofi(r))
    codec.plan_encode(A.lofi_ptrs(), A.parity_ptrs(), chunk, A.cell_stride).execute()
    torch.cuda.synchronize()
    pab = torch.cat([A.parity(r) for r in range(p)])
    assert torch.equal(pab, pa ^ pb)


@pytest.mark.slow
def test_full_size_xor_c2(rd, oracle):
    p, chunk = 8, 64 << 20
    lay = rd.SetLayout.allocate(p, p - 1, 1, chunk)
    _fill_random(lay, 3)
    rd.xor_plan_encode(p, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).execute()
    torch.cuda.synchronize()
    # XOR of all cells of a stripe (data + parity) is zero, for every stripe
    for c in range(p):
        acc = lay.parity_cell(c, 0).clone()
        for s in range(p):
            if s != c:
                acc ^= lay.data_cell(s, c if c < s else c - 1)
        assert not acc.any().item()
    ref = lay.storage.clone()
    lay.lofi(3).fill_(0)
    lay.parity(3).fill_(0)
    rd.xor_plan_rebuild(p, 3, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).execute()
    torch.cuda.synchronize()
    assert torch.equal(lay.storage, ref)


def test_sharded_runner_world1_hip(rd, oracle):
    """redset_amd.dist at world size 1: the C sharded plan (column-slab
    layout, the process's own slices computed in place, the slab pitch padded
    past the chunk) with the RCCL transport (a one-rank communicator with
    nothing to send), checked against the oracle."""
    from redset_amd.dist import ShardedSetRunner

    p, e, chunk = 11, 3, 300_000
    run = ShardedSetRunner(p, e, chunk, [1, 2], world=1, rank=0, seed=3)
    data = run.D_host.cpu().numpy()
    run.encode()
    torch.cuda.synchronize()
    par = run.P_host.cpu().numpy()
    # hosted index of member r (lost members are hosted last)
    j = [run.host_of(0, r)[1] for r in range(p)]
    lofi = [np.ascontiguousarray(data[0, j[r], :, :chunk]).reshape(-1) for r in range(p)]
    want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    for r in range(p):
        assert np.array_equal(np.ascontiguousarray(par[0, j[r], :, :chunk]).reshape(-1), want[r])
    run.erase()
    run.rebuild()
    torch.cuda.synchronize()
    assert np.array_equal(run.D_host.cpu().numpy()[..., :chunk], data[..., :chunk])
    assert np.array_equal(run.P_host.cpu().numpy()[..., :chunk], par[..., :chunk])


@pytest.mark.parametrize("case", range(12))
def test_random_shapes_encode_rebuild(rd, oracle, case):
    """Seeded random set shapes (p up to 60, e up to 8, odd chunks, packed or
    padded cells): GPU encode and rebuild plans against the oracle."""
    rng = np.random.default_rng(1000 + case)
    p = int(rng.integers(2, 61))
    e = int(rng.integers(1, min(p - 1, 8) + 1))
    chunk = int(rng.integers(1, 5000))
    padded = bool(rng.integers(0, 2))
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=case)
    lay = upload_set(rd, lofi, parity, p - e, e, chunk, padded=padded)
    codec = rd.RSCodec(p, e)
    codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).execute()
    torch.cuda.synchronize()
    st = oracle.OracleRS(p, e)
    st.encode_set(lofi, parity, chunk)
    _, got = download_set(lay)
    for r in range(p):
        assert np.array_equal(got[r], parity[r]), (p, e, chunk, r)
    m = int(rng.integers(1, e + 1))
    lost = sorted(rng.choice(p, size=m, replace=False).tolist())
    for r in lost:
        lay.lofi(r).fill_(0xEE)
        lay.parity(r).fill_(0xEE)
    codec.plan_rebuild(lost, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).execute()
    torch.cuda.synchronize()
    gl, gp = download_set(lay)
    for r in range(p):
        assert np.array_equal(gl[r], lofi[r]) and np.array_equal(gp[r], parity[r]), (p, e, chunk, lost, r)
