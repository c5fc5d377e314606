"""GPU tests of the host-resident streaming pipeline (pinned staging <-> HBM):
host-memory and file-backed sets against the oracle, and the redset
test_redset.c round trip (write files, encode, delete a member's files,
rebuild, compare CRC32) through the file I/O with logical-file padding."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def rd():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import redset_amd
    from redset_amd import stream

    redset_amd.load()
    return redset_amd, stream


def _host_set(lofi, parity):
    """numpy member arrays -> HostIO-compatible pointer lists (stride = chunk)"""
    return [a.ctypes.data for a in lofi], [a.ctypes.data for a in parity]


@pytest.mark.parametrize("p,e,chunk,slice_bytes", [(11, 3, 100_003, 16384), (20, 4, 65536, 0), (4, 2, 5000, 1024),
                                                     (12, 6, 8192, 4096), (24, 4, 4096, 1024)])
def test_rs_encode_stream_hostio(rd, oracle, p, e, chunk, slice_bytes):
    redset_amd, stream = rd
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=chunk + p)
    lp, pp = _host_set(lofi, parity)
    io = stream.HostIO(p, lp, pp, chunk, keepalive=(lofi, parity))
    codec = redset_amd.RSCodec(p, e)
    st = stream.rs_encode_stream(codec, chunk, io, slice_bytes=slice_bytes, io_threads=4)
    want = [np.zeros_like(x) for x in parity]
    oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    for r in range(p):
        assert np.array_equal(parity[r], want[r]), r
    assert st["bytes_written"] == p * e * chunk
    assert st["units"] >= p


def test_rs_encode_stream_stripe_range(rd, oracle):
    redset_amd, stream = rd
    p, e, chunk = 11, 3, 40000
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=1)
    io = stream.HostIO(p, *_host_set(lofi, parity), chunk, keepalive=(lofi, parity))
    st = stream.rs_encode_stream(redset_amd.RSCodec(p, e), chunk, io, first=3, nstripes=2)
    want = [np.zeros_like(x) for x in parity]
    oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    # only the parity cells of stripes 3 and 4 are written
    for r in range(p):
        for i in range(e):
            c = (r + i) % p
            got = parity[r][i * chunk:(i + 1) * chunk]
            if c in (3, 4):
                assert np.array_equal(got, want[r][i * chunk:(i + 1) * chunk])
            else:
                assert not got.any()
    assert st["bytes_read"] == 2 * (p - e) * chunk


@pytest.mark.parametrize("p,e,lost", [(11, 3, [1, 2]), (11, 3, [0, 5, 10]), (20, 4, [3, 4, 17, 19]), (6, 3, [5])])
def test_rs_rebuild_stream_hostio(rd, oracle, p, e, lost):
    redset_amd, stream = rd
    chunk = 30001
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=p * 7)
    oracle.OracleRS(p, e).encode_set(lofi, parity, chunk)
    ref_l = [x.copy() for x in lofi]
    ref_p = [x.copy() for x in parity]
    for r in lost:
        lofi[r][:] = 0
        parity[r][:] = 0
    io = stream.HostIO(p, *_host_set(lofi, parity), chunk, keepalive=(lofi, parity))
    stream.rs_rebuild_stream(redset_amd.RSCodec(p, e), lost, chunk, io, slice_bytes=8192)
    for r in range(p):
        assert np.array_equal(lofi[r], ref_l[r]) and np.array_equal(parity[r], ref_p[r]), r


def test_xor_stream_hostio(rd, oracle):
    redset_amd, stream = rd
    p, chunk = 8, 70001
    lofi, xorc = oracle.random_set(p, p - 1, 1, chunk, seed=4)
    io = stream.HostIO(p, *_host_set(lofi, xorc), chunk, keepalive=(lofi, xorc))
    stream.xor_encode_stream(p, chunk, io, slice_bytes=16384)
    want = [np.zeros_like(x) for x in xorc]
    oracle.xor_encode_set(p, lofi, want, chunk)
    assert all(np.array_equal(a, b) for a, b in zip(xorc, want))
    ref = lofi[6].copy()
    lofi[6][:] = 0
    xorc[6][:] = 0
    stream.xor_rebuild_stream(p, 6, chunk, io)
    assert np.array_equal(lofi[6], ref) and np.array_equal(xorc[6], want[6])


def _write_member_files(tmp, r, rng, nfiles, maxsize):
    files = []
    for k in range(nfiles):
        size = int(rng.integers(0, maxsize))
        path = os.path.join(tmp, f"rank{r}_file{k}.dat")
        data = rng.integers(0, 256, size, dtype=np.uint8)
        data.tofile(path)
        files.append((path, size))
    return files


def _logical(files, total):
    """redset logical file: concatenation zero-padded to `total` bytes"""
    parts = [np.fromfile(p, dtype=np.uint8) for p, _ in files]
    cat = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    out = np.zeros(total, np.uint8)
    out[:cat.size] = cat
    return out


@pytest.mark.parametrize("scheme", ["rs", "xor"])
def test_file_round_trip_crc(rd, oracle, tmp_path, scheme):
    """test/test_redset.c semantics: each rank writes files, apply, delete a
    rank's files, recover, check CRC32 of every rebuilt file
    (test_redset.c:459-589), here for a whole set in one process."""
    redset_amd, stream = rd
    rng = np.random.default_rng(11)
    p, e = (8, 3) if scheme == "rs" else (4, 1)
    d = p - e
    tmp = str(tmp_path)
    files = [_write_member_files(tmp, r, rng, nfiles=int(rng.integers(1, 4)), maxsize=300_000) for r in range(p)]
    max_bytes = max(sum(s for _, s in f) for f in files)
    chunk = stream.chunk_size_for(max_bytes, d)
    header = [4096 + 13 * r for r in range(p)]  # stands in for the kvtree header
    reds = [os.path.join(tmp, f"rank{r}.{scheme}.redset") for r in range(p)]
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for f in files for path, _ in f}
    io = stream.FileIO(files, reds, header, chunk)
    if scheme == "rs":
        codec = redset_amd.RSCodec(p, e)
        stream.rs_encode_stream(codec, chunk, io, slice_bytes=65536)
    else:
        stream.xor_encode_stream(p, chunk, io, slice_bytes=65536)
    io.close()
    # parity bytes after the header equal the oracle's on the padded logical files
    lofi = [_logical(f, d * chunk) for f in files]
    want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    if scheme == "rs":
        oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    else:
        oracle.xor_encode_set(p, lofi, want, chunk)
    for r in range(p):
        got = np.fromfile(reds[r], dtype=np.uint8)[header[r]:header[r] + e * chunk]
        assert np.array_equal(got, want[r]), r
    # lose members (files and redundancy file), rebuild, check CRC32
    lost = [1, 6] if scheme == "rs" else [2]
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    io = stream.FileIO(files, reds, header, chunk, writable=[r in lost for r in range(p)])
    if scheme == "rs":
        stream.rs_rebuild_stream(codec, lost, chunk, io, slice_bytes=32768)
    else:
        stream.xor_rebuild_stream(p, lost[0], chunk, io, slice_bytes=32768)
    io.close()
    for r in lost:
        for path, size in files[r]:
            assert os.path.getsize(path) == size
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
        got = np.fromfile(reds[r], dtype=np.uint8)[header[r]:header[r] + e * chunk]
        assert np.array_equal(got, want[r]), r


@pytest.mark.parametrize("zero_copy", ["1", pytest.param("0", marks=pytest.mark.knobs)])
@pytest.mark.parametrize("p,e,chunk", [(11, 3, 200_001), (20, 4, 65536)])
def test_stream_direct_dma_pinned(rd, oracle, monkeypatch, p, e, chunk, zero_copy):
    """page-locked host cells: by default the kernel reads and writes them
    over PCIe in place (zero copy); with the test twin library,
    REDSET_HIP_ZERO_COPY=0 runs the staged pipeline with direct DMA of the
    mapped cells instead. Same bytes."""
    monkeypatch.setenv("REDSET_HIP_ZERO_COPY", zero_copy)
    redset_amd, stream = rd
    d = p - e
    lofi_np, parity_np = oracle.random_set(p, d, e, chunk, seed=p * 3)
    per = (d + e) * chunk
    buf = torch.empty(p * per, dtype=torch.uint8, pin_memory=True)
    for r in range(p):
        buf[r * per:r * per + d * chunk].copy_(torch.from_numpy(lofi_np[r]))
    base = buf.data_ptr()
    io = stream.HostIO(p, [base + r * per for r in range(p)], [base + r * per + d * chunk for r in range(p)],
                       chunk, keepalive=(buf,), pinned=True)
    codec = redset_amd.RSCodec(p, e)
    stream.rs_encode_stream(codec, chunk, io, slice_bytes=1 << 16)
    oracle.OracleRS(p, e).encode_set(lofi_np, parity_np, chunk)
    host = buf.numpy()
    for r in range(p):
        assert np.array_equal(host[r * per + d * chunk:(r + 1) * per], parity_np[r]), r
    ref = buf.clone()
    for r in (0, 7):
        buf[r * per:(r + 1) * per].zero_()
    stream.rs_rebuild_stream(codec, [0, 7], chunk, io, slice_bytes=1 << 16)
    assert torch.equal(buf, ref)


@pytest.mark.parametrize("victim", ["data", "parity"])
def test_short_survivor_file_fails_the_rebuild(rd, oracle, tmp_path, victim):
    """A survivor's data file or redundancy file that is shorter than its
    recorded size must fail the rebuild, as a short redset_read_attempt does
    (src/redset_lofi.c:74-77, src/redset_reedsolomon.c:678-681), instead of
    reading as zeros and reporting success with wrong bytes. Zero padding
    applies only past a member's last file."""
    redset_amd, stream = rd
    rng = np.random.default_rng(5)
    p, e = 6, 2
    tmp = str(tmp_path)
    files = [_write_member_files(tmp, r, rng, nfiles=2, maxsize=100_000) for r in range(p)]
    chunk = stream.chunk_size_for(max(sum(s for _, s in f) for f in files), p - e)
    header = [512] * p
    reds = [os.path.join(tmp, f"rank{r}.rs.redset") for r in range(p)]
    codec = redset_amd.RSCodec(p, e)
    io = stream.FileIO(files, reds, header, chunk)
    stream.rs_encode_stream(codec, chunk, io, slice_bytes=16384)
    io.close()
    lost = [1]
    for path, _ in files[1]:
        os.unlink(path)
    os.unlink(reds[1])
    survivor = 3
    if victim == "data":
        path, size = max(files[survivor], key=lambda f: f[1])
        assert size > 10
        os.truncate(path, size // 2)
    else:
        # slot 0 = stripe 3, whose rebuild of member 1's data reads it (row 0)
        os.truncate(reds[survivor], header[survivor] + chunk // 2)
    io = stream.FileIO(files, reds, header, chunk, writable=[r in lost for r in range(p)])
    with pytest.raises(redset_amd.RedsetHipError, match="I/O"):
        stream.rs_rebuild_stream(codec, lost, chunk, io, slice_bytes=16384)
    io.close()


@pytest.mark.slow
def test_config4_full_chunk_stream_windows_and_round_trip(rd, oracle):
    """BASELINE.json configs[4] at its own sizes: RS(16+4), p = 20, 256 MiB
    chunks, host-resident cells streamed through the pinned pipeline
    (redset_hip_rs_encode_stream / _rebuild_stream). Three of the 20 stripes
    run (the pipeline takes a stripe range; every stripe reads a cell of every
    member, so the whole set's layout is addressed): their parity is checked
    against the oracle on random byte windows, then four members' cells of
    those stripes are erased and rebuilt bit for bit. Cells of other stripes
    are never touched (their host pages are never committed)."""
    redset_amd, stream = rd
    p, e, C = 20, 4, 256 << 20
    d = p - e
    stripes = [0, 7, 19]
    lofi = [np.empty(d * C, np.uint8) for _ in range(p)]
    parity = [np.empty(e * C, np.uint8) for _ in range(p)]
    codec = redset_amd.RSCodec(p, e)
    rng = np.random.default_rng(2024)
    cells = {}  # (member, kind, index) -> view of every cell the chosen stripes touch
    for c in stripes:
        for r in range(p):
            enc = codec.encoding_id(r, c)
            if enc < p:
                k = codec.data_id(r, c)
                v = lofi[r][k * C:(k + 1) * C]
                v[:] = np.frombuffer(rng.bytes(C), np.uint8)
                cells[(r, 0, k)] = v
            else:
                v = parity[r][(enc - p) * C:(enc - p + 1) * C]
                v[:] = 0
                cells[(r, 1, enc - p)] = v
    io = stream.HostIO(p, [a.ctypes.data for a in lofi], [a.ctypes.data for a in parity], C,
                       keepalive=(lofi, parity))
    for c in stripes:
        st = stream.rs_encode_stream(codec, C, io, first=c, nstripes=1)
        assert st["bytes_written"] == e * C
    # oracle on byte windows of the chosen stripes (parity is byte-wise)
    orc = oracle.OracleRS(p, e)
    for _ in range(6):
        w = int(rng.integers(1, 4096))
        off = int(rng.integers(0, C - w))
        lw = [np.zeros(d * w, np.uint8) for _ in range(p)]
        pw = [np.zeros(e * w, np.uint8) for _ in range(p)]
        for (r, kind, k), v in cells.items():
            if kind == 0:
                lw[r][k * w:(k + 1) * w] = v[off:off + w]
        orc.encode_set(lw, pw, w)
        for (r, kind, k), v in cells.items():
            if kind == 1:
                assert np.array_equal(v[off:off + w], pw[r][k * w:(k + 1) * w]), (r, k, off, w)
    # lose four members, rebuild the chosen stripes
    lost = [0, 5, 13, 19]
    snap = {key: v.copy() for key, v in cells.items() if key[0] in lost}
    for key in snap:
        cells[key][:] = 0xEE
    for c in stripes:
        stream.rs_rebuild_stream(codec, lost, C, io, first=c, nstripes=1)
    for key, want in snap.items():
        assert np.array_equal(cells[key], want), key


@pytest.mark.parametrize("seed", range(8))
def test_file_stream_random(rd, oracle, tmp_path, seed):
    """Seeded random file sets through the streaming pipeline: scheme, ranks,
    encoding, file lists (empty files included), headers, slice size and I/O
    threads; parity against the oracle, then a rebuild of random members
    compared by CRC32. Runs back to back in one process, so later cases draw
    streams and staging slots from the cache earlier ones filled."""
    redset_amd, stream = rd
    rng = np.random.default_rng(7000 + seed)
    scheme = "xor" if seed % 4 == 3 else "rs"
    p = int(rng.integers(2 if scheme == "xor" else 3, 25))
    e = 1 if scheme == "xor" else int(rng.integers(1, min(p - 1, 6) + 1))
    d = p - e
    tmp = str(tmp_path)
    maxsize = int(rng.choice([1, 5000, 120_000, 400_000]))
    files = [_write_member_files(tmp, r, rng, nfiles=int(rng.integers(0, 4)), maxsize=maxsize) for r in range(p)]
    max_bytes = max([sum(s for _, s in f) for f in files] + [0])
    chunk = stream.chunk_size_for(max_bytes, d)
    header = [int(rng.integers(0, 9000)) for _ in range(p)]
    reds = [os.path.join(tmp, f"rank{r}.{scheme}.redset") for r in range(p)]
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for f in files for path, _ in f}
    slice_bytes = int(rng.choice([0, 256, 4096, 65536]))
    threads = int(rng.integers(1, 9))
    io = stream.FileIO(files, reds, header, chunk)
    codec = redset_amd.RSCodec(p, e) if scheme == "rs" else None
    if scheme == "rs":
        stream.rs_encode_stream(codec, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    else:
        stream.xor_encode_stream(p, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    io.close()
    lofi = [_logical(f, d * chunk) for f in files]
    want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    if scheme == "rs":
        oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    else:
        oracle.xor_encode_set(p, lofi, want, chunk)
    for r in range(p):
        got = np.fromfile(reds[r], dtype=np.uint8)[header[r]:header[r] + e * chunk]
        assert np.array_equal(got, want[r]), (scheme, p, e, chunk, r)
    m = 1 if scheme == "xor" else int(rng.integers(1, e + 1))
    lost = sorted(rng.choice(p, size=m, replace=False).tolist())
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    io = stream.FileIO(files, reds, header, chunk, writable=[r in lost for r in range(p)])
    if scheme == "rs":
        stream.rs_rebuild_stream(codec, lost, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    else:
        stream.xor_rebuild_stream(p, lost[0], chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    io.close()
    for r in lost:
        for path, size in files[r]:
            assert os.path.getsize(path) == size
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
        got = np.fromfile(reds[r], dtype=np.uint8)[header[r]:header[r] + e * chunk]
        assert np.array_equal(got, want[r]), (scheme, p, e, chunk, lost, r)
