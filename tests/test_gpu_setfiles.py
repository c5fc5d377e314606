"""GPU tests of redundancy sets on disk with headers (redset_amd.setfiles):
apply_set writes every member's redundancy file (header + parity), members
are lost, and rebuild_set learns the set from the surviving headers alone
(src/redset_reedsolomon_serial.c:355-500), rebuilds the lost members' data
files, metadata and redundancy files, and everything must match what was
there before byte for byte (CRC32 as test/test_redset.c:459-589 checks,
plus the whole redundancy files, headers included). The parity bytes after
each header are checked against the CPU oracle."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def sf():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import redset_amd
    from redset_amd import setfiles

    redset_amd.load()
    return setfiles


def _members(tmp, p, sizes, seed):
    rng = np.random.default_rng(seed)
    out = []
    for r in range(p):
        fl = []
        for k, size in enumerate(sizes[r]):
            path = os.path.join(tmp, "data", f"rank{r}_file{k}.dat")
            os.makedirs(os.path.dirname(path), exist_ok=True)
            rng.integers(0, 256, size, dtype=np.uint8).tofile(path)
            os.chmod(path, 0o640 if r % 2 else 0o600)
            os.utime(path, ns=(1_596_610_023_010_398_911 + r, 1_596_610_023_005_398_943 + k))
            fl.append(path)
        out.append(fl)
    return out


def _logical(paths, total):
    parts = [np.fromfile(p, dtype=np.uint8) for p in paths]
    cat = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    out = np.zeros(total, np.uint8)
    out[:cat.size] = cat
    return out


def _snapshot(oracle, paths):
    snap = {}
    for p in paths:
        st = os.stat(p)
        meta = (st.st_mode, st.st_mtime_ns) if not p.endswith(".redset") else ()  # data files get their stats back
        snap[p] = (oracle.crc32(np.fromfile(p, dtype=np.uint8)), st.st_size) + meta
    return snap


@pytest.mark.parametrize("scheme,p,k,lost,sizes", [
    ("XOR", 4, 1, [2], [[1 << 20]] * 4),                 # configs[0]'s shape, 1 MiB files
    ("RS", 6, 2, [0, 4], [[300_000, 77], [1], [250_000], [0, 123_456], [199_999, 5, 60_000], [4096]]),
    ("RS", 11, 3, [1, 2, 9], [[200_003]] * 11),
])
def test_apply_lose_rebuild(sf, oracle, tmp_path, scheme, p, k, lost, sizes):
    from redset_amd import header as H

    tmp = str(tmp_path)
    members = _members(tmp, p, sizes, seed=p * 5 + k)
    res = sf.apply_set(scheme, members, os.path.join(tmp, "ckpt."), encoding=k, slice_bytes=1 << 16)
    reds, chunk = res["redundancy"], res["chunk"]
    assert chunk == H.chunk_size(scheme, max(sum(os.path.getsize(f) for f in fl) for fl in members), p, k)
    d = p - k
    lofi = [_logical(fl, d * chunk) for fl in members]
    want = [np.zeros(k * chunk, np.uint8) for _ in range(p)]
    if scheme == "RS":
        oracle.OracleRS(p, k).encode_set(lofi, want, chunk)
    else:
        oracle.xor_encode_set(p, lofi, want, chunk)
    for r in range(p):
        raw = np.fromfile(reds[r], dtype=np.uint8)
        hs = res["header_bytes"][r]
        assert raw.size == hs + k * chunk
        assert np.array_equal(raw[hs:], want[r]), r
        t, n = H.read_header(reds[r])
        assert n == hs and H.get_int(t, "RANK") == r and H.get_int(t, "CHUNK") == chunk
    allpaths = [f for fl in members for f in fl] + reds
    before = _snapshot(oracle, allpaths)
    # nothing lost: no-op
    assert sf.rebuild_set(reds)["missing"] == []
    for r in lost:
        for f in members[r]:
            os.unlink(f)
        os.unlink(reds[r])
    out = sf.rebuild_set(reds, slice_bytes=1 << 15)
    assert out["missing"] == sorted(lost) and out["ok"], out
    assert _snapshot(oracle, allpaths) == before


def test_truncated_data_file_is_lost(sf, oracle, tmp_path):
    tmp = str(tmp_path)
    members = _members(tmp, 5, [[70_000, 3]] * 5, seed=9)
    reds = sf.apply_set("RS", members, os.path.join(tmp, "c"), encoding=2)["redundancy"]
    allpaths = [f for fl in members for f in fl] + reds
    before = _snapshot(oracle, allpaths)
    with open(members[3][0], "r+b") as f:
        f.truncate(1000)
    out = sf.rebuild_set(reds)
    assert out["missing"] == [3] and out["ok"]
    assert _snapshot(oracle, allpaths) == before


def test_too_many_lost(sf, tmp_path):
    tmp = str(tmp_path)
    members = _members(tmp, 5, [[10_000]] * 5, seed=3)
    reds = sf.apply_set("RS", members, os.path.join(tmp, "c"), encoding=2)["redundancy"]
    os.unlink(members[0][0])
    os.unlink(members[2][0])
    os.unlink(members[4][0])
    with pytest.raises(ValueError, match="tolerates"):
        sf.rebuild_set(reds)


TOOL = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "redset_amd", "bin",
                    "redset_hip_rebuild")


@pytest.mark.parametrize("scheme,p,k,lost", [("RS", 8, 3, [0, 5, 7]), ("RS", 11, 3, [0, 9, 10]), ("XOR", 4, 1, [1])])
def test_rebuild_tool_from_headers(sf, oracle, tmp_path, scheme, p, k, lost):
    """redset_hip_rebuild headers <files>: the C tool reads the set from the
    surviving headers and regenerates the lost members' headers in C; the
    whole redundancy files (headers included) and the data files with their
    stats must come back byte for byte."""
    import json
    import subprocess

    tmp = str(tmp_path)
    sizes = [[150_001 + 17 * r, 3 * r] for r in range(p)]
    members = _members(tmp, p, sizes, seed=p + k)
    reds = sf.apply_set(scheme, members, os.path.join(tmp, "set."), encoding=k)["redundancy"]
    allpaths = [f for fl in members for f in fl] + reds
    before = _snapshot(oracle, allpaths)
    for r in lost:
        for f in members[r]:
            os.unlink(f)
        os.unlink(reds[r])
    res = subprocess.run([TOOL, "headers", *reds], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    out = json.loads(res.stdout)
    assert out["missing"] == sorted(lost) and out["ok"] and out["metadata_ok"], out
    assert _snapshot(oracle, allpaths) == before


@pytest.mark.parametrize("use_tool", [False, True])
def test_rebuild_in_a_strided_group(sf, oracle, tmp_path, use_tool):
    """Set members at parent ranks 3, 7, 11, ... in group 2 of 4: the lost
    members' redundancy file names come back from the GROUP map and the
    descriptors (rs.grp_2_of_4.mem_<r+1>_of_6, src/redset_reedsolomon.c:34-44)."""
    import json
    import subprocess

    tmp = str(tmp_path)
    p, k, lost = 6, 2, [2, 3]
    members = _members(tmp, p, [[40_000 + r] for r in range(p)], seed=21)
    world = [3 + 4 * r for r in range(p)]
    res = sf.apply_set("RS", members, os.path.join(tmp, "g."), encoding=k, world_ranks=world, world_size=32,
                       group_id=1, groups=4)
    reds = res["redundancy"]
    assert os.path.basename(reds[2]) == "g.11.rs.grp_2_of_4.mem_3_of_6.redset"
    allpaths = [f for fl in members for f in fl] + reds
    before = _snapshot(oracle, allpaths)
    for r in lost:
        os.unlink(members[r][0])
        os.unlink(reds[r])
    survivors = [x for i, x in enumerate(reds) if i not in lost]
    if use_tool:
        out = subprocess.run([TOOL, "headers", *survivors], capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stdout + out.stderr
        assert json.loads(out.stdout)["missing"] == lost
    else:
        out = sf.rebuild_set(survivors)
        assert out["missing"] == lost and out["redundancy"] == reds and out["ok"]
    assert _snapshot(oracle, allpaths) == before


@pytest.mark.parametrize("use_tool", [False, True])
def test_truncated_parity_is_lost(sf, oracle, tmp_path, use_tool):
    """A redundancy file cut short after its header is a lost member too."""
    import subprocess

    tmp = str(tmp_path)
    members = _members(tmp, 5, [[30_000]] * 5, seed=13)
    reds = sf.apply_set("RS", members, os.path.join(tmp, "t"), encoding=2)["redundancy"]
    allpaths = [f for fl in members for f in fl] + reds
    before = _snapshot(oracle, allpaths)
    with open(reds[4], "r+b") as f:
        f.truncate(os.path.getsize(reds[4]) - 1)
    if use_tool:
        res = subprocess.run([TOOL, "headers", *reds], capture_output=True, text=True, timeout=300)
        assert res.returncode == 0, res.stdout + res.stderr
    else:
        assert sf.rebuild_set(reds)["missing"] == [4]
    assert _snapshot(oracle, allpaths) == before
