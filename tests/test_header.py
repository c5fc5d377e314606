"""Redundancy-file headers (redset_amd/header.py) against the reference's
documented example headers (tests/golden/header_{xor,rs}_doc.txt, made by
tools/make_header_fixtures.py from doc/rst/schemes.rst:262-327 and :520-603).

The trees are built from the examples' inputs (set of 4, member 0's header,
the documented file stats) through the same construction as
redset_apply_rs / redset_apply_xor (src/redset_reedsolomon.c:430-516,
src/redset_xor.c:310-393) and must render to the documented text exactly.
KVTree's on-disk bytes are unpinned (module docstring); the frame round trip
and the set-facts recovery are checked on their own."""
import os

import pytest

from redset_amd import header as H

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _doc(name):
    with open(os.path.join(GOLD, f"header_{name}_doc.txt")) as f:
        return f.read()


def _meta_from_doc(t, member):
    """FileMeta inputs of the documented member (its stat values)."""
    (path, m), = t["DESC"][str(member)]["FILE"]["0"].items()
    g = lambda k: H.get_int(m, k)  # noqa: E731
    return H.FileMeta(path, g("SIZE"), g("MODE"), g("UID"), g("GID"),
                      (g("ATIME_SECS"), g("ATIME_NSECS")), (g("CTIME_SECS"), g("CTIME_NSECS")),
                      (g("MTIME_SECS"), g("MTIME_NSECS")))


def _build(scheme, text, encoding):
    doc = H.parse(text)
    p, me = 4, 0
    members = []
    for r in range(p):
        if str(r) in doc["DESC"]:
            fm = _meta_from_doc(doc, r)
        else:  # not carried by member 0's header: any stats will do
            fm = H.FileMeta(f"./testfile_{r}.out", 1 << 20)
        d = H.Descriptor(scheme, r, p, r, p, encoding=encoding)
        members.append(H.member_hash(d, [fm]))
    max_bytes = max(H.get_int(list(m["FILE"]["0"].values())[0], "SIZE") for m in members)
    chunk = H.chunk_size(scheme, max_bytes, p, encoding)
    return H.header_tree(scheme, me, members, list(range(p)), chunk, encoding)


@pytest.mark.parametrize("scheme,name,k", [("XOR", "xor", 1), ("RS", "rs", 2)])
def test_documented_header(scheme, name, k):
    text = _doc(name)
    assert H.render(_build(scheme, text, k)) == text


def test_documented_chunk_sizes():
    # XOR example: max file 7340032 over 3 segments; RS: over 4 - 2
    assert H.chunk_size("XOR", 7340032, 4) == 2446678
    assert H.chunk_size("RS", 7340032, 4, 2) == 3670016
    assert H.chunk_size("RS", 0, 4, 2) == 1          # 0-byte files, src/redset_reedsolomon.c:490-493
    with pytest.raises(ValueError):
        H.chunk_size("RS", 10, 3, 3)


def test_parse_render_round_trip():
    for name in ("xor", "rs"):
        text = _doc(name)
        assert H.render(H.parse(text)) == text


def test_frame_round_trip(tmp_path):
    t = H.parse(_doc("rs"))
    path = str(tmp_path / "f.redset")
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    n = H.write_header(fd, t)
    os.write(fd, b"\xAB" * 100)
    assert os.lseek(fd, 0, os.SEEK_CUR) == n + 100
    os.close(fd)
    back, size = H.read_header(path)
    assert size == n and back == t
    with pytest.raises(ValueError):
        H.decode(b"XXXXXXXX" + bytes(16))


def test_filenames():
    assert H.redundancy_filename("RS", "ckpt/", 5, 0, 2, 3, 8) == "ckpt/5.rs.grp_1_of_2.mem_4_of_8.redset"
    assert H.redundancy_filename("XOR", "", 0, 1, 2, 0, 4) == "0.xor.grp_2_of_2.mem_1_of_4.redset"


@pytest.mark.parametrize("scheme,p,k,lost", [("RS", 6, 2, [1, 2]), ("RS", 11, 3, [0, 9, 10]),
                                             ("XOR", 5, 1, [4])])
def test_set_facts_from_survivors(scheme, p, k, lost):
    """Any k lost members' file lists come back from their right neighbours'
    headers (each header carries its k left neighbours,
    src/redset_reedsolomon.c:453-474)."""
    members = []
    for r in range(p):
        files = [H.FileMeta(f"/d/r{r}_f{i}", 1000 * r + i) for i in range(1 + r % 3)]
        members.append(H.member_hash(H.Descriptor(scheme, r, p, 10 + r, 64, encoding=k), files))
    chunk = H.chunk_size(scheme, max(sum(1000 * r + i for i in range(1 + r % 3)) for r in range(p)), p, k)
    heads = [H.decode(H.encode(H.header_tree(scheme, r, members, [10 + i for i in range(p)], chunk, k)))
             for r in range(p) if r not in lost]
    f = H.set_facts(heads)
    assert (f.scheme, f.ranks, f.encoding, f.chunk) == (scheme, p, k, chunk)
    assert f.world_ranks == [10 + i for i in range(p)]
    assert [i for i in range(p) if not f.have_header[i]] == lost
    for r in range(p):
        assert f.files(r) == [(f"/d/r{r}_f{i}", 1000 * r + i) for i in range(1 + r % 3)]
    # one more loss than k neighbours cover: some member's list is gone
    worse = sorted(set(lost) | {(max(lost) + 1) % p} | ({(max(lost) + 2) % p} if scheme == "RS" else set()))
    if len(worse) > k:
        heads2 = [h for h, r in zip(heads, [r for r in range(p) if r not in lost]) if r not in worse]
        with pytest.raises(ValueError):
            H.set_facts(heads2)


def _headers_on_disk(tmp, scheme, p, k):
    """Data files + redundancy files with zero parity (CPU-side checks only)."""
    members, reds = [], []
    for r in range(p):
        path = os.path.join(tmp, f"r{r}.dat")
        with open(path, "wb") as f:
            f.write(bytes([r]) * (100 + r))
        members.append(H.member_hash(H.Descriptor(scheme, r, p, r, p, encoding=k), [H.FileMeta.stat(path)]))
    chunk = H.chunk_size(scheme, 100 + p - 1, p, k)
    for r in range(p):
        red = H.redundancy_filename(scheme, os.path.join(tmp, "ck."), r, 0, 1, r, p)
        fd = os.open(red, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        H.write_header(fd, H.header_tree(scheme, r, members, list(range(p)), chunk, k))
        os.write(fd, bytes(k * chunk))  # parity-sized payload (contents unused here)
        os.close(fd)
        reds.append(red)
    return reds


def test_rebuild_set_detection_without_gpu(tmp_path):
    """rebuild_set's set discovery and loss accounting run before any device
    work: nothing lost is a no-op, more lost than k is refused
    (src/redset_reedsolomon_serial.c:476-519)."""
    from redset_amd import setfiles

    tmp = str(tmp_path)
    reds = _headers_on_disk(tmp, "RS", 6, 2)
    out = setfiles.rebuild_set(reds)
    assert out["missing"] == [] and out["chunk"] == H.chunk_size("RS", 105, 6, 2)
    assert out["redundancy"] == reds
    os.unlink(reds[1])
    os.unlink(os.path.join(tmp, "r3.dat"))
    os.unlink(os.path.join(tmp, "r4.dat"))
    with pytest.raises(ValueError, match="tolerates 2"):
        setfiles.rebuild_set(reds)


TOOL = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "redset_amd", "bin",
                    "redset_hip_rebuild")


@pytest.mark.skipif(not os.path.exists(TOOL), reason="redset_hip_rebuild not built")
def test_rebuild_tool_headers_mode_without_gpu(tmp_path):
    """The C tool's headers mode (header_tree.c) learns the same set from the
    same headers: no-op when nothing is lost, refusal past k."""
    import json
    import subprocess

    tmp = str(tmp_path)
    reds = _headers_on_disk(tmp, "XOR", 5, 1)
    res = subprocess.run([TOOL, "headers", *reds], capture_output=True, text=True, timeout=60)
    assert res.returncode == 0, res.stderr
    out = json.loads(res.stdout)
    assert (out["scheme"], out["ranks"], out["encoding"], out["missing"]) == ("xor", 5, 1, [])
    os.unlink(reds[0])
    os.unlink(os.path.join(tmp, "r2.dat"))
    res = subprocess.run([TOOL, "headers", *reds], capture_output=True, text=True, timeout=60)
    assert res.returncode == 1 and "tolerates 1" in res.stderr


def test_unrepresentable_file_names():
    d = H.Descriptor("RS", 0, 4, 0, 4, encoding=2)
    for bad in ("a = b", "x\ny", " lead", ""):
        with pytest.raises(ValueError):
            H.member_hash(d, [H.FileMeta(bad, 1)])
    t = H.member_hash(d, [H.FileMeta("/dir with space/f.dat", 7)])
    assert H.parse(H.render(t)) == t


@pytest.mark.skipif(not os.path.exists(TOOL), reason="redset_hip_rebuild not built")
@pytest.mark.parametrize("name", ["xor", "rs"])
def test_c_header_reader_renders_documented_header(tmp_path, name):
    """header_tree.c parses the framed header and renders the reference's
    documented text byte for byte (the C twin of test_documented_header)."""
    import subprocess

    text = _doc(name)
    path = str(tmp_path / "h.redset")
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    H.write_header(fd, H.parse(text))
    os.close(fd)
    res = subprocess.run([TOOL, "print-header", path], capture_output=True, text=True, timeout=60)
    assert res.returncode == 0, res.stderr
    assert res.stdout == text


def test_corrupt_headers_count_as_lost(tmp_path):
    """A redundancy file whose header cannot be read is a lost member, in
    the Python rebuild and in the C tool alike (src/redset_reedsolomon_serial.c:370-382)."""
    import subprocess

    from redset_amd import setfiles

    tmp = str(tmp_path)
    reds = _headers_on_disk(tmp, "XOR", 5, 1)
    for r in (1, 3):
        with open(reds[r], "r+b") as f:
            f.write(b"garbage!")
    with pytest.raises(ValueError, match="tolerates 1"):
        setfiles.rebuild_set(reds)
    if os.path.exists(TOOL):
        res = subprocess.run([TOOL, "headers", *reds], capture_output=True, text=True, timeout=60)
        assert res.returncode == 1 and "2 members missing" in res.stderr, res.stderr


@pytest.mark.skipif(not os.path.exists(TOOL), reason="redset_hip_rebuild not built")
def test_c_and_python_agree_on_multi_digit_order(tmp_path):
    """Members 0, 9, 10 of an 11-member set under DESC, GROUP RANK 0..10:
    both renderers sort keys as byte strings ("10" before "9")."""
    import subprocess

    p, k = 11, 3
    members = [H.member_hash(H.Descriptor("RS", r, p, 100 + r, 128, encoding=k),
                             [H.FileMeta(f"/ckpt/rank{r}.dat", 1000 + r)]) for r in range(p)]
    t = H.header_tree("RS", 0, members, [100 + r for r in range(p)], H.chunk_size("RS", 1010, p, k), k)
    text = H.render(t)
    assert text.index("\n  10\n") < text.index("\n  9\n")
    path = str(tmp_path / "h.redset")
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    H.write_header(fd, t)
    os.close(fd)
    res = subprocess.run([TOOL, "print-header", path], capture_output=True, text=True, timeout=60)
    assert res.returncode == 0 and res.stdout == text
