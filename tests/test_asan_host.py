"""AddressSanitizer runs of the library's host code, on CPU (no GPU needed).

tests/asan/Makefile rebuilds the host sources (C planner, transports, codec
host side, offline tool) with clang's ASan -- host only, the kernels' objects
are the regular build's -- and these tests drive them:

* the sharded planner + MPI transport (tests/mpi/sharded_test.c with the
  oracle as compute) under mpirun at world 1-4, leak checking on: plans,
  exchanges and teardown must be free of invalid accesses and leaks;
* the offline tool's header reader (header_tree.c) on intact, truncated and
  bit-flipped redundancy-file headers: it may refuse a header, never read
  out of bounds;
* the drop-in slot's per-rank backends (rank_mpi.c, instrumented, with the
  HIP stand-in tests/mpi/hipstub.c preloaded as in test_mpi_hoststub.py):
  the host ring, the sharded plan over device buffers and over host slabs,
  two calls per process (the second on the cached scratch and slot context),
  encode and rebuild checked against the oracle, leak checking on.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from proc import locked_make, run_group
from redset_amd import header as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_DIR = os.path.join(ROOT, "tests", "asan")
BUILD = os.path.join(ASAN_DIR, "build")
MPIRUN = "/opt/conda/bin/mpirun"
ENV = {**os.environ, "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:exitcode=86"}


@pytest.fixture(scope="module")
def asan_build():
    if not (os.path.exists("/opt/rocm/bin/hipcc") and os.path.exists("/opt/rocm/lib/llvm/bin/clang")):
        pytest.skip("needs hipcc and ROCm's clang")
    if not os.path.exists(os.path.join(ROOT, "redset_amd", "build", "codec_kernels.o")):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "redset_amd", "csrc")], check=True)
    res = locked_make(ASAN_DIR)
    assert res.returncode == 0, res.stdout + res.stderr
    return BUILD


def _clean(res):
    return "AddressSanitizer" not in res.stderr and "LeakSanitizer" not in res.stderr and res.returncode != 86


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="needs MPICH's mpirun")
@pytest.mark.parametrize("np_", [1, 2, 3, 4])
@pytest.mark.parametrize("args", [(11, 3, 3001, 1, 2), (20, 4, 777, 0, 5, 19), (4, 2, 1, 0, 3), (5, 1, 65537, 4),
                                  (6, 2, 4096)])
@pytest.mark.parametrize("idle", ["", "0"])
def test_sharded_planner_asan(asan_build, np_, args, idle):
    """idle "0": process 0 computes no column slice (redset_hip_*_sharded_plan_on)"""
    if idle and np_ == 1:
        pytest.skip("someone must compute")
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", os.path.join(asan_build, "sharded_test")] + \
        [str(a) for a in args]
    res = run_group(cmd, 180, env={**ENV, "SHARDED_TEST_IDLE": idle} if idle else ENV)
    assert _clean(res), res.stderr[-4000:]
    assert res.returncode == 0, res.stdout + res.stderr[-4000:]


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="needs MPICH's mpirun")
@pytest.mark.parametrize("np_", [2, 3, 4])
@pytest.mark.parametrize("args", [(11, 3, 3001, 1, 2), (6, 2, 1, 0, 3), (5, 1, 65537, 4)])
@pytest.mark.parametrize("shape", ["reduce", "auto"])
def test_sharded_partial_sums_asan(asan_build, np_, args, shape):
    """The partial-sum shape's planner (sharded.c ra_build / plan_reduce:
    row allocation for every process, merged messages, combine job lists)
    and its execute, under ASan + LeakSanitizer; a forced plan that does
    not fit must fail cleanly (no leak on the error path)."""
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", os.path.join(asan_build, "sharded_test")] + \
        [str(a) for a in args]
    env = {**ENV, "SHARDED_TEST_SHAPE": shape}
    if args[1] == 1:
        env["SHARDED_TEST_SCHEME"] = "xor"
    res = run_group(cmd, 180, env=env)
    assert _clean(res), res.stderr[-4000:]
    assert res.returncode == 0 or (shape == "reduce" and "do not fit" in res.stderr), res.stdout + res.stderr[-4000:]


def _framed(path, text):
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    H.write_header(fd, H.parse(text))
    os.write(fd, bytes(64))
    os.close(fd)


@pytest.mark.parametrize("name", ["xor", "rs"])
def test_header_reader_asan_on_corrupt_headers(asan_build, tmp_path, name):
    tool = os.path.join(asan_build, "redset_hip_rebuild")
    with open(os.path.join(ROOT, "tests", "golden", f"header_{name}_doc.txt")) as f:
        text = f.read()
    good = str(tmp_path / "good.redset")
    _framed(good, text)
    res = subprocess.run([tool, "print-header", good], capture_output=True, text=True, errors="replace", timeout=60, env=ENV)
    assert _clean(res) and res.returncode == 0 and res.stdout == text, res.stderr[-4000:]
    blob = open(good, "rb").read()
    rng = np.random.default_rng(7 if name == "xor" else 8)
    variants = [blob[:n] for n in (0, 4, 8, 12, 16, 24, len(blob) // 2, len(blob) - 65)]
    for _ in range(24):
        b = bytearray(blob)
        for i in rng.integers(0, len(blob) - 64, size=int(rng.integers(1, 6))):
            b[i] ^= int(rng.integers(1, 256))
        variants.append(bytes(b))
    for k in range(8, 16):  # the frame's length field: huge, zero, off by a few
        b = bytearray(blob)
        b[k] = 0xFF
        variants.append(bytes(b))
    bad = str(tmp_path / "bad.redset")
    for i, v in enumerate(variants):
        with open(bad, "wb") as f:
            f.write(v)
        res = subprocess.run([tool, "print-header", bad], capture_output=True, text=True, errors="replace", timeout=60, env=ENV)
        assert _clean(res), (i, res.stderr[-4000:])
        assert res.returncode in (0, 1), (i, res.returncode, res.stderr[-2000:])


def test_header_set_discovery_asan(asan_build, tmp_path):
    """`headers` mode over a set with intact, missing and corrupt members."""
    tool = os.path.join(asan_build, "redset_hip_rebuild")
    p, k = 6, 2
    members, reds = [], []
    tmp = str(tmp_path)
    for r in range(p):
        path = os.path.join(tmp, f"r{r}.dat")
        with open(path, "wb") as f:
            f.write(bytes([r]) * (100 + r))
        members.append(H.member_hash(H.Descriptor("RS", r, p, r, p, encoding=k), [H.FileMeta.stat(path)]))
    chunk = H.chunk_size("RS", 100 + p - 1, p, k)
    for r in range(p):
        red = H.redundancy_filename("RS", os.path.join(tmp, "ck."), r, 0, 1, r, p)
        fd = os.open(red, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        H.write_header(fd, H.header_tree("RS", r, members, list(range(p)), chunk, k))
        os.write(fd, bytes(k * chunk))
        os.close(fd)
        reds.append(red)
    res = subprocess.run([tool, "headers", *reds], capture_output=True, text=True, errors="replace", timeout=60, env=ENV)
    assert _clean(res) and res.returncode == 0, res.stderr[-4000:]
    with open(reds[2], "r+b") as f:
        f.write(b"garbage!")
    os.unlink(reds[4])
    shutil.copy(reds[0], reds[0] + ".bak")
    with open(reds[0], "r+b") as f:
        f.truncate(20)
    res = subprocess.run([tool, "headers", *reds], capture_output=True, text=True, errors="replace", timeout=60, env=ENV)
    assert _clean(res), res.stderr[-4000:]
    assert res.returncode == 1 and "3 members missing" in res.stderr, res.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="needs MPICH's mpirun")
@pytest.mark.parametrize("exchange", ["host", "sharded-mpi", "sharded-host"])
@pytest.mark.parametrize("scheme,p,e,lost", [("rs", 6, 2, [1, 4]), ("rs", 5, 3, [0, 2, 4]), ("xor", 4, 1, [2])])
def test_slot_backends_asan(asan_build, oracle, tmp_path, exchange, scheme, p, e, lost):
    """rank_mpi.c's host code (the instrumented product build: tests/asan's
    libredset_hip_mpi.so, loaded through rank_test's RUNPATH) under ASan +
    LeakSanitizer, for every exchange of the slot."""
    import test_mpi_hoststub as hs

    if not os.path.exists(hs.MPIRUN):
        pytest.skip("needs MPICH")
    subprocess.run(["make", "-s", "-C", hs.MPI_DIR], check=True, capture_output=True)
    env = {"_DRIVER": os.path.join(asan_build, "rank_test"), "RANK_TEST_EXCHANGE": exchange, "RANK_TEST_REPEAT": "2",
           "ASAN_OPTIONS": "verify_asan_link_order=0:detect_leaks=1:halt_on_error=1:exitcode=86",
           "LSAN_OPTIONS": "suppressions=" + os.path.join(ASAN_DIR, "lsan.supp")}
    enc, reb, _ = hs._round_trip(oracle, str(tmp_path), scheme, p, e, lost, 16384, 300 + p, 120_000, env=env)
    for res in (enc, reb):
        assert f"exchange {exchange}" in res.stdout, res.stdout
