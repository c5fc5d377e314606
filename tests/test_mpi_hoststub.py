"""The per-rank backends' host code on the CPU (no GPU needed).

libredset_hip_mpi.so's host-MPI path (redset_amd/csrc/rank_mpi.c: file reads,
the ring exchange of redset's per-rank encode/rebuild, the scratch pool, the
per-call stats, the writes) runs here with tests/mpi/hipstub.c preloaded in
place of the HIP runtime and the two combine calls. The stub is test
infrastructure only; the GPU suite (tests/test_gpu_mpi.py) runs the same
driver, tests/mpi/rank_test.c, on the real runtime and kernels. A host-code
regression (a self-recursive MPI wrapper once slipped through, because on a
GPU-less machine the backends stop at hipStreamCreate) fails here first.

Checks as in test_gpu_mpi.py: parity after each rank's header equals the
oracle's on the padded logical files (test/test_redset.c:459-589), rebuilt
files match by CRC32, and a member's I/O error fails every rank without a
hang (src/redset_reedsolomon.c:338-342)."""
import json
import os
import subprocess

import numpy as np
import pytest

from proc import locked_make, run_group
from test_gpu_mpi import _logical, _manifests, _setup

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPI_DIR = os.path.join(ROOT, "tests", "mpi")
# RANK_TEST_BIN: another build of the driver (tests/asan: host ASan)
RANK_TEST = os.environ.get("RANK_TEST_BIN") or os.path.join(MPI_DIR, "build", "rank_test")
STUB = os.path.join(MPI_DIR, "build", "libhipstub.so")
MPIRUN = "/opt/conda/bin/mpirun"


@pytest.fixture(scope="module")
def stub():
    if not os.path.exists(MPIRUN):
        pytest.skip("needs MPICH")
    if not os.path.exists(os.path.join(ROOT, "redset_amd", "lib", "libredset_hip_mpi.so")):
        pytest.skip("libredset_hip_mpi.so not built")
    subprocess.run(["make", "-s", "-C", MPI_DIR], check=True, capture_output=True)
    return STUB


def _run(np_, args, env=None, timeout=120):
    env = {**os.environ, **(env or {})}
    drv = env.pop("_DRIVER", RANK_TEST)
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", "-env", "LD_PRELOAD", STUB, drv] + [str(a) for a in args]
    res = run_group(cmd, timeout, env=env)
    assert "AddressSanitizer" not in res.stderr and "LeakSanitizer" not in res.stderr, res.stderr[-4000:]
    return res


def _stats(stdout, tag="first"):
    for line in stdout.splitlines():
        if line.startswith(f"rank_stats {tag} "):
            return json.loads(line.split(" ", 2)[2])
    raise AssertionError(stdout)


def _round_trip(oracle, tmp, scheme, p, e, lost, buf, seed, maxsize, header=None, env=None):
    d = p - e
    rng = np.random.default_rng(seed)
    files, chunk = _setup(tmp, p, d, rng, maxsize)
    header = header or [int(rng.integers(0, 5000)) for _ in range(p)]
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for fl in files for path, _ in fl}
    res = _run(p, [scheme, "encode", e, tmp, buf], env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    lofi = [_logical(fl, d * chunk) for fl in files]
    want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    if scheme == "rs":
        oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    else:
        oracle.xor_encode_set(p, lofi, want, chunk)
    for r in range(p):
        blob = np.fromfile(reds[r], dtype=np.uint8)
        assert blob.size == header[r] + e * chunk
        assert np.array_equal(blob[header[r]:], want[r]), (scheme, p, e, r)
    enc = res
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    res = _run(p, [scheme, "rebuild", e, tmp, buf] + lost, env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    assert f"rebuild exchange {(env or {}).get('RANK_TEST_EXCHANGE', 'host')}" in res.stdout, res.stdout
    for r in lost:
        for path, size in files[r]:
            assert os.path.getsize(path) == size
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
        blob = np.fromfile(reds[r], dtype=np.uint8)
        assert np.array_equal(blob[header[r]:header[r] + e * chunk], want[r]), r
    return enc, res, chunk


@pytest.mark.parametrize("scheme,p,e,lost,buf", [("rs", 6, 2, [1, 4], 65536), ("rs", 5, 3, [0, 2, 4], 40000),
                                                  ("xor", 4, 1, [2], 50000), ("xor", 2, 1, [0], 4096),
                                                  ("rs", 3, 1, [2], 100_003)])
def test_host_path_round_trip(stub, oracle, tmp_path, scheme, p, e, lost, buf):
    _round_trip(oracle, str(tmp_path), scheme, p, e, lost, buf, p * 10 + e, 200_000)


@pytest.mark.parametrize("seed", range(6))
def test_host_path_random(stub, oracle, tmp_path, seed):
    rng = np.random.default_rng(4400 + seed)
    scheme = "xor" if seed % 3 == 2 else "rs"
    p = int(rng.integers(3 if scheme == "rs" else 2, 9))
    e = 1 if scheme == "xor" else int(rng.integers(1, min(p - 1, 4) + 1))
    buf = int(rng.choice([4096, 65536, 100_003]))
    m = 1 if scheme == "xor" else int(rng.integers(1, e + 1))
    lost = sorted(rng.choice(p, size=m, replace=False).tolist())
    _round_trip(oracle, str(tmp_path), scheme, p, e, lost, buf, 5500 + seed, int(rng.choice([1000, 150_000])))


@pytest.mark.parametrize("scheme,p,e,lost", [("rs", 6, 2, [1, 4]), ("xor", 5, 1, [3])])
def test_host_path_repeated_calls_and_stats(stub, oracle, tmp_path, scheme, p, e, lost):
    """Three calls per process on the cached scratch; the per-call stats
    (include/redset_hip_mpi.h redset_hip_rank_last_stats) count the bytes the
    call moved: every rank reads its d*chunk data bytes and writes its
    e*chunk parity bytes on encode, and sends what its peers receive."""
    enc, _, chunk = _round_trip(oracle, str(tmp_path), scheme, p, e, lost, 32768, 77 + p, 400_000,
                                header=[256] * p, env={"RANK_TEST_REPEAT": "3"})
    assert "call 3 of 3" in enc.stdout, enc.stdout
    d = p - e
    for tag in ("first", "warm"):
        st = _stats(enc.stdout, tag)
        assert st["read_bytes"] == [d * chunk, p * d * chunk], st
        assert st["write_bytes"] == [e * chunk, p * e * chunk], st
        assert st["sent_bytes"][1] == st["recv_bytes"][1] > 0, st
        assert st["seconds"][0] >= st["mpi_seconds"][0] >= 0, st


@pytest.mark.parametrize("scheme,op,fail", [("rs", "encode", 2), ("rs", "rebuild", 3), ("xor", "rebuild", 0),
                                             ("xor", "encode", 1)])
def test_host_path_read_failure_fails_every_rank(stub, oracle, tmp_path, scheme, op, fail):
    tmp = str(tmp_path)
    p, e = (4, 2) if scheme == "rs" else (4, 1)
    rng = np.random.default_rng(3)
    files, chunk = _setup(tmp, p, p - e, rng, 300_000)
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, [512] * p, reds)
    buf = 16384
    args = [scheme, "encode", e, tmp, buf]
    if op == "rebuild":
        res = _run(p, args)
        assert res.returncode == 0, res.stdout + res.stderr
        lost = [1] if scheme == "rs" else [2]
        for r in lost:
            for path, _ in files[r]:
                os.unlink(path)
            os.unlink(reds[r])
        args = [scheme, "rebuild", e, tmp, buf] + lost
    res = _run(p, args, env={"RANK_TEST_FAIL_READ": str(fail)}, timeout=90)
    assert res.returncode != 0, res.stdout + res.stderr
    assert "backend failed" in res.stderr, res.stderr
    assert "signal" not in res.stderr, res.stderr


@pytest.mark.parametrize("scheme,p,e,lost", [("rs", 5, 2, [0, 3]), ("xor", 4, 1, [1])])
def test_host_path_slices_larger_than_buffer(stub, oracle, tmp_path, scheme, p, e, lost):
    """Chunks of ~20 MB with a 64 KiB buffer: the RS backends move slices of
    chunk/16 (~1.3 MB, rank_mpi.c slice_bytes), not the caller's buffer, and
    the RS encode stages whole ring windows (XOR keeps the buffer: the same
    shapes as a control); parity and rebuilt files must not depend on the
    slice."""
    _round_trip(oracle, str(tmp_path), scheme, p, e, lost, 65536, 31 + p, 20_000_000)


ASAN_DRIVER = os.path.join(ROOT, "tests", "asan", "build", "rank_test")


@pytest.mark.parametrize("scheme,p,e,lost,buf,maxsize", [("rs", 6, 2, [1, 4], 65536, 200_000),
                                                          ("rs", 5, 2, [0, 3], 65536, 20_000_000),
                                                          ("xor", 4, 1, [2], 50000, 200_000),
                                                          ("xor", 8, 1, [5], 2048, 200_000)])  # the chain
def test_host_path_under_asan(stub, oracle, tmp_path, scheme, p, e, lost, buf, maxsize):
    """The same host path with the backends' host code built under
    AddressSanitizer (tests/asan, as tests/test_asan_host.py builds it):
    round trips, the RS slice rule's large slices, and repeated calls on
    cached scratch."""
    if not (os.path.exists("/opt/rocm/bin/hipcc") and os.path.exists("/opt/rocm/lib/llvm/bin/clang")):
        pytest.skip("needs hipcc and ROCm's clang")
    res = locked_make(os.path.join(ROOT, "tests", "asan"))
    assert res.returncode == 0, res.stdout + res.stderr
    env = {"_DRIVER": ASAN_DRIVER, "RANK_TEST_REPEAT": "2",
           "ASAN_OPTIONS": "verify_asan_link_order=0:detect_leaks=0:exitcode=86"}
    _, reb, chunk = _round_trip(oracle, str(tmp_path), scheme, p, e, lost, buf, 7 + p, maxsize, env=env)
    if scheme == "xor":
        # the product's order rule (rank_mpi.c xor_decode_host): the chain for
        # p >= 6 with >= 4 slices per hop, else the gather
        chain = p >= 6 and -(-chunk // buf) >= 4 * (p - 1)
        got = _stats(reb.stdout)["recv_bytes"][0]
        assert got == (p if chain else (p - 1) * p) * chunk, (chain, got, chunk)


TWIN_DIR = os.path.join(ROOT, "redset_amd", "lib_test")


@pytest.mark.parametrize("order", ["chain", "gather"])
@pytest.mark.parametrize("p,lost,buf", [(2, [0], 4096), (3, [2], 65536), (6, [1], 40000), (8, [7], 100_003)])
def test_host_path_xor_decode_orders(stub, oracle, tmp_path, order, p, lost, buf):
    """Both orders of the XOR host decode (the chain through the survivors,
    the gather to the root), forced through the test twin's backends."""
    if not os.path.exists(os.path.join(TWIN_DIR, "libredset_hip_mpi.so")):
        pytest.skip("test twin not built")
    ld = os.environ.get("LD_LIBRARY_PATH")
    env = {"REDSET_HIP_TEST_XOR_DECODE": order, "LD_LIBRARY_PATH": TWIN_DIR + (":" + ld if ld else "")}
    _, reb, chunk = _round_trip(oracle, str(tmp_path), "xor", p, 1, lost, buf, 900 + p, 300_000, env=env)
    # the busiest receiver: every member gets p cells in the chain, the root
    # (p - 1) * p in the gather
    got = _stats(reb.stdout)["recv_bytes"][0]
    assert got == (p if order == "chain" else (p - 1) * p) * chunk, (got, chunk)


@pytest.mark.parametrize("exchange", ["host", "sharded-mpi", "sharded-host"])
@pytest.mark.parametrize("scheme,op,rank", [("rs", "encode", 1), ("rs", "rebuild", 3), ("xor", "encode", 0),
                                             ("xor", "rebuild", 2)])
def test_hang_capped_kernel_wait_fails_the_call(stub, oracle, tmp_path, scheme, op, rank, exchange):
    """The fault contract (include/redset_hip.h redset_hip_hang_faults): when
    the kernels' hang count moves during a backend call on one member -- a
    wait with no fallback gave up, so that member's kernel outputs are wrong
    -- that member's call returns REDSET_FAILURE after the collective has run
    (no peer hangs), and the AND-reduce fails every rank
    (src/redset_reedsolomon.c:336-341). The stub moves the count on the named
    rank only."""
    tmp = str(tmp_path)
    p, e = (4, 2) if scheme == "rs" else (4, 1)
    rng = np.random.default_rng(11)
    files, chunk = _setup(tmp, p, p - e, rng, 200_000)
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, [512] * p, reds)
    args = [scheme, "encode", e, tmp, 16384]
    if op == "rebuild":
        res = _run(p, args)
        assert res.returncode == 0, res.stdout + res.stderr
        lost = [1, 2] if scheme == "rs" else [2]
        for r in lost:
            for path, _ in files[r]:
                os.unlink(path)
            os.unlink(reds[r])
        args = [scheme, "rebuild", e, tmp, 16384] + lost
    res = _run(p, args, env={"HIPSTUB_HANG_RANK": str(rank), "RANK_TEST_EXCHANGE": exchange}, timeout=90)
    assert res.returncode != 0, res.stdout + res.stderr
    assert f"{op} exchange {exchange}" in res.stdout, res.stdout
    assert f"rank {rank}: backend failed: a kernel wait hit its hang cap" in res.stderr, res.stderr
    others = [r for r in range(p) if r != rank]
    assert not any(f"rank {r}: backend failed" in res.stderr for r in others), res.stderr
    assert "signal" not in res.stderr, res.stderr


TWIN_DIR = os.path.join(ROOT, "redset_amd", "lib_test")


@pytest.mark.parametrize("scheme,p,e,lost,window", [("rs", 6, 2, [1, 4], 0), ("rs", 5, 3, [0, 2, 4], 0),
                                                     ("xor", 4, 1, [2], 0), ("rs", 4, 2, [0, 3], 65536),
                                                     ("xor", 5, 1, [0], 40000), ("rs", 7, 3, [2, 5, 6], 5000)])
@pytest.mark.parametrize("exchange", ["sharded-mpi", "sharded-host"])
def test_sharded_slot_round_trip(stub, oracle, tmp_path, scheme, p, e, lost, window, exchange):
    """The per-rank backends' sharded exchange on the CPU: the HIP stand-in
    also runs the whole-set plans the sharded plan computes with, so the
    slot's windows, planning, transport reserve, staging and exchanges run end
    to end, encode and rebuild, checked against the oracle. "sharded-mpi":
    rank_mpi.c sharded_slot, the RCCL path's slot over the MPI transport with
    device buffers; "sharded-host": sharded_slot_host, every slab in pinned
    host memory (slice-by-slice reads and writes, no staging). window > 0: the
    test twin with windows of that many bytes, so a set takes several
    (double-buffered, a tail window; 5000-B windows cut ragged slices)."""
    env = {"RANK_TEST_EXCHANGE": exchange, "RANK_TEST_REPEAT": "2"}
    if window:
        env["REDSET_HIP_TEST_SHARDED_WINDOW"] = str(window)
        env["LD_LIBRARY_PATH"] = TWIN_DIR + (":" + os.environ["LD_LIBRARY_PATH"] if os.environ.get("LD_LIBRARY_PATH")
                                               else "")
    enc, reb, chunk = _round_trip(oracle, str(tmp_path), scheme, p, e, lost, 32768, 900 + p, 300_000, env=env)
    assert f"encode exchange {exchange}" in enc.stdout, enc.stdout
    assert f"rebuild exchange {exchange}" in reb.stdout, reb.stdout
    classes = ["read_seconds", "mpi_seconds", "gpu_seconds", "write_seconds", "stage_seconds", "copy_seconds",
               "plan_seconds", "setup_seconds"]
    for res in (enc, reb):
        first, warm = _stats(res.stdout, "first"), _stats(res.stdout, "warm")
        for st in (first, warm):
            # the disjoint classes never exceed the call (per rank: compare sums)
            assert sum(st[k][1] for k in classes) <= st["seconds"][1] * 1.0001, st
            assert st["exchange_seconds"][0] > 0, st
            assert st["sent_bytes"][1] == st["recv_bytes"][1] > 0, st
        # the first call plans its windows; the second finds them in the
        # communicator's slot context (rank_mpi.c slot_ctx_get) and plans nothing
        assert first["plan_seconds"][0] > 0 and warm["plan_seconds"][1] == 0, (first, warm)


@pytest.mark.parametrize("exchange", ["sharded-mpi", "sharded-host"])
def test_sharded_slot_without_the_cache_plans_every_call(stub, oracle, tmp_path, exchange):
    """REDSET_HIP_SCRATCH_CACHE=0: the slot context goes with every call (as the
    reference allocates per call, src/redset_reedsolomon.c:298-302), so the
    second call plans again -- and is still bit-exact."""
    env = {"RANK_TEST_EXCHANGE": exchange, "RANK_TEST_REPEAT": "2", "REDSET_HIP_SCRATCH_CACHE": "0"}
    enc, reb, _ = _round_trip(oracle, str(tmp_path), "rs", 5, 2, [1, 3], 32768, 77, 200_000, env=env)
    for res in (enc, reb):
        assert _stats(res.stdout, "warm")["plan_seconds"][0] > 0, res.stdout


@pytest.mark.parametrize("scheme,p,e,want", [("rs", 6, 2, "sharded-host"), ("rs", 5, 1, "host"), ("xor", 4, 1, "host"),
                                             ("rs", 3, 2, "host"), ("rs", 33, 2, "host")])
def test_auto_encode_exchange(stub, oracle, tmp_path, scheme, p, e, want):
    """AUTO's encode (rank_mpi.c choose_exchange): the host slabs for RS with
    d, e >= 2 up to p = 32 (fewer bytes than the ring), the host ring for XOR,
    e = 1 or d = 1 (the same bytes) and wider sets (a window's messages shrink
    as 1/p); either way bit-exact against the oracle."""
    env = {k: v for k, v in os.environ.items() if k != "RANK_TEST_EXCHANGE"}
    env["_DRIVER"] = RANK_TEST
    tmp = str(tmp_path)
    d = p - e
    rng = np.random.default_rng(p)
    files, chunk = _setup(tmp, p, d, rng, 3000)
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, [100] * p, reds)
    res = _run(p, [scheme, "encode", e, tmp, 4096], env=env, timeout=240)
    assert res.returncode == 0, res.stdout + res.stderr[-3000:]
    assert f"encode exchange {want}" in res.stdout, res.stdout
    lofi = [_logical(fl, d * chunk) for fl in files]
    par = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    if scheme == "rs":
        oracle.OracleRS(p, e).encode_set(lofi, par, chunk)
    else:
        oracle.xor_encode_set(p, lofi, par, chunk)
    for r in range(p):
        assert np.array_equal(np.fromfile(reds[r], dtype=np.uint8)[100:], par[r]), r
