"""GPU + MPI tests of the per-rank backends (libredset_hip_mpi.so): a set of
P MPI processes (sharing the GPU) run redset's per-rank encode / rebuild
calling convention through tests/mpi/rank_test.c. Checks: parity after the
header equals the oracle's on the ranks' padded logical files, and a rebuild
after deleting ranks' files restores them with identical CRC32
(test/test_redset.c:459-589 semantics)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from proc import run_group

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RANK_TEST_BIN: another build of the driver (tools/gpu_asan.sh: host ASan)
RANK_TEST = os.environ.get("RANK_TEST_BIN") or os.path.join(ROOT, "tests", "mpi", "build", "rank_test")
MPIRUN = "/opt/conda/bin/mpirun"


def _have():
    try:
        import torch

        if not torch.cuda.is_available():
            return False
    except Exception:
        return False
    if not os.path.exists(MPIRUN):
        return False
    if not os.path.exists(RANK_TEST):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "mpi")], check=False)
    return os.path.exists(RANK_TEST)


def _mpirun(np_, args, timeout=300, env=None):
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", RANK_TEST] + [str(a) for a in args]
    return run_group(cmd, timeout, env={**os.environ, **(env or {})})


# the multi-rank rebuild's exchange (include/redset_hip_mpi.h): "auto" picks
# RCCL over xGMI when every member owns a GPU of one node -- on the test box
# the members share one GPU, so auto must take the host path --, and
# "sharded-mpi" runs the same sharded plan (gather column slices, gf_mac on
# every GPU, return) over the MPI transport with device buffers, and
# "sharded-host" over slabs in page-locked host memory (the kernels read and
# write them in place; rank_mpi.c sharded_slot_host)
EXCHANGES = ["auto", "sharded-mpi", "sharded-mpi-windows", "sharded-host", "sharded-host-windows"]
TWIN_DIR = os.path.join(ROOT, "redset_amd", "lib_test")


def _exchange_env(exchange):
    if exchange.endswith("-windows"):
        # the test twin (loaded ahead of the driver's RUNPATH) with 64 KiB
        # windows: small sets take several windows
        ld = os.environ.get("LD_LIBRARY_PATH")
        return {"RANK_TEST_EXCHANGE": exchange[:-len("-windows")], "REDSET_HIP_TEST_SHARDED_WINDOW": "65536",
                "LD_LIBRARY_PATH": TWIN_DIR + (":" + ld if ld else "")}
    return {"RANK_TEST_EXCHANGE": exchange}


def _auto_exchange(op, scheme, e, p):
    """what AUTO picks on the test box (its members share one GPU): the host
    path, but an RS encode with e >= 2 over host slabs (rank_mpi.c
    choose_exchange, AUTO_ENCODE_SLABS)"""
    return "sharded-host" if op == "encode" and scheme == "rs" and e >= 2 and p - e >= 2 and p <= 32 else "host"


def _check_exchange(res, exchange, op="rebuild", scheme="rs", e=2, p=6):
    used = _auto_exchange(op, scheme, e, p) if exchange == "auto" else exchange.replace("-windows", "")
    assert f"{op} exchange {used}" in res.stdout, res.stdout


def _setup(tmp, p, d, rng, maxsize):
    files = []
    for r in range(p):
        fl = []
        for k in range(int(rng.integers(1, 4))):
            size = int(rng.integers(0, maxsize))
            path = os.path.join(tmp, f"r{r}_f{k}.dat")
            rng.integers(0, 256, size, dtype=np.uint8).tofile(path)
            fl.append((path, size))
        files.append(fl)
    max_bytes = max(sum(s for _, s in f) for f in files)
    chunk = max(1, -(-max_bytes // d))  # src/redset_reedsolomon.c:485-493
    return files, chunk


def _manifests(tmp, files, chunk, header, reds):
    for r, fl in enumerate(files):
        with open(os.path.join(tmp, f"manifest_{r}.txt"), "w") as f:
            f.write(f"{len(fl)}\n")
            for path, size in fl:
                f.write(f"{path} {size}\n")
            f.write(f"{chunk}\n{header[r]}\n{reds[r]}\n")


def _logical(fl, total):
    cat = np.concatenate([np.fromfile(p, dtype=np.uint8) for p, _ in fl]) if fl else np.zeros(0, np.uint8)
    out = np.zeros(total, np.uint8)
    out[:cat.size] = cat
    return out


@pytest.mark.parametrize("exchange", EXCHANGES)
@pytest.mark.parametrize("scheme,p,e,lost,buf", [("rs", 6, 2, [1, 4], 65536), ("rs", 5, 3, [0, 2, 4], 40000),
                                                  ("xor", 4, 1, [2], 50000)])
def test_mpi_rank_backends(oracle, tmp_path, scheme, p, e, lost, buf, exchange):
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    tmp = str(tmp_path)
    d = p - e
    rng = np.random.default_rng(p * 10 + e)
    files, chunk = _setup(tmp, p, d, rng, 200_000)
    header = [1000 + 7 * r for r in range(p)]
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for fl in files for path, _ in fl}

    res = _mpirun(p, [scheme, "encode", e, tmp, buf], env=_exchange_env(exchange))
    assert res.returncode == 0, res.stdout + res.stderr
    _check_exchange(res, exchange, "encode", scheme, e, p)
    lofi = [_logical(fl, d * chunk) for fl in files]
    want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    if scheme == "rs":
        oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    else:
        oracle.xor_encode_set(p, lofi, want, chunk)
    for r in range(p):
        blob = np.fromfile(reds[r], dtype=np.uint8)
        assert blob.size == header[r] + e * chunk
        assert np.array_equal(blob[header[r]:], want[r]), r

    # lose ranks: files and redundancy file gone (fault injection by unlink)
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    res = _mpirun(p, [scheme, "rebuild", e, tmp, buf] + lost, env=_exchange_env(exchange))
    assert res.returncode == 0, res.stdout + res.stderr
    _check_exchange(res, exchange)
    for r in lost:
        for path, size in files[r]:
            assert os.path.getsize(path) == size
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
        blob = np.fromfile(reds[r], dtype=np.uint8)
        assert np.array_equal(blob[header[r]:header[r] + e * chunk], want[r]), r


@pytest.mark.parametrize("scheme,op,env", [
    ("rs", "encode", {"RANK_TEST_FAIL_READ": "2"}),
    ("rs", "encode", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "1"}),
    ("rs", "rebuild", {"RANK_TEST_FAIL_READ": "3"}),
    ("rs", "rebuild", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "0"}),
    ("xor", "encode", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "2"}),
    # small chunks take the gather to the root, which runs the GPU work
    ("xor", "rebuild", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "2"}),
    # the chain (forced: test twin) runs it on its middle survivors
    # (lost [2]: chain 3 -> 0 -> 1 -> root 2)
    ("xor", "rebuild", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "1", "REDSET_HIP_TEST_XOR_DECODE": "chain"}),
    ("xor", "rebuild", {"RANK_TEST_FAIL_READ": "3", "REDSET_HIP_TEST_XOR_DECODE": "chain"}),
    ("xor", "rebuild", {"RANK_TEST_FAIL_READ": "0"}),
    # the sharded exchange: every member's state is agreed on before each
    # window's exchange, so one member's error stops all of them
    ("rs", "rebuild", {"RANK_TEST_FAIL_READ": "3", "RANK_TEST_EXCHANGE": "sharded-mpi"}),
    ("rs", "rebuild", {"RANK_TEST_FAIL_READ": "0", "RANK_TEST_EXCHANGE": "sharded-mpi"}),
    ("xor", "rebuild", {"RANK_TEST_FAIL_READ": "1", "RANK_TEST_EXCHANGE": "sharded-mpi"}),
    # a device error after the window's agreement: the failing member still
    # runs the window's exchange (its peers are in it) and every member stops
    # at the next agreement (test twin: 64 KiB windows, several per call)
    ("rs", "rebuild", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "2", "RANK_TEST_EXCHANGE": "sharded-mpi",
                       "REDSET_HIP_TEST_SHARDED_WINDOW": "65536"}),
    ("xor", "rebuild", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "3", "RANK_TEST_EXCHANGE": "sharded-mpi",
                        "REDSET_HIP_TEST_SHARDED_WINDOW": "65536"}),
    ("rs", "rebuild", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "0", "RANK_TEST_EXCHANGE": "sharded-mpi"}),
    # the encodes through the sharded exchange (the path a node with a GPU
    # per member takes over RCCL)
    ("rs", "encode", {"RANK_TEST_FAIL_READ": "2", "RANK_TEST_EXCHANGE": "sharded-mpi"}),
    ("rs", "encode", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "1", "RANK_TEST_EXCHANGE": "sharded-mpi",
                      "REDSET_HIP_TEST_SHARDED_WINDOW": "65536"}),
    ("xor", "encode", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "3", "RANK_TEST_EXCHANGE": "sharded-mpi",
                       "REDSET_HIP_TEST_SHARDED_WINDOW": "65536"}),
    # the same over host slabs
    ("rs", "rebuild", {"RANK_TEST_FAIL_READ": "3", "RANK_TEST_EXCHANGE": "sharded-host"}),
    ("rs", "encode", {"RANK_TEST_FAIL_READ": "2", "RANK_TEST_EXCHANGE": "sharded-host"}),
    ("rs", "encode", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "1", "RANK_TEST_EXCHANGE": "sharded-host",
                      "REDSET_HIP_TEST_SHARDED_WINDOW": "65536"}),
    ("xor", "rebuild", {"REDSET_HIP_INJECT_DEVICE_FAILURE": "3", "RANK_TEST_EXCHANGE": "sharded-host",
                        "REDSET_HIP_TEST_SHARDED_WINDOW": "65536"}),
])
def test_mpi_rank_failure_fails_every_rank_without_hang(oracle, tmp_path, scheme, op, env):
    """One member's I/O or device error in the middle of the loop: that member
    keeps every MPI call of the collective going (as src/redset_reedsolomon.c:
    338-342 does on read errors), returns REDSET_FAILURE, and the caller's
    AND-reduce (redset_alltrue) fails every rank. No rank may hang."""
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    tmp = str(tmp_path)
    p, e = (4, 2) if scheme == "rs" else (4, 1)
    d = p - e
    rng = np.random.default_rng(3)
    files, chunk = _setup(tmp, p, d, rng, 300_000)
    header = [512] * p
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    buf = 16384  # several slices per chunk: the failure lands mid-loop
    if op == "rebuild":
        res = _mpirun(p, [scheme, "encode", e, tmp, buf])
        assert res.returncode == 0, res.stdout + res.stderr
        lost = [1] if scheme == "rs" else [2]
        for r in lost:
            for path, _ in files[r]:
                os.unlink(path)
            os.unlink(reds[r])
        args = [scheme, "rebuild", e, tmp, buf] + lost
    else:
        args = [scheme, "encode", e, tmp, buf]
    cmd = [MPIRUN, "-np", str(p), "-host", "localhost", RANK_TEST] + [str(a) for a in args]
    env = {**os.environ, **env}
    if any(k == "REDSET_HIP_INJECT_DEVICE_FAILURE" or k.startswith("REDSET_HIP_TEST_") for k in env):
        # only the test twin honours the injection knob (the product reads no
        # environment): the driver loads it ahead of its RUNPATH
        twin = os.path.join(ROOT, "redset_amd", "lib_test")
        env["LD_LIBRARY_PATH"] = twin + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else "")
    res = run_group(cmd, 90, env=env)
    assert res.returncode != 0, res.stdout + res.stderr  # every rank exits 1 (alltrue is false)
    assert "backend failed" in res.stderr
    assert "Sanitizer" not in res.stderr, res.stderr[-4000:]  # tools/gpu_asan.sh builds


@pytest.mark.parametrize("mode", ["--gpu", "--gpu-host", "--gpu-host-null"])
@pytest.mark.parametrize("np_,p,e,chunk,lost", [(2, 11, 3, 300_001, [1, 2]), (4, 20, 4, 65536, [0, 5, 19]),
                                                 (3, 6, 3, 1000, [2])])
def test_mpi_sharded_gpu(np_, p, e, chunk, lost, mode):
    """The sharded path with the real HIP kernels at world > 1: gf_mac plans
    over each process's column slice (the processes share the box's one GPU;
    RCCL needs one GPU per rank). --gpu: slabs in HBM, the MPI transport
    staging through pinned memory. --gpu-host: slabs in page-locked host
    memory that the kernels read and write in place and MPI sends directly,
    so the transport must wait for the stream's kernels before a return
    exchange (rank_mpi.c mpi_exchange). tests/mpi/sharded_test.c
    checks hosted parity and the rebuilt members against the oracle."""
    driver = os.environ.get("SHARDED_TEST_BIN") or os.path.join(ROOT, "tests", "mpi", "build", "sharded_test")
    if not _have() or not os.path.exists(driver):
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/sharded_test")
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", driver, mode, str(p), str(e), str(chunk)] + \
        [str(x) for x in lost]
    res = run_group(cmd, 120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == np_


@pytest.mark.parametrize("exchange", EXCHANGES)
def test_mpi_config0_xor_4_ranks_16MiB(oracle, tmp_path, exchange):
    """BASELINE.json configs[0] at its own shape through the drop-in per-rank
    XOR backend: 4 MPI ranks, one 16 MiB file each (chunk = ceil(16 MiB / 3),
    src/redset_xor.c's rule), 1 MiB MPI buffer; encode, lose rank 2, rebuild."""
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    tmp = str(tmp_path)
    p, e, size = 4, 1, 16 << 20
    rng = np.random.default_rng(0xC0)
    files = []
    for r in range(p):
        path = os.path.join(tmp, f"r{r}.dat")
        rng.integers(0, 256, size, dtype=np.uint8).tofile(path)
        files.append([(path, size)])
    chunk = -(-size // (p - 1))
    header = [4096] * p
    reds = [os.path.join(tmp, f"r{r}.xor.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    res = _mpirun(p, ["xor", "encode", e, tmp, 1 << 20], env=_exchange_env(exchange))
    assert res.returncode == 0, res.stdout + res.stderr
    _check_exchange(res, exchange, "encode", "xor", e, p)
    lofi = [_logical(fl, (p - 1) * chunk) for fl in files]
    want = [np.zeros(chunk, np.uint8) for _ in range(p)]
    oracle.xor_encode_set(p, lofi, want, chunk)
    for r in range(p):
        assert np.array_equal(np.fromfile(reds[r], dtype=np.uint8)[4096:], want[r]), r
    crc = oracle.crc32(lofi[2][:size])
    os.unlink(files[2][0][0])
    os.unlink(reds[2])
    res = _mpirun(p, ["xor", "rebuild", e, tmp, 1 << 20, 2], env=_exchange_env(exchange))
    assert res.returncode == 0, res.stdout + res.stderr
    _check_exchange(res, exchange)
    assert os.path.getsize(files[2][0][0]) == size
    assert oracle.crc32(np.fromfile(files[2][0][0], dtype=np.uint8)) == crc
    assert np.array_equal(np.fromfile(reds[2], dtype=np.uint8)[4096:], want[2])


@pytest.mark.parametrize("seed", range(6))
def test_mpi_sharded_gpu_random(seed):
    """tests/test_mpi_sharded.py's random shapes and placements with the HIP
    kernels and the pipelined execute (even seeds: slabs in HBM, MPI
    transport staging through pinned memory; odd seeds: page-locked host
    slabs; the processes share the box's GPU)."""
    mode = "--gpu-host" if seed % 2 else "--gpu"
    driver = os.environ.get("SHARDED_TEST_BIN") or os.path.join(ROOT, "tests", "mpi", "build", "sharded_test")
    if not _have() or not os.path.exists(driver):
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/sharded_test")
    rng = np.random.default_rng(5000 + seed)
    np_ = int(rng.integers(1, 5))
    p = int(rng.integers(2, 24))
    e = int(rng.integers(1, min(p - 1, 6) + 1))
    chunk = int(rng.choice([1, 255, 257, int(rng.integers(2, 200_000))]))
    m = int(rng.integers(1, e + 1))
    lost = sorted(rng.choice(p, size=m, replace=False).tolist())
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", driver, mode, str(p), str(e), str(chunk)] + \
        [str(x) for x in lost]
    res = run_group(cmd, 120, env={**os.environ, "SHARDED_TEST_SEED": str(seed)})
    assert res.returncode == 0, (np_, p, e, chunk, lost, res.stdout + res.stderr)
    assert res.stdout.count("rebuild gather") == np_


@pytest.mark.parametrize("exchange", EXCHANGES)
@pytest.mark.parametrize("scheme,p,e,lost", [("rs", 6, 2, [1, 4]), ("xor", 5, 1, [3])])
def test_mpi_rank_backends_repeated_calls(oracle, tmp_path, scheme, p, e, lost, exchange):
    """Three backend calls per process (RANK_TEST_REPEAT=3): the second and
    third run on the scratch and stream the first left in the process-wide
    cache (dirty buffers), and must write the same bytes."""
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    tmp = str(tmp_path)
    d = p - e
    rng = np.random.default_rng(77 + p)
    files, chunk = _setup(tmp, p, d, rng, 400_000)
    header = [256] * p
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for fl in files for path, _ in fl}
    env = {**os.environ, "RANK_TEST_REPEAT": "3", **_exchange_env(exchange)}
    cmd = [MPIRUN, "-np", str(p), "-host", "localhost", RANK_TEST, scheme, "encode", str(e), tmp, "32768"]
    res = run_group(cmd, 120, env=env)
    assert res.returncode == 0 and "call 3 of 3" in res.stdout, res.stdout + res.stderr
    _check_exchange(res, exchange, "encode", scheme, e, p)
    lofi = [_logical(fl, d * chunk) for fl in files]
    want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    if scheme == "rs":
        oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    else:
        oracle.xor_encode_set(p, lofi, want, chunk)
    for r in range(p):
        assert np.array_equal(np.fromfile(reds[r], dtype=np.uint8)[256:], want[r]), r
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    cmd = [MPIRUN, "-np", str(p), "-host", "localhost", RANK_TEST, scheme, "rebuild", str(e), tmp, "32768"] + \
        [str(x) for x in lost]
    res = run_group(cmd, 120, env={**env, **_exchange_env(exchange)})
    assert res.returncode == 0 and "call 3 of 3" in res.stdout, res.stdout + res.stderr
    _check_exchange(res, exchange)
    for r in lost:
        for path, _ in files[r]:
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
        assert np.array_equal(np.fromfile(reds[r], dtype=np.uint8)[256:256 + e * chunk], want[r]), r


@pytest.mark.parametrize("seed", range(8))
def test_mpi_rank_backends_random(oracle, tmp_path, seed):
    """Seeded random sets through the per-rank backends: scheme, ranks (2-12,
    within the box's GPU-process limit), encoding, MPI buffer size (odd sizes
    included), file lists and erasures; parity against the oracle, rebuilt
    files by CRC32."""
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    rng = np.random.default_rng(9000 + seed)
    scheme = "xor" if seed % 3 == 2 else "rs"
    p = int(rng.integers(3 if scheme == "rs" else 2, 13))
    e = 1 if scheme == "xor" else int(rng.integers(1, min(p - 1, 5) + 1))
    d = p - e
    buf = int(rng.choice([4096, 65536, 100_003, 1 << 20]))
    m = 1 if scheme == "xor" else int(rng.integers(1, e + 1))
    lost = sorted(rng.choice(p, size=m, replace=False).tolist())
    tmp = str(tmp_path)
    files, chunk = _setup(tmp, p, d, rng, int(rng.choice([1000, 150_000, 700_000])))
    header = [int(rng.integers(0, 5000)) for _ in range(p)]
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for fl in files for path, _ in fl}
    exchange = EXCHANGES[seed % len(EXCHANGES)]
    res = _mpirun(p, [scheme, "encode", e, tmp, buf], timeout=120, env=_exchange_env(exchange))
    assert res.returncode == 0, (scheme, p, e, buf, exchange, res.stdout + res.stderr)
    _check_exchange(res, exchange, "encode", scheme, e, p)
    lofi = [_logical(fl, d * chunk) for fl in files]
    want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    if scheme == "rs":
        oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    else:
        oracle.xor_encode_set(p, lofi, want, chunk)
    for r in range(p):
        assert np.array_equal(np.fromfile(reds[r], dtype=np.uint8)[header[r]:], want[r]), (scheme, p, e, r)
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    res = _mpirun(p, [scheme, "rebuild", e, tmp, buf] + lost, timeout=120, env=_exchange_env(exchange))
    assert res.returncode == 0, (scheme, p, e, buf, lost, exchange, res.stdout + res.stderr)
    _check_exchange(res, exchange)
    for r in lost:
        for path, size in files[r]:
            assert os.path.getsize(path) == size
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
        blob = np.fromfile(reds[r], dtype=np.uint8)
        assert np.array_equal(blob[header[r]:header[r] + e * chunk], want[r]), r


def test_mpi_forced_rccl_exchange_on_a_shared_gpu_fails_every_rank(tmp_path):
    """`redset_hip_rank_set_exchange(SHARDED_RCCL)` with the members sharing
    the box's one GPU: RCCL refuses the communicator ("Duplicate GPU"), the
    members agree on that (rank_mpi.c rccl_create's MPI_Allreduce) and every
    one returns failure before any exchange -- no hang, no partial writes."""
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    tmp = str(tmp_path)
    p, e = 4, 2
    rng = np.random.default_rng(5)
    files, chunk = _setup(tmp, p, p - e, rng, 100_000)
    reds = [os.path.join(tmp, f"r{r}.rs.redset") for r in range(p)]
    _manifests(tmp, files, chunk, [128] * p, reds)
    res = _mpirun(p, ["rs", "encode", e, tmp, 65536])
    assert res.returncode == 0, res.stdout + res.stderr
    for path, _ in files[1]:
        os.unlink(path)
    os.unlink(reds[1])
    res = _mpirun(p, ["rs", "rebuild", e, tmp, 65536, 1], timeout=120, env={"RANK_TEST_EXCHANGE": "rccl"})
    assert res.returncode != 0, res.stdout + res.stderr
    assert res.stderr.count("backend failed") == p, res.stderr
    # the driver creates the lost member's files at their recorded sizes
    # (zeros); nothing was written into them
    for path, _ in files[1]:
        assert not os.path.exists(path) or not np.fromfile(path, dtype=np.uint8).any(), path


@pytest.mark.parametrize("order", ["chain", "gather"])
@pytest.mark.parametrize("p,lost,buf", [(2, 0, 4096), (3, 2, 65536), (5, 1, 40000), (8, 6, 100_003)])
def test_mpi_xor_decode_orders(oracle, tmp_path, order, p, lost, buf):
    """Both host orders of the XOR rebuild (rank_mpi.c xor_decode_host: the
    chain through the survivors, the gather to the root), forced through the
    test twin whatever the chunk size picks: rebuilt files by CRC32 and the
    root's parity bytes against the oracle."""
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    tmp = str(tmp_path)
    rng = np.random.default_rng(600 + p)
    files, chunk = _setup(tmp, p, p - 1, rng, 300_000)
    header = [int(rng.integers(0, 3000)) for _ in range(p)]
    reds = [os.path.join(tmp, f"r{r}.xor.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for path, _ in files[lost]}
    res = _mpirun(p, ["xor", "encode", 1, tmp, buf])
    assert res.returncode == 0, res.stdout + res.stderr
    want = np.fromfile(reds[lost], dtype=np.uint8)[header[lost]:].copy()
    for path, _ in files[lost]:
        os.unlink(path)
    os.unlink(reds[lost])
    ld = os.environ.get("LD_LIBRARY_PATH")
    env = {"REDSET_HIP_TEST_XOR_DECODE": order, "LD_LIBRARY_PATH": TWIN_DIR + (":" + ld if ld else "")}
    res = _mpirun(p, ["xor", "rebuild", 1, tmp, buf, lost], env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    for path, size in files[lost]:
        assert os.path.getsize(path) == size
        assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
    assert np.array_equal(np.fromfile(reds[lost], dtype=np.uint8)[header[lost]:], want)


@pytest.mark.parametrize("exchange", ["auto", "sharded-mpi", "sharded-host"])
def test_mpi_rs_slices_larger_than_the_buffer(oracle, tmp_path, exchange):
    """~20 MB chunks with a 64 KiB buffer: the RS backends move slices of
    chunk/16 (rank_mpi.c slice_bytes) and the encode stages whole ring
    windows, on the GPU; parity against the oracle, rebuilt files by CRC32."""
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    tmp = str(tmp_path)
    p, e, lost, buf = 6, 2, [0, 3], 65536
    d = p - e
    rng = np.random.default_rng(4242)
    files, chunk = _setup(tmp, p, d, rng, 30_000_000)
    header = [4096] * p
    reds = [os.path.join(tmp, f"r{r}.rs.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for r in lost for path, _ in files[r]}
    res = _mpirun(p, ["rs", "encode", e, tmp, buf], env=_exchange_env(exchange))
    assert res.returncode == 0, res.stdout + res.stderr
    lofi = [_logical(fl, d * chunk) for fl in files]
    want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    for r in range(p):
        assert np.array_equal(np.fromfile(reds[r], dtype=np.uint8)[4096:], want[r]), r
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    res = _mpirun(p, ["rs", "rebuild", e, tmp, buf] + lost, env=_exchange_env(exchange))
    assert res.returncode == 0, res.stdout + res.stderr
    for r in lost:
        for path, size in files[r]:
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
        assert np.array_equal(np.fromfile(reds[r], dtype=np.uint8)[4096:], want[r]), r


@pytest.mark.parametrize("exchange", ["sharded-mpi", "sharded-host"])
@pytest.mark.parametrize("scheme,op", [("rs", "encode"), ("rs", "rebuild")])
def test_mpi_hang_cap_fails_the_call(oracle, tmp_path, scheme, op, exchange):
    """The fault contract through the drop-in slot (include/redset_hip.h
    redset_hip_hang_faults): the sharded exchange's plans forced into streamed
    pairs (test twin, REDSET_HIP_SEQUENTIAL=3) with a loader that sleeps
    before it publishes a job's tables and a 1-poll hang cap, so the
    consumers' table hand-over gives up and the kernels' outputs are wrong.
    Every member whose kernels hit the cap must return REDSET_FAILURE -- the
    call never reports success with those bytes -- and no member may hang
    (src/redset_reedsolomon.c:336-341). The control run with the product's
    hang cap and the same delay succeeds and is checked like any other."""
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    tmp = str(tmp_path)
    p, e = (4, 2) if scheme == "rs" else (4, 1)
    d = p - e
    rng = np.random.default_rng(21)
    files, chunk = _setup(tmp, p, d, rng, 400_000)
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, [512] * p, reds)
    ld = os.environ.get("LD_LIBRARY_PATH")
    stall = {"RANK_TEST_EXCHANGE": exchange, "REDSET_HIP_SEQUENTIAL": "3",
             "REDSET_HIP_TEST_TABLE_DELAY": "400", "LD_LIBRARY_PATH": TWIN_DIR + (":" + ld if ld else "")}
    args = [scheme, "encode", e, tmp, 16384]
    if op == "rebuild":
        res = _mpirun(p, args, env=stall)  # control: the product's hang cap
        assert res.returncode == 0, res.stdout + res.stderr
        lost = [0, 3] if scheme == "rs" else [1]
        for r in lost:
            for path, _ in files[r]:
                os.unlink(path)
            os.unlink(reds[r])
        args = [scheme, "rebuild", e, tmp, 16384] + lost
    res = _mpirun(p, args, timeout=120, env={**stall, "REDSET_HIP_TEST_HANG_CAP": "1"})
    assert res.returncode != 0, res.stdout + res.stderr
    assert "hit its hang cap" in res.stderr, res.stderr[-4000:]
    assert "signal" not in res.stderr, res.stderr[-4000:]
    if op == "encode":
        res = _mpirun(p, args, env=stall)  # control
        assert res.returncode == 0, res.stdout + res.stderr
        lofi = [_logical(fl, d * chunk) for fl in files]
        want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
        oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
        for r in range(p):
            assert np.array_equal(np.fromfile(reds[r], dtype=np.uint8)[512:], want[r]), r


@pytest.mark.parametrize("scheme,p,e,lost", [("rs", 4, 2, [1, 3]), ("xor", 3, 1, [2])])
def test_mpi_auto_rebuild_takes_rccl_with_a_gpu_per_member(oracle, tmp_path, scheme, p, e, lost):
    """AUTO's production layout: members on one node, each on its
    own GPU. The encode stays off RCCL (host ring or host slabs); the rebuild must take the
    RCCL exchange (rank_mpi.c choose_exchange) and restore the lost members
    bit for bit. Needs >= p GPUs: the one-GPU test box skips it, a node with
    8 GPUs runs it (src/redset_reedsolomon.c:646-733 replaced)."""
    if not _have():
        pytest.skip("needs a GPU, MPICH and tests/mpi/build/rank_test")
    import torch

    if torch.cuda.device_count() < p:
        pytest.skip(f"needs {p} GPUs, one per member ({torch.cuda.device_count()} here)")
    tmp = str(tmp_path)
    d = p - e
    rng = np.random.default_rng(17)
    files, chunk = _setup(tmp, p, d, rng, 3_000_000)
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, [256] * p, reds)
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for fl in files for path, _ in fl}
    env = {"RANK_TEST_DEVICE_PER_RANK": "1"}
    res = _mpirun(p, [scheme, "encode", e, tmp, 1 << 20], env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    assert f"encode exchange {_auto_exchange('encode', scheme, e, p)}" in res.stdout, res.stdout
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    res = _mpirun(p, [scheme, "rebuild", e, tmp, 1 << 20] + lost, env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "rebuild exchange rccl" in res.stdout, res.stdout
    for r in lost:
        for path, size in files[r]:
            assert os.path.getsize(path) == size
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
