"""The sharded path's C planner under mpirun on CPU (no GPU): each MPI
process plays one GPU of the node, column slices move through the MPI
transport of libredset_hip_mpi.so (redset_hip_mpi_transport_*, host buffers),
and the compute is a callback into the CPU oracle. tests/mpi/sharded_test.c
checks every process's hosted parity after the encode and its lost members'
cells after the rebuild against the oracle's whole-set answer."""
import os
import shutil
import subprocess

import pytest

from proc import leaked_stub_shm, run_group, stub_shm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "mpi", "build", "sharded_test")
MPIRUN = "/opt/conda/bin/mpirun"


def _have():
    if not os.path.exists(MPIRUN) or not os.path.exists(os.path.join(ROOT, "redset_amd", "lib",
                                                                     "libredset_hip_mpi.so")):
        return False
    if not os.path.exists(DRIVER) and shutil.which("make"):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "mpi")], check=False)
    return os.path.exists(DRIVER)


@pytest.mark.parametrize("np_,p,e,chunk,lost", [
    (2, 11, 3, 3001, [1, 2]),      # configs[3]'s shape, small chunk
    (4, 11, 3, 4096, [1, 2]),
    (4, 20, 4, 777, [0, 5, 19]),   # configs[4]'s shape
    (3, 5, 2, 1000, [0, 4]),
    (2, 6, 3, 1, [2]),             # one-byte chunk: the second slice is empty
    (1, 11, 3, 500, [4, 7, 10]),
])
def test_sharded_plan_over_mpi_matches_oracle(oracle, np_, p, e, chunk, lost):
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, str(p), str(e), str(chunk)] + [str(x) for x in lost]
    res = run_group(cmd, 120, cwd="/tmp")
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == np_


@pytest.mark.parametrize("seed", range(30))
def test_sharded_plan_random_shapes_and_placements(oracle, seed):
    """Seeded random set shapes, erasures, chunk sizes, world sizes and
    member placements (pseudo-random processes, unbalanced slot counts):
    the planner's gather/return against the oracle's whole-set answer."""
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    import numpy as np

    rng = np.random.default_rng(4000 + seed)
    np_ = int(rng.integers(1, 5))
    p = int(rng.integers(2, 24))
    e = int(rng.integers(1, min(p - 1, 6) + 1))
    chunk = int(rng.choice([1, 255, 256, 257, int(rng.integers(2, 5000))]))
    m = int(rng.integers(1, e + 1))
    lost = sorted(rng.choice(p, size=m, replace=False).tolist())
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, str(p), str(e), str(chunk)] + [str(x) for x in lost]
    res = run_group(cmd, 120, env={**os.environ, "SHARDED_TEST_SEED": str(seed)}, cwd="/tmp")
    assert res.returncode == 0, (np_, p, e, chunk, lost, res.stdout + res.stderr)
    assert res.stdout.count("rebuild gather") == np_


@pytest.mark.parametrize("scheme,np_,p,e,chunk,lost,idle", [
    ("rs", 4, 11, 3, 3001, [1, 2], "1"), ("rs", 4, 11, 3, 4096, [1, 2], "0,2"), ("rs", 3, 6, 2, 1000, [0, 4], "2"),
    ("rs", 4, 20, 4, 777, [0, 5, 19], "3"), ("rs", 2, 6, 3, 1, [2], "0"), ("xor", 4, 5, 1, 999, [3], "1,3")])
@pytest.mark.parametrize("shape", ["", "auto"])
def test_sharded_plan_with_idle_processes(oracle, scheme, np_, p, e, chunk, lost, idle, shape):
    """redset_hip_{rs,xor}_sharded_plan_on: some processes compute no column
    slice (the slot's host-slab decode keeps its lost members out of the
    compute), the others take slices 0 .. K - 1 of ceil(C / K); every process
    still hosts members, sends their cells and receives their outputs.
    Parity after the encode and the lost members after the rebuild against the
    oracle."""
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, str(p), str(e), str(chunk)] + [str(x) for x in lost]
    env = {**os.environ, "SHARDED_TEST_IDLE": idle}
    if scheme == "xor":
        env["SHARDED_TEST_SCHEME"] = "xor"
    if shape:
        # through the _ex entry point: a compute mask keeps the gather shape,
        # and the driver checks the shape info's byte counts against the lists
        env["SHARDED_TEST_SHAPE"] = shape
    res = run_group(cmd, 120, env=env, cwd="/tmp")
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == np_
    if shape:
        assert res.stdout.count("rebuild shape gather") == np_, res.stdout


@pytest.mark.parametrize("np_,p,chunk,root", [
    (2, 8, 3001, 3),     # configs[1]'s shape, small chunk
    (4, 4, 4096, 0),     # configs[0]'s set size
    (3, 5, 1, 4),        # one-byte chunk
    (4, 9, 777, 8),
    (1, 6, 500, 2),
])
def test_xor_sharded_plan_over_mpi_matches_oracle(oracle, np_, p, chunk, root):
    """XOR sets through the same planner (redset_hip_xor_sharded_plan): the
    encode gathers every member's p - 1 logical-file segments, the rebuild
    every survivor's every cell (in place of the reference's pipelined reduce
    to the lost member, src/redset_xor.c:466-524); parity and the rebuilt
    member against the oracle's XOR (src/redset_xor.c:220-295,
    src/redset_xor_serial.c:161-275)."""
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, str(p), "1", str(chunk), str(root)]
    res = run_group(cmd, 120, env={**os.environ, "SHARDED_TEST_SCHEME": "xor"}, cwd="/tmp")
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == np_


@pytest.mark.parametrize("seed", range(8))
def test_xor_sharded_plan_random(oracle, seed):
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    import numpy as np

    rng = np.random.default_rng(7000 + seed)
    np_ = int(rng.integers(1, 5))
    p = int(rng.integers(2, 20))
    chunk = int(rng.choice([1, 255, 257, int(rng.integers(2, 5000))]))
    root = int(rng.integers(0, p))
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, str(p), "1", str(chunk), str(root)]
    env = {**os.environ, "SHARDED_TEST_SCHEME": "xor", "SHARDED_TEST_SEED": str(seed)}
    res = run_group(cmd, 120, env=env, cwd="/tmp")
    assert res.returncode == 0, (np_, p, chunk, root, res.stdout + res.stderr)
    assert res.stdout.count("rebuild gather") == np_


RANK_TEST = os.path.join(ROOT, "tests", "mpi", "build", "rank_test")


def _rank_test_set(tmp, p, chunk):
    for r in range(p):
        path = os.path.join(tmp, f"r{r}.dat")
        with open(path, "wb") as f:
            f.write(bytes((r * 7 + i) & 0xFF for i in range(chunk * 2)))
        with open(os.path.join(tmp, f"manifest_{r}.txt"), "w") as f:
            f.write(f"1\n{path} {chunk * 2}\n{chunk}\n64\n{os.path.join(tmp, f'r{r}.red')}\n")
        with open(os.path.join(tmp, f"r{r}.red"), "wb") as f:
            f.write(b"H" * 64 + bytes(chunk * 2))


@pytest.mark.parametrize("op", ["rebuild", "encode"])
@pytest.mark.parametrize("exchange,used", [("", None), ("host", "host"), ("sharded-mpi", "sharded-mpi"),
                                           ("sharded-host", "sharded-host")])
def test_rebuild_exchange_choice_on_cpu(tmp_path, exchange, used, op):
    """The per-rank backends' exchange choice (rank_mpi.c choose_exchange) is
    collective and agreed before any exchange: on a machine without a GPU,
    "auto" finds no GPU per member and takes the host path for the decode
    (and, RS(2+2) here, the host slabs for the encode), a forced mode is taken
    as asked, and the call then fails on every member (no HIP device) without
    a hang. The GPU tests run the same choices to completion."""
    if used is None:
        used = "sharded-host" if op == "encode" else "host"
    if not _have() or not os.path.exists(RANK_TEST):
        pytest.skip("needs MPICH and tests/mpi/build/rank_test")
    from conftest import gpu_available

    if gpu_available():
        pytest.skip("CPU-only check (on a GPU box the decode runs: tests/test_gpu_mpi.py)")
    tmp = str(tmp_path)
    _rank_test_set(tmp, 4, 1000)
    env = {**os.environ}
    env.pop("RANK_TEST_EXCHANGE", None)
    if exchange:
        env["RANK_TEST_EXCHANGE"] = exchange
    cmd = [MPIRUN, "-np", "4", "-host", "localhost", RANK_TEST, "rs", op, "2", tmp, "4096"] + \
        (["1", "2"] if op == "rebuild" else [])
    res = run_group(cmd, 60, env=env, cwd="/tmp")
    assert res.returncode != 0
    assert f"{op} exchange {used}" in res.stdout, res.stdout + res.stderr
    assert res.stderr.count("backend failed") == 4, res.stderr


def test_rebuild_exchange_members_must_agree(tmp_path):
    """Members asking for different exchanges fail together (one allreduce
    of the mode) instead of deadlocking in mismatched exchanges."""
    if not _have() or not os.path.exists(RANK_TEST):
        pytest.skip("needs MPICH and tests/mpi/build/rank_test")
    tmp = str(tmp_path)
    _rank_test_set(tmp, 4, 1000)
    args = [RANK_TEST, "rs", "rebuild", "2", tmp, "4096", "1", "2"]
    cmd = [MPIRUN, "-host", "localhost", "-n", "1", "-env", "RANK_TEST_EXCHANGE", "sharded-mpi"] + args + \
        [":", "-n", "3", "-env", "RANK_TEST_EXCHANGE", "host"] + args
    res = run_group(cmd, 60, cwd="/tmp")
    assert res.returncode != 0
    assert "disagree on the rebuild exchange" in res.stderr, res.stderr
    assert res.stderr.count("backend failed") == 4, res.stderr


@pytest.mark.parametrize("scheme,np_,p,e,fail", [("rs", 3, 11, 3, 1), ("rs", 4, 6, 2, 0), ("xor", 3, 5, 1, 2)])
def test_sharded_compute_failure_keeps_the_exchange_going(scheme, np_, p, e, fail):
    """One process's compute fails inside the sharded encode: its plan still
    runs the return exchange its peers are waiting in (sharded.c
    execute_pipelined / redset_hip_sharded_execute), so every process comes
    back, the failing one with an error, and the AND of the results fails
    (src/redset_reedsolomon.c:338-342)."""
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, str(p), str(e), "5000"]
    env = {**os.environ, "SHARDED_TEST_FAIL_COMPUTE": str(fail)}
    if scheme == "xor":
        env["SHARDED_TEST_SCHEME"] = "xor"
    res = run_group(cmd, 60, env=env, cwd="/tmp")
    assert res.returncode != 0, res.stdout + res.stderr
    assert f"rank {fail}: encode:" in res.stderr, res.stderr
    assert "compute callback failed" in res.stderr, res.stderr


# ---- the partial-sum shape (REDSET_HIP_SHAPE_REDUCE) ----------------------


def _shapes(stdout):
    """(op, planned shape, gather busiest, reduce busiest) per printed line"""
    import re

    return [(m.group(1), m.group(2), int(m.group(3)), int(m.group(4)))
            for m in re.finditer(r"rank \d+: (encode|rebuild) shape (\w+) \(asked \w+\): gather busiest (\d+) B, "
                                 r"reduce busiest (\d+) B", stdout)]


@pytest.mark.parametrize("shape", ["reduce", "auto"])
@pytest.mark.parametrize("scheme,np_,p,e,chunk,lost", [
    ("rs", 2, 11, 3, 3001, [1, 2]),     # configs[3]'s shape
    ("rs", 3, 11, 3, 4096, [1, 2]),
    ("rs", 2, 20, 4, 777, [0, 5, 19]),  # configs[4]'s shape
    ("rs", 3, 5, 2, 1000, [0, 4]),
    ("rs", 2, 6, 3, 1, [2]),            # one-byte chunk: one slice with bytes
    ("rs", 6, 7, 2, 1, [4, 6]),
    ("xor", 3, 8, 1, 3001, [3]),        # configs[1]'s shape
    ("xor", 4, 12, 1, 1, [5]),
])
def test_reduce_shape_matches_oracle(oracle, shape, scheme, np_, p, e, chunk, lost):
    """The sharded plan's partial-sum shape (sharded.c plan_reduce): every
    process combines ITS members' cells into partial outputs with the stripe's
    own coefficients (the oracle's multadd does the combines here), sends one
    partial per output it feeds to the output's host, which XORs them in.
    Parity after the encode and the lost members after the rebuild against the
    oracle's whole-set answer; every process plans the same shape from the
    same byte counts, and AUTO takes the one whose busiest process moves
    fewer bytes."""
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, str(p), str(e), str(chunk)] + [str(x) for x in lost]
    env = {**os.environ, "SHARDED_TEST_SHAPE": shape}
    if scheme == "xor":
        env["SHARDED_TEST_SCHEME"] = "xor"
    res = run_group(cmd, 120, env=env, cwd="/tmp")
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == np_
    lines = _shapes(res.stdout)
    assert len(lines) == 2 * np_, res.stdout
    for op in ("encode", "rebuild"):
        mine = {x[1:] for x in lines if x[0] == op}
        assert len(mine) == 1, mine  # the same plan everywhere
        planned, gb, rb = mine.pop()
        if shape == "reduce":
            assert planned == "reduce"
        else:
            assert planned == ("reduce" if rb < gb else "gather"), (op, planned, gb, rb)


def test_reduce_shape_moves_fewer_bytes_at_the_bench_shape(oracle):
    """configs[3] at N = 2, two sets of RS(8+3) with members 1, 2 lost: the
    rebuild's busiest process sends 2.5x fewer bytes as partial sums than as
    gathered input slices."""
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    cmd = [MPIRUN, "-np", "2", "-host", "localhost", DRIVER, "11", "3", "4096", "1", "2"]
    res = run_group(cmd, 120, env={**os.environ, "SHARDED_TEST_SHAPE": "auto"}, cwd="/tmp")
    assert res.returncode == 0, res.stdout + res.stderr
    reb = [x for x in _shapes(res.stdout) if x[0] == "rebuild"]
    assert reb and all(x[1] == "reduce" for x in reb), reb
    _, _, gb, rb = reb[0]
    assert gb == 2.5 * rb, (gb, rb)


@pytest.mark.parametrize("seed", range(16))
def test_reduce_shape_random(oracle, seed):
    """Seeded random shapes, erasures, chunks, worlds 2..8 and placements
    through the partial-sum shape (odd seeds forced, even seeds AUTO) against
    the oracle. A forced plan whose partial sums do not fit the gathered
    slabs must fail on every process with that reason, not hang."""
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    import numpy as np

    rng = np.random.default_rng(9100 + seed)
    np_ = int(rng.integers(2, 9))
    p = int(rng.integers(2, 24))
    e = int(rng.integers(1, min(p - 1, 6) + 1))
    chunk = int(rng.choice([1, 255, 256, 257, int(rng.integers(2, 5000))]))
    m = int(rng.integers(1, e + 1))
    lost = sorted(rng.choice(p, size=m, replace=False).tolist())
    shape = "reduce" if seed % 2 else "auto"
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, str(p), str(e), str(chunk)] + [str(x) for x in lost]
    env = {**os.environ, "SHARDED_TEST_SEED": str(seed), "SHARDED_TEST_SHAPE": shape}
    res = run_group(cmd, 120, env=env, cwd="/tmp")
    if res.returncode != 0 and shape == "reduce" and res.stderr.count("do not fit the gathered slabs") == np_:
        return
    assert res.returncode == 0, (np_, p, e, chunk, lost, res.stdout + res.stderr)
    assert res.stdout.count("rebuild gather") == np_


def test_reduce_shape_compute_failure_keeps_the_exchange_going():
    """A process whose combines fail still runs the partial-sum exchange its
    peers wait in; every process returns and the AND fails."""
    if not _have():
        pytest.skip("needs MPICH (mpirun) and libredset_hip_mpi.so")
    cmd = [MPIRUN, "-np", "3", "-host", "localhost", DRIVER, "11", "3", "5000"]
    env = {**os.environ, "SHARDED_TEST_FAIL_COMPUTE": "1", "SHARDED_TEST_SHAPE": "reduce"}
    res = run_group(cmd, 60, env=env, cwd="/tmp")
    assert res.returncode != 0, res.stdout + res.stderr
    assert "rank 1: encode:" in res.stderr and "combine callback failed" in res.stderr, res.stderr


# ---- the RCCL transport at world > 1, over the test stand-in -------------

HIPSTUB = os.path.join(ROOT, "tests", "mpi", "build", "libhipstub.so")
RCCLSTUB_DIR = os.path.join(ROOT, "tests", "rcclstub", "lib")


@pytest.mark.parametrize("shape", ["gather", "reduce"])
@pytest.mark.parametrize("scheme,np_,p,e,chunk,lost", [
    ("rs", 2, 11, 3, 30001, [1, 2]), ("rs", 3, 11, 3, 4096, [1, 2]), ("rs", 4, 6, 2, 999, [0, 5]),
    ("xor", 3, 8, 1, 3001, [3])])
def test_rccl_transport_at_world_above_one_on_cpu(oracle, shape, scheme, np_, p, e, chunk, lost):
    """transport_rccl.c (grouped ncclSend / ncclRecv, local copies) at world
    2-4, on the CPU: tests/rcclstub's librccl.so.1 moves the messages through
    shared memory and tests/mpi/hipstub.c stands in for the HIP runtime, so
    the transport's grouping, peer matching and message lengths are checked
    against the oracle here; tests/test_gpu_rccl_stub.py runs the same on
    the GPU."""
    if not _have() or not os.path.exists(os.path.join(RCCLSTUB_DIR, "librccl.so.1")) or not os.path.exists(HIPSTUB):
        pytest.skip("needs MPICH, tests/rcclstub and tests/mpi/build/libhipstub.so")
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", "-genv", "LD_PRELOAD", HIPSTUB, DRIVER, str(p), str(e),
           str(chunk)] + [str(x) for x in lost]
    ld = os.environ.get("LD_LIBRARY_PATH")
    env = {**os.environ, "SHARDED_TEST_TRANSPORT": "rccl", "SHARDED_TEST_SHAPE": shape,
           "LD_LIBRARY_PATH": RCCLSTUB_DIR + (":" + ld if ld else "")}
    if scheme == "xor":
        env["SHARDED_TEST_SCHEME"] = "xor"
    before = stub_shm()
    res = run_group(cmd, 120, env=env, cwd="/tmp")
    if res.returncode != 0 and shape == "reduce" and "do not fit" in res.stderr:
        pytest.skip("the partial sums do not fit this placement's scratch")
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == np_
    assert not leaked_stub_shm(before), "stand-in left shared memory"


@pytest.mark.parametrize("transport", ["mpi", "rccl"])
@pytest.mark.parametrize("shape", ["gather", "reduce", "auto"])
@pytest.mark.parametrize("mode", ["--gpu", "--gpu-host"])
@pytest.mark.parametrize("scheme,np_,p,e,chunk,lost", [("rs", 3, 11, 3, 30001, [1, 2]), ("rs", 2, 20, 4, 4097, [0, 5, 19]),
                                                        ("xor", 3, 8, 1, 3001, [3])])
def test_hip_plan_paths_on_cpu(oracle, transport, shape, mode, scheme, np_, p, e, chunk, lost):
    """sharded_test's HIP modes with tests/mpi/hipstub.c standing in for the
    runtime and the plans (the set plans and, round 6, redset_hip_plan_combine):
    the pipelined executes of both shapes -- the plan's exchange stream and
    events, set k's exchange after its compute, the partial sums' accumulate
    after its exchange -- over the MPI transport with device staging (--gpu)
    or host slabs, and over the RCCL transport (tests/rcclstub), against the
    oracle. The GPU suite runs the same with the real kernels."""
    if not _have() or not os.path.exists(HIPSTUB) or not os.path.exists(os.path.join(RCCLSTUB_DIR, "librccl.so.1")):
        pytest.skip("needs MPICH, tests/mpi/build/libhipstub.so and tests/rcclstub")
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", "-genv", "LD_PRELOAD", HIPSTUB, DRIVER, mode, str(p), str(e),
           str(chunk)] + [str(x) for x in lost]
    ld = os.environ.get("LD_LIBRARY_PATH")
    env = {**os.environ, "SHARDED_TEST_TRANSPORT": transport, "SHARDED_TEST_SHAPE": shape,
           "LD_LIBRARY_PATH": RCCLSTUB_DIR + (":" + ld if ld else "")}
    if scheme == "xor":
        env["SHARDED_TEST_SCHEME"] = "xor"
    res = run_group(cmd, 120, env=env, cwd="/tmp")
    if res.returncode != 0 and shape == "reduce" and "do not fit" in res.stderr:
        pytest.skip("the partial sums do not fit this placement's scratch")
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == np_
    if shape != "auto":
        assert res.stdout.count(f"rebuild shape {shape}") == np_, res.stdout


TWIN_DIR = os.path.join(ROOT, "redset_amd", "lib_test")


@pytest.mark.parametrize("direct", [0, 1])
@pytest.mark.parametrize("stand_in", [False, True])
@pytest.mark.parametrize("scheme,np_,p,e,chunk,lost", [("rs", 2, 11, 3, 30001, [1, 2]), ("rs", 3, 11, 3, 4096, [1, 2]),
                                                        ("rs", 3, 12, 4, 777, [1, 2, 3]), ("xor", 3, 8, 1, 3001, [3])])
def test_reduce_shape_both_allocations(oracle, direct, stand_in, scheme, np_, p, e, chunk, lost):
    """The partial-sum shape's two row allocations (sharded.c ra_build):
    fused -- an output's host folds its own inputs in with the partials it
    makes and receives every partial into scratch -- and direct -- the first
    remote partial lands in the output, the host's own share is combined
    after the exchange (less scratch). The planner takes fused where it
    fits; the test twin's REDSET_HIP_TEST_REDUCE_DIRECT forces direct. Both
    against the oracle, with the oracle's combine callback and (stand_in)
    with the HIP combine plans on the CPU stand-in."""
    if not _have() or not os.path.exists(os.path.join(TWIN_DIR, "libredset_hip.so")):
        pytest.skip("needs MPICH and the test twin")
    pre = ["-genv", "LD_PRELOAD", HIPSTUB] if stand_in else []
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost"] + pre + [DRIVER] + (["--gpu"] if stand_in else []) + \
        [str(p), str(e), str(chunk)] + [str(x) for x in lost]
    ld = os.environ.get("LD_LIBRARY_PATH")
    env = {**os.environ, "SHARDED_TEST_SHAPE": "reduce", "LD_LIBRARY_PATH": TWIN_DIR + (":" + ld if ld else "")}
    if direct:
        env["REDSET_HIP_TEST_REDUCE_DIRECT"] = "1"
    if scheme == "xor":
        env["SHARDED_TEST_SCHEME"] = "xor"
    res = run_group(cmd, 120, env=env, cwd="/tmp")
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == np_
    assert res.stdout.count(f"rebuild shape reduce") == np_, res.stdout
    assert f"fused {1 - direct}" in res.stdout, res.stdout
