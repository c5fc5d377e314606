"""The sharded path's RCCL transport (redset_amd/csrc/transport_rccl.c) at
world > 1 on the one-GPU test box, over tests/rcclstub's librccl.so.1: the
real RCCL refuses two ranks on one device ("Duplicate GPU",
tests/test_gpu_mpi.py::test_mpi_forced_rccl_exchange_on_a_shared_gpu_fails_every_rank),
so before the driver's 8-GPU node these tests are the only execution of the
transport's grouped ncclSend / ncclRecv, its local copies, the per-rank
slot's cached RCCL communicator (rank_mpi.c rccl_create, forced
_SHARDED_RCCL) and dist.py's RcclTransport beyond world 1. The stand-in moves
the bytes through shared memory with hipMemcpy and accepts any number of
ranks per GPU; the HIP kernels, plans, streams and the transport code are
the product's. Everything is checked against the CPU oracle.

The C drivers find the stand-in through LD_LIBRARY_PATH (transport_rccl.c
dlopens "librccl.so.1"); a torch process has already mapped torch's real
librccl.so.1, so dist.py's runner loads it by path through the test twin's
REDSET_HIP_TEST_RCCL_LIBRARY (the product library reads no such variable).
Replaces, in the reference: the decode ring and gather of
src/redset_reedsolomon.c:690-699 and :713-733."""
import json
import os
import tempfile

import numpy as np
import pytest

from proc import leaked_stub_shm, run_group, stub_shm
from test_gpu_mpi import MPIRUN, _have, _logical, _manifests, _mpirun, _setup

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB_DIR = os.path.join(ROOT, "tests", "rcclstub", "lib")
STUB = os.path.join(STUB_DIR, "librccl.so.1")
TWIN = os.path.join(ROOT, "redset_amd", "lib_test", "libredset_hip.so")
# SHARDED_TEST_BIN: another build of the driver (tools/gpu_asan.sh: host ASan)
DRIVER = os.environ.get("SHARDED_TEST_BIN") or os.path.join(ROOT, "tests", "mpi", "build", "sharded_test")


def _stub_env(extra=None):
    ld = os.environ.get("LD_LIBRARY_PATH")
    env = {"LD_LIBRARY_PATH": STUB_DIR + (":" + ld if ld else "")}
    env.update(extra or {})
    return env


_before = set()


@pytest.fixture(autouse=True)
def _shm_snapshot():
    global _before
    _before = stub_shm()
    yield


def _no_leftover_shm():
    return not leaked_stub_shm(_before)


def _need():
    if not _have() or not os.path.exists(DRIVER):
        pytest.skip("needs a GPU, MPICH and tests/mpi/build")
    if not os.path.exists(STUB):
        pytest.skip("tests/rcclstub not built (make -C tests/rcclstub)")


@pytest.mark.parametrize("shape", ["gather", "reduce"])
@pytest.mark.parametrize("np_,p,e,chunk,lost", [(2, 11, 3, 300_001, [1, 2]), (3, 11, 3, 65536, [1, 2]),
                                                 (4, 6, 2, 99_999, [0, 5]), (2, 20, 4, 65536, [0, 5, 19])])
def test_sharded_rccl_transport_with_hip_kernels(shape, np_, p, e, chunk, lost):
    """tests/mpi/sharded_test.c --gpu over the RCCL transport: slabs in HBM,
    the gf_mac plans (gather shape) or the combine plans (partial-sum shape),
    the exchanges as grouped ncclSend / ncclRecv on the plan's exchange
    stream. Hosted parity and rebuilt members against the oracle."""
    _need()
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, "--gpu", str(p), str(e), str(chunk)] + \
        [str(x) for x in lost]
    res = run_group(cmd, 120, env={**os.environ, **_stub_env({"SHARDED_TEST_TRANSPORT": "rccl",
                                                               "SHARDED_TEST_SHAPE": shape})})
    if res.returncode != 0 and shape == "reduce" and res.stderr.count("do not fit") == np_:
        pytest.skip("the partial sums do not fit this placement's scratch")
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == np_
    assert res.stdout.count(f"rebuild shape {shape}") == np_, res.stdout
    assert _no_leftover_shm()


@pytest.mark.parametrize("alloc", ["planner", "direct"])
@pytest.mark.parametrize("mode", ["--gpu", "--gpu-host"])
@pytest.mark.parametrize("np_,p,e,chunk,lost,scheme", [(2, 11, 3, 300_001, [1, 2], "rs"), (3, 6, 2, 40_000, [0, 4], "rs"),
                                                        (3, 8, 1, 65536, [3], "xor")])
def test_sharded_reduce_shape_over_mpi(alloc, mode, np_, p, e, chunk, lost, scheme):
    """The partial-sum shape with the HIP combine plans (redset_hip_plan_combine)
    over the MPI transport: slabs in HBM (staged through pinned memory) or in
    page-locked host memory that the combines read and write in place; both
    row allocations (fused: the product's choice where it fits; direct:
    forced through the test twin's REDSET_HIP_TEST_REDUCE_DIRECT)."""
    _need()
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER, mode, str(p), str(e), str(chunk)] + \
        [str(x) for x in lost]
    env = {**os.environ, "SHARDED_TEST_SHAPE": "reduce"}
    if alloc == "direct":
        ld = os.environ.get("LD_LIBRARY_PATH")
        env["LD_LIBRARY_PATH"] = os.path.dirname(TWIN) + (":" + ld if ld else "")
        env["REDSET_HIP_TEST_REDUCE_DIRECT"] = "1"
    if scheme == "xor":
        env["SHARDED_TEST_SCHEME"] = "xor"
    res = run_group(cmd, 120, env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild shape reduce") == np_, res.stdout
    if alloc == "direct":
        assert "fused 0" in res.stdout and "fused 1" not in res.stdout, res.stdout
    # (the product's choice: fused where it fits -- (2, 11, 3) and the XOR set
    # here -- else direct, as (3, 6, 2)'s scratch allows only the direct rows)


def test_sharded_rccl_transport_xor():
    _need()
    cmd = [MPIRUN, "-np", "3", "-host", "localhost", DRIVER, "--gpu", "8", "1", "200001", "3"]
    res = run_group(cmd, 120, env={**os.environ, **_stub_env({"SHARDED_TEST_TRANSPORT": "rccl",
                                                               "SHARDED_TEST_SHAPE": "auto",
                                                               "SHARDED_TEST_SCHEME": "xor"})})
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("rebuild gather") == 3


@pytest.mark.parametrize("scheme,p,e,lost", [("rs", 6, 2, [1, 4]), ("rs", 5, 3, [0, 2, 4]), ("xor", 4, 1, [2])])
def test_rank_backends_forced_rccl(oracle, tmp_path, scheme, p, e, lost):
    """The drop-in slot with redset_hip_rank_set_exchange(SHARDED_RCCL): the
    communicator's RCCL transport is created once (rank_mpi.c rccl_create,
    unique id by MPI_Bcast) and cached on the communicator; the encode and
    the rebuild run the sharded slot over it, three calls per process
    (RANK_TEST_REPEAT) so the cached communicator and slot context are
    reused. Parity after the header against the oracle, rebuilt files by
    CRC32 (test/test_redset.c:459-589)."""
    _need()
    tmp = str(tmp_path)
    d = p - e
    rng = np.random.default_rng(600 + p)
    files, chunk = _setup(tmp, p, d, rng, 300_000)
    header = [777] * p
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for fl in files for path, _ in fl}
    env = _stub_env({"RANK_TEST_EXCHANGE": "rccl", "RANK_TEST_REPEAT": "3"})
    res = _mpirun(p, [scheme, "encode", e, tmp, 65536], env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "encode exchange rccl" in res.stdout, res.stdout
    lofi = [_logical(fl, d * chunk) for fl in files]
    want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    if scheme == "rs":
        oracle.OracleRS(p, e).encode_set(lofi, want, chunk)
    else:
        oracle.xor_encode_set(p, lofi, want, chunk)
    for r in range(p):
        assert np.array_equal(np.fromfile(reds[r], dtype=np.uint8)[header[r]:], want[r]), r
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    res = _mpirun(p, [scheme, "rebuild", e, tmp, 65536] + lost, env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "rebuild exchange rccl" in res.stdout, res.stdout
    for r in lost:
        for path, size in files[r]:
            assert os.path.getsize(path) == size
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
        blob = np.fromfile(reds[r], dtype=np.uint8)
        assert np.array_equal(blob[header[r]:header[r] + e * chunk], want[r]), r
    assert _no_leftover_shm()


def _dist_worker(rank, world, port, p, e, chunk, lost, shape, outdir):
    import sys

    sys.path.insert(0, ROOT)
    # the twin honours REDSET_HIP_TEST_RCCL_LIBRARY (torch has mapped the
    # real librccl.so.1 in this process); set before redset_amd loads it
    os.environ["REDSET_HIP_LIBRARY"] = TWIN
    os.environ["REDSET_HIP_TEST_RCCL_LIBRARY"] = STUB
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import redset_amd
    from redset_amd.dist import RcclTransport, ShardedSetRunner

    runner = ShardedSetRunner(p, e, chunk, lost, world=world, rank=rank, device="cuda:0", backend=None,
                              seed=11, transport="rccl", shape=shape)
    assert isinstance(runner._transport, RcclTransport)
    save = lambda name, t: np.save(os.path.join(outdir, f"{name}_{rank}.npy"), t.cpu().numpy())
    if rank == 0:
        with open(os.path.join(outdir, "where.json"), "w") as f:
            json.dump({str(m): list(v) for m, v in runner._where.items()}, f)
    save("data", runner.D_host)
    runner.encode()
    torch.cuda.synchronize()
    save("par", runner.P_host)
    snap = runner.lost_snapshot()
    runner.erase()
    runner.D_gath.fill_(0xA5)
    runner.P_gath.fill_(0x5A)
    runner.rebuild()
    torch.cuda.synchronize()
    save("data2", runner.D_host)
    save("par2", runner.P_host)
    hang = ctypes_hang()
    with open(os.path.join(outdir, f"rec_{rank}.json"), "w") as f:
        json.dump({"matches": bool(runner.matches(snap)), "shape": runner.shape("rebuild")["shape"],
                   "hang_faults": hang, "twin": bool(redset_amd._lib.load().redset_hip_test_build())}, f)
    runner.close()
    dist.barrier()
    dist.destroy_process_group()


def ctypes_hang():
    import ctypes

    import redset_amd._lib as L

    c = ctypes.c_uint(0)
    L.load().redset_hip_hang_faults(None, ctypes.byref(c), 0)
    return int(c.value)


@pytest.mark.parametrize("shape", ["gather", "reduce"])
def test_dist_runner_over_rccl_at_world_2(oracle, shape):
    """dist.ShardedSetRunner at world 2 with RcclTransport while the process
    group is gloo (the unique id goes out over gloo): the bench's sharded leg
    at N = 2 as the driver's 8-GPU node will run it, two ranks on this box's
    one GPU. Parity and rebuilt members against the oracle, cell by cell."""
    import torch.multiprocessing as mp

    from test_dist import _assemble, _free_port

    from conftest import gpu_available

    if not gpu_available():
        pytest.skip("needs an MI355X")
    if not os.path.exists(STUB) or not os.path.exists(TWIN):
        pytest.skip("needs tests/rcclstub and the test twin")
    world, p, e, chunk, lost = 2, 11, 3, 65536 + 48, [1, 2]
    port = _free_port()
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_dist_worker, args=(world, port, p, e, chunk, lost, shape, td), nprocs=world, join=True)
        load = lambda name: [np.load(os.path.join(td, f"{name}_{g}.npy")) for g in range(world)]
        data, par, data2, par2 = load("data"), load("par"), load("data2"), load("par2")
        W = data[0].shape[-1]
        with open(os.path.join(td, "where.json")) as f:
            where = json.load(f)
        for g in range(world):
            with open(os.path.join(td, f"rec_{g}.json")) as f:
                rec = json.load(f)
            assert rec["matches"] and rec["twin"] and rec["hang_faults"] == 0, (g, rec)
            assert rec["shape"] == shape, rec
        st = oracle.OracleRS(p, e)
        for k in range(world):
            lofi = [_assemble(data, where, world, p, chunk, W, k, r) for r in range(p)]
            want = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
            st.encode_set(lofi, want, chunk)
            for r in range(p):
                assert np.array_equal(_assemble(par, where, world, p, chunk, W, k, r), want[r]), (k, r)
                assert np.array_equal(_assemble(data2, where, world, p, chunk, W, k, r), lofi[r]), (k, r)
                assert np.array_equal(_assemble(par2, where, world, p, chunk, W, k, r), want[r]), (k, r)
    assert _no_leftover_shm()
