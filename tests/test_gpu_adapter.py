"""The reference-signature backend slot, executed.

integration/redset_hip_backend.c holds the four functions a redset build
calls for REDSET_ENCODE=HIP, with exactly the signatures of the CUDA ones
(src/redset_internal.h:345-381). tests/adapter/adapter_test.c links them
into a driver that calls them as redset's scheme drivers do, with redset's
own redset_base / redset_reedsolomon / redset_lofi types, under mpirun on
the box's GPU (every rank shares it). The logical-file reads and writes go
through the adapter's lofi mapping (segment index * chunk_size + offset ->
redset_lofi_pread / pwrite, src/redset_lofi.c:424-451), restated test-only
in the driver with the reference's padding rules. The parity after each
header and the rebuilt files are compared with the oracle.

The driver is built where the reference's headers exist (this container,
tests/adapter/Makefile) and travels to the GPU box prebuilt.
"""
import os

import numpy as np
import pytest

from proc import run_group
from test_gpu_mpi import MPIRUN, _have, _logical, _manifests, _setup

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "adapter", "build", "adapter_test")


def _run(np_, args, env=None, timeout=240):
    cmd = [MPIRUN, "-np", str(np_), "-host", "localhost", DRIVER] + [str(a) for a in args]
    return run_group(cmd, timeout, env={**os.environ, **(env or {})})


def _need():
    if not _have():
        pytest.skip("needs a GPU and MPICH")
    assert os.path.exists(DRIVER), f"{DRIVER} missing: build it with `make -C tests/adapter` (needs the reference headers)"


@pytest.mark.parametrize("exchange", ["auto", "sharded-mpi", "sharded-host"])
@pytest.mark.parametrize("scheme,p,e,lost,buf,repeat", [
    ("rs", 4, 2, [1, 2], 65536, 1),
    ("rs", 4, 2, [0, 3], 1 << 20, 2),   # the second call reuses the adapter's cached codec
    ("rs", 6, 3, [0, 2, 5], 40000, 1),
    ("xor", 4, 1, [2], 50000, 1),
    ("xor", 5, 1, [0], 1 << 20, 2),
])
def test_adapter_slot_encode_and_rebuild(oracle, tmp_path, scheme, p, e, lost, buf, repeat, exchange):
    """Encode, lose members, rebuild through the reference-signature slot.
    exchange "auto": on the box's one GPU the members share a device, so the
    rebuild takes the host-MPI path (and an RS encode with e >= 2 the host
    slabs); "sharded-mpi": the path redset_recover() takes when every member
    owns a GPU -- the sharded plan (column slices gathered onto every GPU,
    gf_mac, rebuilt slices returned) -- over the MPI transport with device
    buffers in place of RCCL (RCCL needs one GPU per rank); "sharded-host":
    the same plan over slabs in page-locked host memory."""
    _need()
    tmp = str(tmp_path)
    d = p - e
    rng = np.random.default_rng(p * 100 + e * 10 + len(lost))
    files, chunk = _setup(tmp, p, d, rng, 300_000)
    header = [512 + 13 * r for r in range(p)]
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    crcs = {path: oracle.crc32(np.fromfile(path, dtype=np.uint8)) for fl in files for path, _ in fl}
    env = {"ADAPTER_TEST_REPEAT": str(repeat), "ADAPTER_TEST_EXCHANGE": exchange}

    res = _run(p, [scheme, "encode", e, tmp, buf], env)
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
        assert np.array_equal(blob[header[r]:], want[r]), r

    # lose members: data files and redundancy file gone (test_redset.c's fault injection)
    for r in lost:
        for path, _ in files[r]:
            os.unlink(path)
        os.unlink(reds[r])
    res = _run(p, [scheme, "rebuild", e, tmp, buf] + lost, env)
    assert res.returncode == 0, res.stdout + res.stderr
    assert f"rebuild exchange {'host' if exchange == 'auto' else exchange}" in res.stdout, res.stdout
    for r in lost:
        for path, size in files[r]:
            assert os.path.getsize(path) == size
            assert oracle.crc32(np.fromfile(path, dtype=np.uint8)) == crcs[path], path
        blob = np.fromfile(reds[r], dtype=np.uint8)
        assert np.array_equal(blob[header[r]:header[r] + e * chunk], want[r]), r


@pytest.mark.parametrize("exchange", ["auto", "sharded-mpi"])
@pytest.mark.parametrize("scheme", ["rs", "xor"])
def test_adapter_short_survivor_file_fails_every_rank(oracle, tmp_path, scheme, exchange):
    """A survivor's data file shorter than its recorded size makes
    redset_lofi_pread fail (as redset_read_attempt's short read does,
    src/redset_lofi.c:74-77); through the adapter that member's slot returns
    REDSET_FAILURE, the collective loop keeps going, and the AND-reduce fails
    every rank with no hang."""
    _need()
    tmp = str(tmp_path)
    p, e = (4, 2) if scheme == "rs" else (4, 1)
    d = p - e
    rng = np.random.default_rng(77)
    files, chunk = _setup(tmp, p, d, rng, 200_000)
    header = [256] * p
    reds = [os.path.join(tmp, f"r{r}.{scheme}.redset") for r in range(p)]
    _manifests(tmp, files, chunk, header, reds)
    res = _run(p, [scheme, "encode", e, tmp, 65536])
    assert res.returncode == 0, res.stdout + res.stderr
    lost = [1]
    for path, _ in files[1]:
        os.unlink(path)
    os.unlink(reds[1])
    # the survivor with the most data loses its file contents (sizes on
    # record unchanged), so its reads of every segment it holds come up short
    big = max((r for r in range(p) if r not in lost), key=lambda r: sum(s for _, s in files[r]))
    assert sum(s for _, s in files[big]) > (d - 1) * chunk
    for path, _ in files[big]:
        os.truncate(path, 0)
    res = _run(p, [scheme, "rebuild", e, tmp, 65536] + lost, {"ADAPTER_TEST_EXCHANGE": exchange})
    assert res.returncode != 0
    assert "slot failed" in res.stderr
