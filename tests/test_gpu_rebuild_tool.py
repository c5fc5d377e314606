"""GPU tests of the single-process offline rebuild tool (redset_amd/bin/
redset_hip_rebuild; the job of redset_rebuild_rs / redset_rebuild_xor,
src/redset_reedsolomon_serial.c:345-693, src/redset_xor_serial.c:277-622).
A set's files and redundancy files are written from oracle parity, some
members' files are deleted, the tool detects and rebuilds them, and the
rebuilt files must match byte for byte (CRC32 as in test/test_redset.c).
Includes BASELINE.json configs[0]'s shape: XOR, 4 ranks, one 16 MiB file each."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# REDSET_HIP_REBUILD_TOOL: another build of the tool (tools/gpu_asan.sh runs
# the host-ASan one from tests/asan)
TOOL = os.environ.get("REDSET_HIP_REBUILD_TOOL") or os.path.join(ROOT, "redset_amd", "bin", "redset_hip_rebuild")


def _need():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    if not os.path.exists(TOOL):
        pytest.skip("redset_hip_rebuild not built")


def _write_set(tmp, oracle, scheme, p, e, sizes, seed):
    rng = np.random.default_rng(seed)
    d = p - e
    files = []
    for r in range(p):
        fl = []
        for k, size in enumerate(sizes[r]):
            path = os.path.join(tmp, f"rank{r}_file{k}.dat")
            rng.integers(0, 256, size, dtype=np.uint8).tofile(path)
            fl.append((path, size))
        files.append(fl)
    max_bytes = max(sum(s for _, s in fl) for fl in files)
    chunk = max(1, -(-max_bytes // d))  # src/redset_reedsolomon.c:485-493, src/redset_xor.c:362-365
    lofi = []
    for fl in files:
        cat = np.concatenate([np.fromfile(pth, dtype=np.uint8) for pth, _ in fl])
        lf = np.zeros(d * chunk, np.uint8)
        lf[:cat.size] = cat
        lofi.append(lf)
    par = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    if scheme == "rs":
        oracle.OracleRS(p, e).encode_set(lofi, par, chunk)
    else:
        oracle.xor_encode_set(p, lofi, par, chunk)
    reds, headers = [], []
    for r in range(p):
        hdr = bytes([0x40 + r]) * (512 + 64 * r)
        red = os.path.join(tmp, f"rank{r}.{scheme}.redset")
        with open(red, "wb") as f:
            f.write(hdr)
            f.write(par[r].tobytes())
        with open(os.path.join(tmp, f"header_{r}.bin"), "wb") as f:
            f.write(hdr)
        reds.append(red)
        headers.append(len(hdr))
        with open(os.path.join(tmp, f"manifest_{r}.txt"), "w") as f:
            f.write(f"{len(files[r])}\n")
            for pth, size in files[r]:
                f.write(f"{pth} {size}\n")
            f.write(f"{chunk}\n{len(hdr)}\n{red}\n")
    return files, reds


def _crcs(oracle, paths):
    return {p: oracle.crc32(np.fromfile(p, dtype=np.uint8)) for p in paths}


@pytest.mark.parametrize("scheme,p,e,lost,sizes", [
    ("xor", 4, 1, [2], [[16 << 20]] * 4),                               # configs[0]
    ("rs", 6, 2, [0, 4], [[300_000, 77], [1], [250_000], [0, 123_456], [199_999, 5, 60_000], [4096]]),
    ("rs", 11, 3, [1, 2, 9], [[1 << 20]] * 11),
])
def test_offline_rebuild(oracle, tmp_path, scheme, p, e, lost, sizes):
    _need()
    tmp = str(tmp_path)
    files, reds = _write_set(tmp, oracle, scheme, p, e, sizes, seed=p * 7 + e)
    allpaths = [pth for fl in files for pth, _ in fl] + reds
    want = _crcs(oracle, allpaths)
    # nothing missing: no-op
    res = subprocess.run([TOOL, scheme, str(p), str(e), tmp], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    assert json.loads(res.stdout)["missing"] == []
    for r in lost:
        for pth, _ in files[r]:
            os.unlink(pth)
        os.unlink(reds[r])
    res = subprocess.run([TOOL, scheme, str(p), str(e), tmp], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    out = json.loads(res.stdout)
    assert out["missing"] == sorted(lost) and out["ok"]
    assert _crcs(oracle, allpaths) == want


def test_offline_rebuild_too_many_missing(oracle, tmp_path):
    _need()
    tmp = str(tmp_path)
    files, reds = _write_set(tmp, oracle, "rs", 5, 2, [[10_000]] * 5, seed=3)
    for r in (0, 1, 2):
        os.unlink(reds[r])
    res = subprocess.run([TOOL, "rs", "5", "2", tmp], capture_output=True, text=True, timeout=300)
    assert res.returncode != 0 and "tolerates" in res.stderr
    assert "Sanitizer" not in res.stderr, res.stderr[-4000:]  # tools/gpu_asan.sh builds
