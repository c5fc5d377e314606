"""The loader ring's fallbacks keep every byte right.

The kernels stream their inputs through an LDS ring fed by one loader wave
(redset_amd/csrc/codec_device.h ring_sweep). Every handshake poll is
bounded. A consumer whose item does not arrive in time loads its bytes
straight from HBM; a loader whose slot is not released in time stops and
raises the block's BYPASS word, so the consumers load every item it has not
published. The shipped build caps a poll at 2^24 spins, so these paths
almost never run there. The twin library redset_amd/lib_spincap/ is the same
source built with -DREDSET_RING_SPIN_CAP=4, where both fallbacks run on
nearly every launch.

This test runs the whole GPU suite once more, in a child process, against
that twin. The Python paths load it through REDSET_HIP_LIBRARY; the C
drivers (rank_test, sharded_test, redset_hip_rebuild) load it through
LD_LIBRARY_PATH, which their RUNPATH defers to. Every test compares bytes
with the oracle or the golden digests, so a fallback that dropped or
misplaced a byte fails that test. The child also reports how many capped
spins it counted, which must be many, and which codec library it mapped.
The reference's rule this serves: a backend either returns correct data or
REDSET_FAILURE (src/redset_reedsolomon.c:338-342, :382-387).
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TWIN_DIR = os.path.join(ROOT, "redset_amd", "lib_spincap")
TWIN = os.path.join(TWIN_DIR, "libredset_hip.so")


@pytest.mark.timeout(1200)
def test_gpu_suite_bit_exact_with_ring_fallbacks(tmp_path):
    from conftest import gpu_available

    if not gpu_available():
        pytest.skip("needs an MI355X")
    assert os.path.exists(TWIN), f"{TWIN} missing: build with `make -C redset_amd/csrc`"
    log = tmp_path / "faults.txt"
    env = dict(os.environ)
    env.update({
        "REDSET_HIP_LIBRARY": TWIN,
        "LD_LIBRARY_PATH": TWIN_DIR + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else ""),
        "REDSET_RING_FALLBACK_RUN": "1",
        "REDSET_RING_FAULT_LOG": str(log),
    })
    # the child's report goes to a file as it runs (REDSET_TEST_PROGRESS_DIR, if
    # set, else the test's tmp dir), one line per test, so a long run shows
    # progress to whoever watches that directory
    out_dir = os.environ.get("REDSET_TEST_PROGRESS_DIR") or str(tmp_path)
    os.makedirs(out_dir, exist_ok=True)
    child_log = os.path.join(out_dir, "spincap_twin_suite.log")
    with open(child_log, "w") as f:
        res = subprocess.run(
            [sys.executable, "-u", "-m", "pytest", os.path.join(ROOT, "tests"), "-m", "gpu", "-x", "-v",
             "-p", "no:cacheprovider", "--timeout", "300", "--timeout-method", "thread",
             "--deselect", "tests/test_gpu_ring_fallback.py::test_gpu_suite_bit_exact_with_ring_fallbacks"],
            cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT, text=True, timeout=1150)
    with open(child_log) as f:
        text = f.read()
    assert res.returncode == 0, text[-6000:]
    lines = log.read_text().split()
    faults, libs = int(lines[0]), lines[1:]
    print(f"spin-cap twin: {faults} capped spins; mapped {libs}; {text.strip().splitlines()[-1]}")
    assert libs == [TWIN], libs
    # thousands of launches, each with a capped handshake or several
    assert faults > 1000, faults
