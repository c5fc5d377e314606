"""The GPU suite against the test twin library.

The product library (redset_amd/lib/) reads no environment knob: its job
orders, occupancy and ring constants are fixed (redset_hip.cpp,
codec_device.h). The twin (redset_amd/lib_test/) is the same source built
with -DREDSET_HIP_TEST_KNOBS=1; its planner and launchers honour the knobs
the suite uses to reach paths the product takes only at some sizes or never
on a healthy GPU:

* REDSET_HIP_TEST_SPIN_CAP: the loader ring's poll cap. Every handshake poll
  is bounded; a consumer whose item does not arrive in time loads its bytes
  straight from HBM, and a loader whose slot is not released in time stops
  and raises the block's BYPASS word, so the consumers load every item it
  has not published. The product caps a poll at 2^24 spins, so these paths
  almost never run there; at 4 they run on nearly every launch.
* REDSET_HIP_TEST_CLAIM_DELAY: the claimed kernel's claimer sleeps between
  taking a batch from its queue and recording it, the window in which a
  stopping loader once could end the block's sequence without that batch
  (codec_device.h gf_mac_claimed CLAIMER_DONE).
* REDSET_HIP_TEST_HANG_CAP / _TABLE_DELAY (round 5): the cap of the waits
  with no fallback and a loader that publishes a job's tables late, so the
  hang word (include/redset_hip.h redset_hip_hang_faults) can be made to
  count and the per-rank backends to fail the call
  (tests/test_gpu_hang_contract.py, test_gpu_mpi.py::test_mpi_hang_cap_*).
  In the runs below the hang cap stays at the product's 2^26 polls, and every
  test asserts the hang word is 0.
* REDSET_HIP_SEQUENTIAL / _STREAM_JOBS / _STRIPES_PER_LAUNCH / _XOR_STREAM /
  _ZERO_COPY (tests marked `knobs`): every job order and pipeline mode at
  small sizes.

Two child runs of the suite, each in one process:
1. the kernel-facing GPU tests (TWIN_FILES: every plan order, stripe width
   and cell size against the oracle, the streaming pipeline, full-size
   digests and the hang contract) with a 4-poll cap and a claimer delay: every test
   compares bytes with the oracle or the golden digests, so a fallback that
   dropped or misplaced a byte fails that test; the child reports how many
   capped spins it counted (must be many) and which codec library it mapped.
   The mpirun matrices (per-rank backends, adapter, RCCL stand-in), the doc
   examples, the sharded compute over gloo and the offline tool run the same
   kernels through the same plans, and the twin changes none of their host
   code, so they are not rerun (round 6: the rerun took 256 s of the GPU
   suite's 598);
2. the `knobs` tests with the product's cap, so every forced order also runs
   its normal ring path (no capped spin allowed).
The Python paths load the twin through REDSET_HIP_LIBRARY; the C drivers
(rank_test, sharded_test, redset_hip_rebuild, adapter_test) through
LD_LIBRARY_PATH, which their RUNPATH defers to. The reference's rule this
serves: a backend either returns correct data or REDSET_FAILURE
(src/redset_reedsolomon.c:338-342, :382-387).
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TWIN_DIR = os.path.join(ROOT, "redset_amd", "lib_test")
TWIN = os.path.join(TWIN_DIR, "libredset_hip.so")
SELF = "tests/test_gpu_test_build.py"
# the tests whose kernels the twin's ring and claim knobs change
TWIN_FILES = ("test_gpu_parity.py", "test_gpu_stream.py", "test_gpu_full_digests.py", "test_gpu_hang_contract.py")


def _child(tmp_path, name, extra_env, args, timeout, files=None):
    env = dict(os.environ)
    env.update({
        "REDSET_HIP_LIBRARY": TWIN,
        "LD_LIBRARY_PATH": TWIN_DIR + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else ""),
    })
    env.update(extra_env)
    # the child's report goes to a file as it runs (REDSET_TEST_PROGRESS_DIR, if
    # set, else the test's tmp dir), one line per test, so a long run shows
    # progress to whoever watches that directory
    out_dir = os.environ.get("REDSET_TEST_PROGRESS_DIR") or str(tmp_path)
    os.makedirs(out_dir, exist_ok=True)
    child_log = os.path.join(out_dir, name)
    with open(child_log, "w") as f:
        res = subprocess.run(
            [sys.executable, "-u", "-m", "pytest"] +
            ([os.path.join(ROOT, "tests", f) for f in files] if files else [os.path.join(ROOT, "tests")]) +
            ["-x", "-v",
             "-p", "no:cacheprovider", "--timeout", "300", "--timeout-method", "thread",
             "--deselect", f"{SELF}::test_gpu_suite_bit_exact_with_ring_fallbacks",
             "--deselect", f"{SELF}::test_knob_tests_with_the_normal_ring",
             # bench.py end to end is the product's; its kernels run in this suite anyway
             "--ignore", os.path.join(ROOT, "tests", "test_gpu_bench.py")] + args,
            cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    with open(child_log) as f:
        text = f.read()
    return res, text


@pytest.mark.timeout(1200)
def test_gpu_suite_bit_exact_with_ring_fallbacks(tmp_path):
    from conftest import gpu_available

    if not gpu_available():
        pytest.skip("needs an MI355X")
    assert os.path.exists(TWIN), f"{TWIN} missing: build with `make -C redset_amd/csrc`"
    log = tmp_path / "faults.txt"
    res, text = _child(tmp_path, "test_twin_suite.log", {
        "REDSET_HIP_TEST_SPIN_CAP": "4",
        "REDSET_HIP_TEST_CLAIM_DELAY": "2",
        "REDSET_RING_FALLBACK_RUN": "1",
        "REDSET_RING_FAULT_LOG": str(log),
    }, ["-m", "gpu"], 1100, files=TWIN_FILES)
    assert res.returncode == 0, text[-6000:]
    lines = log.read_text().split()
    faults, libs = int(lines[0]), lines[1:]
    print(f"test twin, 4-poll cap: {faults} capped spins; mapped {libs}; {text.strip().splitlines()[-1]}")
    assert libs == [TWIN], libs
    # thousands of launches, each with a capped handshake or several
    assert faults > 1000, faults
    # the knob tests were collected in the child (the twin was loaded)
    assert "test_plan_job_order" in text, text[-3000:]


@pytest.mark.timeout(600)
def test_knob_tests_with_the_normal_ring(tmp_path):
    """Every forced job order and pipeline mode once more with the product's
    poll cap: the normal ring path of each order, no capped spin allowed."""
    from conftest import gpu_available

    if not gpu_available():
        pytest.skip("needs an MI355X")
    assert os.path.exists(TWIN), f"{TWIN} missing: build with `make -C redset_amd/csrc`"
    res, text = _child(tmp_path, "test_twin_knobs.log", {}, ["-m", "gpu and knobs"], 550)
    assert res.returncode == 0, text[-6000:]
    assert " passed" in text.strip().splitlines()[-1], text[-2000:]
    print(f"test twin, knob tests: {text.strip().splitlines()[-1]}")


def test_product_library_ignores_the_knobs(monkeypatch):
    """The product library's plans do not change with the test knobs set
    (a forced order would change the launch count)."""
    from conftest import gpu_available

    if not gpu_available():
        pytest.skip("needs an MI355X")
    import torch

    import redset_amd
    import redset_amd._lib as L

    if L.load().redset_hip_test_build():
        pytest.skip("this process loaded the test twin")
    p, e, chunk = 11, 3, 40_000
    lay = redset_amd.SetLayout.allocate(p, p - e, e, chunk)
    codec = redset_amd.RSCodec(p, e)
    base = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).launches
    for mode in "1234":
        monkeypatch.setenv("REDSET_HIP_SEQUENTIAL", mode)
        monkeypatch.setenv("REDSET_HIP_STREAM_JOBS", "1")
        assert codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).launches == base
    torch.cuda.synchronize()
