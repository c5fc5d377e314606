"""The fault contract's second word: kernel waits with no fallback (VERDICT r4
weak item 3, include/redset_hip.h redset_hip_hang_faults).

The streamed and claimed kernels have waits that end by construction -- the
loader's hand-over of a job's GF tables, the claimer's records, the loader's
wait for the claimer at a stop. Their cap (2^26 polls) only keeps a bug from
hanging the GPU, and a capped one makes the launch's outputs wrong, so it
counts in the hang word, not in the spin counter whose events are harmless.
These tests run in the test twin (knobs), whose launches take the hang cap
and a loader table delay from the environment, and make those waits give up
on purpose: the hang word must count them, and with the product's cap the
same stalled launches must wait and stay bit-exact. The per-rank backends'
use of the word -- fail the call when it moved -- is tested through mpirun in
tests/test_gpu_mpi.py (test_mpi_hang_cap_fails_the_call) and on the CPU in
tests/test_mpi_hoststub.py. The rule served: a backend returns correct bytes
or REDSET_FAILURE (src/redset_reedsolomon.c:336-341)."""
import numpy as np
import pytest

from test_gpu_parity import download_set, upload_set

pytestmark = [pytest.mark.gpu, pytest.mark.knobs]

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def rd():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import redset_amd

    redset_amd.load()
    assert redset_amd.load().redset_hip_test_build() == 1
    return redset_amd


def _encode(rd, oracle, p, e, chunk, seed, runs=1):
    lofi, parity = oracle.random_set(p, p - e, e, chunk, seed=seed)
    lay = upload_set(rd, lofi, parity, p - e, e, chunk)
    codec = rd.RSCodec(p, e)
    enc = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    for _ in range(runs):
        enc.execute()
    torch.cuda.synchronize()
    oracle.OracleRS(p, e).encode_set(lofi, parity, chunk)
    _, got = download_set(lay)
    return all(np.array_equal(a, b) for a, b in zip(got, parity))


def test_streamed_table_stall_counts_in_the_hang_word(rd, oracle, monkeypatch):
    """Streamed pairs (REDSET_HIP_SEQUENTIAL=3) whose loader sleeps before it
    publishes job 1's tables: with a 1-poll hang cap the consumers stop
    waiting for them (their outputs are then wrong) and the hang word counts
    it; with the product's cap they wait and the parity is bit-exact."""
    monkeypatch.setenv("REDSET_HIP_SEQUENTIAL", "3")
    monkeypatch.setenv("REDSET_HIP_TEST_TABLE_DELAY", "400")
    p, e, chunk = 11, 3, 300_016
    rd.hang_faults()  # start from zero
    monkeypatch.setenv("REDSET_HIP_TEST_HANG_CAP", "1")
    _encode(rd, oracle, p, e, chunk, seed=5)
    hangs = rd.hang_faults()
    assert hangs > 0, "a capped table hand-over was not counted"
    monkeypatch.delenv("REDSET_HIP_TEST_HANG_CAP")
    assert _encode(rd, oracle, p, e, chunk, seed=6, runs=2)
    assert rd.hang_faults() == 0


def test_claimed_stop_counts_in_the_hang_word(rd, oracle, monkeypatch):
    """The claimed order (REDSET_HIP_SEQUENTIAL=4) with a 4-poll spin cap, so
    loaders stop and hand their rows to the consumers, a slow claimer, and a
    1-poll hang cap: the loaders' wait for the claimer and the consumers' wait
    for a claim record give up and are counted. With the product's hang cap
    the same stopped launches are bit-exact."""
    monkeypatch.setenv("REDSET_HIP_SEQUENTIAL", "4")
    monkeypatch.setenv("REDSET_HIP_TEST_SPIN_CAP", "4")
    monkeypatch.setenv("REDSET_HIP_TEST_CLAIM_DELAY", "4")
    p, e, chunk = 11, 3, (4 << 20) + 5 * 1024 + 48
    rd.hang_faults()
    rd.ring_faults()
    monkeypatch.setenv("REDSET_HIP_TEST_HANG_CAP", "1")
    _encode(rd, oracle, p, e, chunk, seed=7)
    assert rd.hang_faults() > 0, "a capped claim wait was not counted"
    monkeypatch.delenv("REDSET_HIP_TEST_HANG_CAP")
    assert _encode(rd, oracle, p, e, chunk, seed=8)
    assert rd.hang_faults() == 0
    rd.ring_faults()  # the 4-poll cap's spins are expected here
