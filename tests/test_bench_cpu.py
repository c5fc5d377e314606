"""bench.py's CPU baseline legs on this container (no GPU): the oracle's port
of the reference's pthreads encode + serial rebuild (RS, XOR) at small
chunks, as the N > 1 rehearsals run them. At 4 MiB chunks the single-thread
multadd sample once read 64 MiB from a 32 MiB source (a crash at N = 4 in
session r06s7); the oracle binding now refuses a short source."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("chunk", [1 << 20])
def test_cpu_baseline_small_chunks(oracle, chunk):
    sys.path.insert(0, ROOT)
    import bench

    r = bench.cpu_baseline(11, 3, [1, 2], 0.1, chunk)
    assert r["round_trip_equal"] is True and r["value"] > 0 and r["kind"] == "port"
    assert r["multadd_1thread_GBps"] > 0.05, r  # a sane single-thread rate, not a page-fault crawl
    x = bench.cpu_baseline_xor(8, 3, 0.1, chunk)
    assert x["round_trip_equal"] is True and x["value"] > 0


def test_oracle_multadd_refuses_a_short_source(oracle):
    st = oracle.OracleRS(4, 2)
    with pytest.raises(ValueError):
        st.multadd(np.zeros(1024, np.uint8), 3, np.zeros(512, np.uint8))
