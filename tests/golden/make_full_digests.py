"""Regenerate tests/golden/full_size_digests.json (from the repo root:
``python tests/golden/make_full_digests.py``; ~10 GB of host memory, a few
minutes).

The CPU oracle (oracle/redset_oracle.c, pinned as described in make_golden.py)
encodes the full-size sets of tests/full_size.py -- BASELINE.json configs[1]
and configs[2] at their own 64 MiB chunks -- and the SHA-256 of every
member's logical file and parity region is recorded. The GPU test
tests/test_gpu_full_digests.py regenerates the same inputs and requires the
HIP path's parity, and the cells its rebuild restores, to hash the same.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import full_size  # noqa: E402
import oracle_lib  # noqa: E402


def main():
    oracle_lib.build()
    out = {}
    for name, case in full_size.CASES.items():
        t0 = time.time()
        p, e, C = case["ranks"], case["encoding"], case["chunk"]
        lofi = [full_size.member_lofi(case, r) for r in range(p)]
        parity = [np.zeros(e * C, np.uint8) for _ in range(p)]
        if case["kind"] == "rs":
            oracle_lib.OracleRS(p, e).encode_set(lofi, parity, C)
        else:
            oracle_lib.xor_encode_set(p, lofi, parity, C)
        out[name] = dict(case, numpy=np.__version__, generator="numpy PCG64([seed, member]).bytes(data_cells * chunk)",
                         lofi_sha256=[full_size.sha256(x) for x in lofi],
                         parity_sha256=[full_size.sha256(x) for x in parity])
        print(f"{name}: {time.time() - t0:.1f} s", flush=True)
        del lofi, parity
    with open(os.path.join(HERE, "full_size_digests.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote full_size_digests.json")


if __name__ == "__main__":
    main()
