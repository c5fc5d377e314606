"""Full-size workloads of BASELINE.json (configs[1] XOR p=8 and configs[2]
RS(8+3), 64 MiB chunks) with inputs any machine can regenerate: member r's
logical file = numpy PCG64([seed, r]).bytes(d * chunk). The oracle's parity
digests for them are committed in tests/golden/full_size_digests.json
(tests/golden/make_full_digests.py) and checked against the HIP path by
tests/test_gpu_full_digests.py -- bit-exact parity at the benchmark's own
size, without shipping gigabytes of fixtures."""
import hashlib

import numpy as np

MIB = 1 << 20

CASES = {
    # BASELINE.json configs[2]: REDSET_COPY_RS k=8 m=3, 64 MiB chunks (p = 11)
    "rs_p11_e3_c64MiB": {"kind": "rs", "ranks": 11, "encoding": 3, "chunk": 64 * MIB, "seed": 0x5EED,
                         "lost": [1, 2]},
    # BASELINE.json configs[1]: REDSET_COPY_XOR, 8 ranks, 64 MiB chunks
    "xor_p8_c64MiB": {"kind": "xor", "ranks": 8, "encoding": 1, "chunk": 64 * MIB, "seed": 0x5EED + 1,
                      "lost": [3]},
}


def data_cells(case) -> int:
    return case["ranks"] - case["encoding"] if case["kind"] == "rs" else case["ranks"] - 1


def member_lofi(case, r: int) -> np.ndarray:
    """Member r's logical file (data_cells * chunk bytes), writable."""
    n = data_cells(case) * case["chunk"]
    g = np.random.Generator(np.random.PCG64([case["seed"], r]))
    return np.frombuffer(bytearray(g.bytes(n)), dtype=np.uint8)


def sha256(a) -> str:
    return hashlib.sha256(memoryview(np.ascontiguousarray(a))).hexdigest()
