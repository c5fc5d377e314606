#!/usr/bin/env python3
"""Kernel access to page-locked host memory over PCIe ("zero copy") vs the
SDMA copies the streaming pipeline uses: gf_mac<8,3> with its 8 inputs
and/or 3 outputs in pinned host memory (the same pointers, mapped into the
GPU's address space by hipHostMalloc), event-timed; and hipMemcpyAsync H2D /
D2H rates of the same bytes for comparison. GB/s = the bytes crossing PCIe."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import redset_amd  # noqa: E402

MIB = 1 << 20


def timeit(fn, reps=5):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    n = int(sys.argv[1]) * MIB if len(sys.argv) > 1 else 256 * MIB
    coef = np.random.default_rng(1).integers(1, 256, (3, 8), dtype=np.uint8)
    h_in = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(8)]
    h_out = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
    for t in h_in:
        t.copy_(torch.randint(0, 256, (n,), dtype=torch.uint8))
    d_in = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(8)]
    d_out = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(3)]
    res = {"cell_MiB": n // MIB}
    # 1. kernel reads host, writes device
    t = timeit(lambda: redset_amd.gf_combine([x.data_ptr() for x in h_in], d_out, coef, n))
    res["kernel_read_host_GBps"] = round(8 * n / t / 1e9, 1)
    # 2. kernel reads device, writes host
    t = timeit(lambda: redset_amd.gf_combine(d_in, [x.data_ptr() for x in h_out], coef, n))
    res["kernel_write_host_GBps"] = round(3 * n / t / 1e9, 1)
    # 3. both: the whole stripe in host memory
    t = timeit(lambda: redset_amd.gf_combine([x.data_ptr() for x in h_in], [x.data_ptr() for x in h_out], coef, n))
    res["kernel_host_to_host_GBps"] = round(11 * n / t / 1e9, 1)
    # parity of the zero-copy result equals the device-resident one
    for a, b in zip(d_in, h_in):
        a.copy_(b)
    redset_amd.gf_combine(d_in, d_out, coef, n)
    torch.cuda.synchronize()
    res["bit_exact"] = all(torch.equal(a.cpu(), b) for a, b in zip(d_out, h_out))
    # 4. SDMA copies of the same bytes (one stream)
    t = timeit(lambda: [d.copy_(h, non_blocking=True) for d, h in zip(d_in, h_in)])
    res["sdma_h2d_GBps"] = round(8 * n / t / 1e9, 1)
    t = timeit(lambda: [h.copy_(d, non_blocking=True) for d, h in zip(d_out, h_out)])
    res["sdma_d2h_GBps"] = round(3 * n / t / 1e9, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
