#!/usr/bin/env python3
"""gf_mac<8,3> rate vs cell size (one stripe per launch, event-timed on the
launch stream): how much of a 64 MiB launch is ramp-up and drain."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import numpy as np  # noqa: E402
import redset_amd  # noqa: E402

MIB = 1 << 20
coef = np.random.default_rng(1).integers(1, 256, (3, 8), dtype=np.uint8)
s = torch.cuda.current_stream()
for mib in [8, 16, 32, 64, 128, 256, 512]:
    n = mib * MIB
    pad = 16 * MIB
    buf = torch.empty(11 * (n + pad), dtype=torch.uint8, device="cuda")
    buf.random_(0, 256)
    cells = [buf[i * (n + pad): i * (n + pad) + n] for i in range(11)]
    ins, outs = cells[:8], cells[8:]
    for _ in range(5):
        redset_amd.gf_combine(ins, outs, coef, n)
    reps = max(5, int(2048 // mib))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        redset_amd.gf_combine(ins, outs, coef, n)
    e1.record(s)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    print(json.dumps({"cell_mib": mib, "us_per_launch": round(t * 1e6, 1), "GBps": round(11 * n / t / 1e9, 1)}), flush=True)
    del buf, cells, ins, outs
