#!/usr/bin/env python3
"""gf_combine of 8 inputs into 1..4 outputs (64 MiB cells, one launch = one
stripe, as the plans run them): GB/s per output count, to separate the cost
of the output count from the cells a rebuild happens to read."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import redset_amd  # noqa: E402

C = 64 << 20
PAD = 16 << 20
redset_amd.load()
arena = torch.empty(12 * (C + PAD), dtype=torch.uint8, device="cuda")
arena.random_(0, 256)
cells = [arena[i * (C + PAD): i * (C + PAD) + C] for i in range(12)]
ins, outs = cells[:8], cells[8:]
rng = np.random.default_rng(1)
s = torch.cuda.current_stream()
res = {}
for rnd in range(3):
    for nout in (1, 2, 3, 4):
        coef = rng.integers(1, 256, (nout, 8), dtype=np.uint8)
        for _ in range(3):
            redset_amd.gf_combine(ins, outs[:nout], coef, C, stream=s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            redset_amd.gf_combine(ins, outs[:nout], coef, C, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        gbps = (8 + nout) * C * 20 / (e0.elapsed_time(e1) * 1e-3) / 1e9
        res.setdefault(nout, []).append(round(gbps, 1))
print(json.dumps({f"nout={k}": v for k, v in res.items()}))
