#!/usr/bin/env python3
"""Rebuild rate of every erasure pair of the bench's RS(8+3) 64 MiB set, PASSES
times, to tell a slow pattern from run-to-run noise. Prints the per-pair mean,
min and max, slowest first."""
import itertools
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import redset_amd  # noqa: E402

PASSES = int(sys.argv[1]) if len(sys.argv) > 1 else 3
p, e, chunk = 11, 3, 64 << 20
redset_amd.load()
codec = redset_amd.RSCodec(p, e)
lay = redset_amd.SetLayout.allocate(p, p - e, e, chunk, pad=16 << 20)
lay.storage.random_(0, 256)
s = torch.cuda.current_stream()
codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride).execute(s)
plans = {pr: codec.plan_rebuild(list(pr), lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
         for pr in itertools.combinations(range(p), 2)}
rates = {pr: [] for pr in plans}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(PASSES):
    for pr, plan in plans.items():
        plan.execute(s)
        e0.record(s)
        for _ in range(5):
            plan.execute(s)
        e1.record(s)
        torch.cuda.synchronize()
        rates[pr].append((plan.bytes_read + plan.bytes_written) * 5 / (e0.elapsed_time(e1) * 1e-3) / 1e9)
order = sorted(rates, key=lambda k: sum(rates[k]) / len(rates[k]))
for pr in order[:8] + ["..."] + order[-4:]:
    if pr == "...":
        print("...")
        continue
    v = rates[pr]
    print(f"pair {pr}: mean {sum(v) / len(v):7.1f}  min {min(v):7.1f}  max {max(v):7.1f} GB/s")
