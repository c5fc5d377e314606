#!/usr/bin/env python3
"""Per-launch encode / rebuild rate over time in one process: does the HBM
rate change with how long the GPU has been streaming (power / clock state)?
usage: time_series.py SECONDS [IDLE_S]  -- stream for SECONDS, idle IDLE_S,
stream again; prints the rate every ~50 ms."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import redset_amd  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
idle = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
kind = sys.argv[3] if len(sys.argv) > 3 else "encode"
p, e, chunk = 11, 3, 64 << 20
redset_amd.load()
codec = redset_amd.RSCodec(p, e)
lay = redset_amd.SetLayout.allocate(p, p - e, e, chunk, pad=16 << 20)
lay.storage.random_(0, 256)
plan = (codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride) if kind == "encode" else
        codec.plan_rebuild([1, 2], lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride))
nbytes = plan.bytes_read + plan.bytes_written
s = torch.cuda.current_stream()
torch.cuda.synchronize()


def burst(label, seconds):
    t0 = time.perf_counter()
    batch = 16
    while time.perf_counter() - t0 < seconds:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(batch + 1)]
        ev[0].record(s)
        for i in range(batch):
            plan.execute(s)
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(batch)]
        print(f"{label} t={time.perf_counter() - t0:6.3f}s  {kind} {nbytes / (sum(ms) / batch) / 1e6:7.1f} GB/s "
              f"(min {nbytes / max(ms) / 1e6:7.1f} max {nbytes / min(ms) / 1e6:7.1f})", flush=True)


burst("A", secs)
time.sleep(idle)
burst("B", secs)
