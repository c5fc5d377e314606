#!/usr/bin/env python3
"""PCIe ceilings for the host-resident pipeline (DESIGN.md §5 end-to-end):
pinned host <-> HBM copy rates with 1 and 2 streams per direction, and both
directions at once. One JSON line."""
import json

import torch

N = 1 << 30
REPS = 8
h = [torch.empty(N, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
d = [torch.empty(N, dtype=torch.uint8, device="cuda") for _ in range(2)]
for t in h:
    t.fill_(1)
streams = [torch.cuda.Stream() for _ in range(4)]


def run(jobs):
    """jobs: list of (stream index, dst, src); returns GB/s of all bytes moved"""
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s in streams:
        s.wait_event(e0)
    for _ in range(REPS):
        for si, dst, src in jobs:
            with torch.cuda.stream(streams[si]):
                dst.copy_(src, non_blocking=True)
    for s in streams:
        torch.cuda.current_stream().wait_stream(s)
    e1.record()
    torch.cuda.synchronize()
    moved = REPS * sum(src.numel() for _, _, src in jobs)
    return round(moved / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)


half = N // 2
out = {
    "h2d_1stream": run([(0, d[0], h[0])]),
    "h2d_2streams": run([(0, d[0][:half], h[0][:half]), (1, d[0][half:], h[0][half:])]),
    "d2h_1stream": run([(0, h[1], d[1])]),
    "d2h_2streams": run([(0, h[1][:half], d[1][:half]), (1, h[1][half:], d[1][half:])]),
    "bidir_1+1": run([(0, d[0], h[0]), (1, h[1], d[1])]),
    "bidir_2+2": run([(0, d[0][:half], h[0][:half]), (1, d[0][half:], h[0][half:]),
                      (2, h[1][:half], d[1][:half]), (3, h[1][half:], d[1][half:])]),
    "bytes_per_copy": N,
}
print(json.dumps(out))
