#!/usr/bin/env python3
"""What per-step timing events cost the bench's step on the GPU: the
default bench workload (RS(8+3), p = 11, 64 MiB cells, full-set encode +
rebuild of {1, 2}) timed K steps by the host clock (synchronize on both
sides) with 0, 1, 2 or 3 timing events recorded per step (torch.cuda.Event
(enable_timing=True).record() on the launch stream, as bench.py does),
interleaved over several rounds so box drift hits every variant alike.
Prints one JSON line.

usage: python tools/event_cost.py [--steps 20] [--rounds 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    import torch

    import redset_amd

    p, e, chunk, lost = 11, 3, 64 << 20, [1, 2]
    codec = redset_amd.RSCodec(p, e)
    lay = redset_amd.SetLayout.allocate(p, p - e, e, chunk)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    for r in range(p):
        n = lay.lofi(r).numel()
        lay.lofi(r).copy_(torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g))
    enc = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    reb = codec.plan_rebuild(lost, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    stream = torch.cuda.current_stream()
    nbytes = enc.bytes_read + enc.bytes_written + reb.bytes_read + reb.bytes_written

    def run(nev):
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            if nev >= 1:
                evs[i][0].record(stream)
            enc.execute(stream)
            if nev >= 3:
                evs[i][1].record(stream)
            reb.execute(stream)
            if nev >= 2:
                evs[i][2].record(stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    for _ in range(3):
        run(0)
    res = {n: [] for n in (0, 1, 2, 3)}
    for _ in range(a.rounds):
        for n in res:
            res[n].append(run(n))
    out = {"workload": "RS(8+3) p=11, 64 MiB cells: encode + rebuild {1,2} (bench.py's step)", "steps": a.steps,
           "rounds": a.rounds}
    for n, v in res.items():
        v = sorted(v)
        med = v[len(v) // 2]
        out[f"events_{n}"] = {"ms_per_step_median": round(med * 1e3, 4), "GBps": round(nbytes / med / 1e9, 1),
                              "ms_all": [round(x * 1e3, 4) for x in res[n]]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
