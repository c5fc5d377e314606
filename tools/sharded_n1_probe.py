#!/usr/bin/env python3
"""configs[3]'s N = 1 point three ways in one process, interleaved over
rounds: the sharded rebuild step as bench.py times it (ShardedSetRunner.
rebuild, with its start / done timing events), the same step without the
events (runner.timing = False), and the decode phase alone
(run_phases(PHASE_COMPUTE)); plus the whole-set rebuild plan over the same
cells' layout for reference. Host clock, K steps bracketed by synchronize.
Prints one JSON line.

--sequence: instead, bench.py's order with one fresh runner -- encode,
snapshot, erase, then K-step loops back to back: step, step, decode, step,
decode -- to see whether the first loop pays for something the later ones
do not.

--placement: instead, the decode phase for runners whose hosted slabs are
separate allocations created behind spacers of 0 / 8 / 24 MiB (where the
allocator puts them), or one allocation with the parity slab 0 .. 56 MiB
after the data slab (ShardedSetRunner parity_gap), and each slab's base
address modulo 64 MiB.

usage: python tools/sharded_n1_probe.py [--steps 20] [--rounds 5] [--placement]
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
    ap.add_argument("--placement", action="store_true")
    ap.add_argument("--sequence", action="store_true")
    a = ap.parse_args()
    if a.placement:
        return placement(a)
    if a.sequence:
        return sequence(a)
    import torch

    from redset_amd import dist as rdist
    from redset_amd._lib import PHASE_COMPUTE

    p, e, chunk, lost = 11, 3, 64 << 20, [1, 2]
    runner = rdist.ShardedSetRunner(p, e, chunk, lost, world=1, rank=0)
    runner.encode()
    nbytes = runner.algorithmic_bytes("rebuild")

    def clock(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    def marked():
        runner.timing = True
        runner.rebuild()

    def unmarked():
        runner.timing = False
        runner.rebuild()

    def decode():
        runner.run_phases("rebuild", [PHASE_COMPUTE])

    variants = {"step_with_events": marked, "step_without_events": unmarked, "decode_phase": decode}
    for fn in variants.values():
        clock(fn)
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, fn in variants.items():
            res[k].append(clock(fn))
            runner.reset_timing()
    out = {"workload": "configs[3] at N = 1: RS(8+3) p=11, 64 MiB, rebuild {1,2}, sharded layout (world 1)",
           "steps": a.steps, "rounds": a.rounds}
    for k, v in res.items():
        med = sorted(v)[len(v) // 2]
        out[k] = {"ms_median": round(med * 1e3, 4), "GBps": round(nbytes / med / 1e9, 1),
                  "ms_all": [round(x * 1e3, 4) for x in v]}
    runner.close()
    print(json.dumps(out))


def sequence(a):
    import torch

    from redset_amd import dist as rdist
    from redset_amd._lib import PHASE_COMPUTE

    p, e, chunk, lost = 11, 3, 64 << 20, [1, 2]
    runner = rdist.ShardedSetRunner(p, e, chunk, lost, world=1, rank=0)
    runner.encode()
    snap = runner.lost_snapshot()
    runner.erase()

    def loop(fn, warm=5):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / a.steps * 1e3, 4)

    step = runner.rebuild
    decode = lambda: runner.run_phases("rebuild", [PHASE_COMPUTE])  # noqa: E731
    seq = [("step", step), ("step", step), ("decode", decode), ("step", step), ("decode", decode)]
    out = {"workload": "configs[3] at N = 1, bench.py's order", "steps": a.steps,
           "ms": [(k, loop(fn)) for k, fn in seq], "bit_exact": runner.matches(snap)}
    runner.close()
    print(json.dumps(out))


def placement(a):
    import torch

    from redset_amd import dist as rdist
    from redset_amd._lib import PHASE_COMPUTE

    p, e, chunk, lost = 11, 3, 64 << 20, [1, 2]
    out = {"workload": "configs[3] at N = 1, decode phase, runner created behind a spacer allocation",
           "steps": a.steps}
    cases = [("spacer", m) for m in (0, 8, 24)] + [("gap", m) for m in range(0, 64, 8)]
    for kind, mib in cases:
        spacer = torch.empty(mib << 20, dtype=torch.uint8, device="cuda") if (kind == "spacer" and mib) else None
        runner = rdist.ShardedSetRunner(p, e, chunk, lost, world=1, rank=0,
                                        parity_gap=(mib << 20) if kind == "gap" else None)
        runner.encode()
        fn = lambda: runner.run_phases("rebuild", [PHASE_COMPUTE])  # noqa: E731
        for _ in range(3):
            fn()
        ts = []
        for _ in range(a.rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / a.steps)
        med = sorted(ts)[len(ts) // 2]
        mod = {k: (t.data_ptr() % (64 << 20)) >> 20 for k, t in
               (("D_host", runner.D_host), ("P_host", runner.P_host))}
        out[f"{kind}_{mib}MiB"] = {"ms_median": round(med * 1e3, 4),
                                   "GBps": round(runner.algorithmic_bytes("rebuild") / med / 1e9, 1),
                                   "base_mod_64MiB_in_MiB": mod}
        runner.close()
        del runner, spacer
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
