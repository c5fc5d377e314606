"""How evenly the blocks of one codec launch finish (timing-only build).

Needs the library built with -DREDSET_BLOCK_CLOCK=1
(tools/build_ab_variant.sh clock -DREDSET_BLOCK_CLOCK=1 -> abx/lib_clock.so),
loaded through REDSET_HIP_LIBRARY. Every block of a gf_mac / xor launch
records its start and end (s_memrealtime, 100 MHz) and its XCC / HW_ID; this
runs the bench's RS(8+3) 64 MiB whole-set encode and rebuild plans (and XOR
p = 8) and reports, for the last launch of each execute:
  ramp   -- last block start - first block start
  span   -- last block end - first block start (the launch)
  busy   -- mean block duration; 1 - busy / span is the share of the launch's
            CU time spent idle at its edges (launch ramp + tail)
  end spread and per-XCC mean durations.
usage: REDSET_HIP_LIBRARY=abx/lib_clock.so python tools/block_clock.py [reps]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import redset_amd  # noqa: E402
from redset_amd import _lib  # noqa: E402

MiB = 1 << 20
TICK_US = 0.01  # s_memrealtime runs at 100 MHz
CLOCK = False


def read_clock(n=4096):
    L = _lib.load()
    fn = L.redset_hip_debug_block_clock
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * (3 * n))()
    torch.cuda.synchronize()
    assert fn(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 3)
    return a[a[:, 0] != 0]


def summarize(rows):
    t0 = rows[:, 0].astype(np.int64)
    t1 = rows[:, 1].astype(np.int64)
    base = t0.min()
    dur = (t1 - t0) * TICK_US
    span = (t1.max() - base) * TICK_US
    xcc = (rows[:, 2] >> np.uint64(32)).astype(np.int64)
    ends = (t1 - base) * TICK_US
    per_xcc = {int(x): round(float(dur[xcc == x].mean()), 2) for x in np.unique(xcc)}
    return {
        "blocks": int(len(rows)),
        "ramp_us": round(float((t0.max() - base) * TICK_US), 2),
        "span_us": round(float(span), 2),
        "busy_mean_us": round(float(dur.mean()), 2),
        "edge_idle_frac": round(float(1 - dur.mean() / span), 4),
        "end_us": {"min": round(float(ends.min()), 2), "p10": round(float(np.percentile(ends, 10)), 2),
                   "median": round(float(np.median(ends)), 2), "p90": round(float(np.percentile(ends, 90)), 2),
                   "max": round(float(ends.max()), 2)},
        "dur_by_xcc_us": per_xcc,
    }


def event_us(plan, reps, launches):
    """mean event-timed microseconds per launch of the plan"""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    plan.execute()
    a.record()
    for _ in range(reps):
        plan.execute()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1000 / reps / launches, 2)


def run(name, plan, reps, launches):
    ev = event_us(plan, reps, launches)
    if not CLOCK:
        print(json.dumps({"case": name, "lib": _lib.LIB_PATH, "event_us_per_launch": ev}), flush=True)
        return
    plan.execute()
    out = []
    for _ in range(reps):
        plan.execute()
        out.append(summarize(read_clock()))
    # is a slow block slow again next launch? end times per CU (XCC_ID, HW_ID's
    # SE / SH / CU fields) across launches
    ends = []
    for _ in range(reps):
        plan.execute()
        rows = read_clock()
        t0 = rows[:, 0].astype(np.int64)
        hw = rows[:, 2].astype(np.int64)
        cu_key = ((hw >> 32) << 16) | ((hw & 0xFFFF) >> 8)  # xcc | se/sh/cu bits of HW_ID
        e = {int(k): float(v) for k, v in zip(cu_key, (rows[:, 1].astype(np.int64) - t0.min()) * TICK_US)}
        ends.append(e)
    common = sorted(set.intersection(*[set(e) for e in ends]))
    M = np.array([[e[k] for k in common] for e in ends])
    M = M - M.mean(axis=1, keepdims=True)
    corr = [float(np.corrcoef(M[i], M[i + 1])[0, 1]) for i in range(len(M) - 1)]
    persist = {"cus": len(common), "end_corr_consecutive_mean": round(float(np.mean(corr)), 3),
               "per_cu_mean_end_spread_us": round(float(M.mean(axis=0).max() - M.mean(axis=0).min()), 2),
               "per_launch_end_spread_us": round(float(np.mean(M.max(axis=1) - M.min(axis=1))), 2)}
    keys = ("ramp_us", "span_us", "busy_mean_us", "edge_idle_frac")
    mean = {k: round(float(np.mean([o[k] for o in out])), 4) for k in keys}
    print(json.dumps({"case": name, "lib": _lib.LIB_PATH, "event_us_per_launch": ev, "mean": mean,
                      "persistence": persist, "last": out[-1]}), flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    global CLOCK
    CLOCK = hasattr(_lib.load(), "redset_hip_debug_block_clock")  # else event times only
    C = 64 * MiB
    p, e = 11, 3
    pad = redset_amd.cell_stride(C) - C
    codec = redset_amd.RSCodec(p, e)
    lay = redset_amd.SetLayout.allocate(p, p - e, e, C, pad=pad)
    for r in range(p):
        lay.lofi(r).random_(0, 256)
    enc = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), C, lay.cell_stride)
    reb = codec.plan_rebuild([1, 2], lay.lofi_ptrs(), lay.parity_ptrs(), C, lay.cell_stride)
    run("rs_encode_8_3", enc, reps, p)
    run("rs_rebuild_8_2", reb, reps, p)
    del enc, reb, lay
    torch.cuda.empty_cache()
    px = 8
    xl = redset_amd.SetLayout.allocate(px, px - 1, 1, C, pad=pad)
    for r in range(px):
        xl.lofi(r).random_(0, 256)
    xe = redset_amd.xor_plan_encode(px, xl.lofi_ptrs(), xl.parity_ptrs(), C, xl.cell_stride)
    run("xor_encode_7", xe, reps, px)


if __name__ == "__main__":
    main()
