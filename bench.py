#!/usr/bin/env python3
"""Device-resident RS/XOR encode+rebuild throughput on MI355X.

Step (N=1, BASELINE.json configs[2] + configs[3]): one redundancy set of
p = 11 members, RS(8+3) (redset ranks=11, encoding=3), 64 MiB chunks, all
cells resident in HBM: encode the parity of all 11 stripes, then rebuild
members {1, 2} from the survivors. Both passes run the gf_mac HIP kernel.
`value` = algorithmic bytes of both passes / wall time of the step, GB/s
(10^9 B). Algorithmic bytes per stripe: encode (d + e)*C, rebuild (d + m)*C
(SURVEY.md §8d).

N>1 (one process per GPU, RCCL): weak scaling. Redundancy sets are
independent objects, so the timed step shards them across ranks with no
data-path collective: every GPU encodes + rebuilds its own set exactly as at
N=1, and `value` = all ranks' algorithmic bytes / the max-over-ranks step
time. The path's one real exchange -- the multi-rank rebuild whose chunks are
gathered over xGMI (BASELINE.json configs[3]) -- is measured
after it as a second timed leg and reported under "sharded": N sets whose
members are spread round-robin over the GPUs, erased members rebuilt
column-sharded over all GPUs after an RCCL P2P gather of the decode inputs'
slices (redset_amd.dist), exchange inside the timing, result checked bit-exact.
The sharded leg runs at N=1 too (world-1 RCCL transport: every slice is
the process's own, computed in place, so no message moves), so configs[3]'s
curve has its base point in every N=1 line; `sharded.value` is configs[3]'s
scaling number at every N.

Launch: under torchrun (RANK / WORLD_SIZE set) every process is one rank.
`--gpus N > 1` without torchrun starts the N ranks itself, as a torchrun child
process, before this process touches the GPU, and relays rank 0's line.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# xGMI: per link and direction (7 links x ~153 GB/s per GPU)
XGMI_LINK_GBPS = 153.0
MODEL_GF_MAC_GBPS = 6300.0  # the whole-set rebuild's measured rate, for the sharded leg's model
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MIB = 1 << 20


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ranks", type=int, default=11, help="redset set size p")
    ap.add_argument("--encoding", type=int, default=3, help="parity cells per stripe e")
    ap.add_argument("--chunk-mib", type=float, default=64.0)
    ap.add_argument("--lost", default="1,2", help="members rebuilt each step")
    ap.add_argument("--cell-pad-mib", type=float, default=-1.0,
                    help="MiB of padding after every cell in HBM; -1 (default) = the library's recommended "
                         "stride (redset_hip_cell_stride: 16 MiB after 64 MiB cells, breaking their 2^26-byte "
                         "aliasing, +2.0%% with stripes in sequence, profiles/r02_ab_cell_pad.txt)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="1: time the CPU port beside (rank 0, every N)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU sample duration (RS; XOR gets half)")
    ap.add_argument("--cpu-chunk-mib", type=float, default=0.0,
                    help="chunk of the CPU baseline's set (0: the GPU workload's own chunk)")
    ap.add_argument("--sharded", type=int, default=1,
                    help="also time the RCCL sharded-rebuild leg (configs[3]; at N=1 over the world-1 transport)")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="self-launched N>1 runs: seconds before the rank processes are stopped")
    ap.add_argument("--sharded-timeout", type=float, default=150.0,
                    help="seconds the sharded leg may take before the main line is printed without it")
    ap.add_argument("--xor", type=int, default=1, help="also time the XOR set of configs[1] (rank 0)")
    ap.add_argument("--sharded-shape", default="auto", choices=["auto", "gather", "reduce"],
                    help="the sharded leg's exchange shape (include/redset_hip.h REDSET_HIP_SHAPE_*): auto lets "
                         "the planner take the one whose busiest GPU moves fewer bytes")
    ap.add_argument("--sharded-transport", default="", choices=["", "rccl", "torch"],
                    help="the sharded leg's transport (default: RCCL under an nccl process group or at N = 1, "
                         "else the torch.distributed callback); tests force rccl under gloo with the test twin "
                         "and tests/rcclstub")
    ap.add_argument("--pairs", type=int, default=1,
                    help="also time the rebuild of every pair of erased members (rank 0; SURVEY.md §8d worst case)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="process-group backend (nccl = RCCL; gloo only to rehearse N>1 on one GPU)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    return ap.parse_args()


def _host_random(n, rng):
    import numpy as np

    return np.frombuffer(bytearray(rng.bytes(n)), dtype=np.uint8)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        return ""


def cpu_baseline(p, e, lost, target_s, chunk):
    """Reference CPU path on host cores: redset_reedsolomon_encode_pthreads
    (src/redset_reedsolomon_pthreads.c:567-699) for the encode and the serial
    CPU decode the reference falls back to for PTHREADS (src/redset_reedsolomon.c:
    994-1000), both as restated in oracle/ (kind "port"), on the bench's own
    set shape and chunk size (64 MiB cells by default: 5.6 GiB of data in
    host memory); passes repeat until `target_s` of CPU work is done."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib

    oracle_lib.build()
    st = oracle_lib.OracleRS(p, e)
    d = p - e
    rng = np.random.default_rng(7)
    lofi = [_host_random(d * chunk, rng) for _ in range(p)]
    parity = [np.zeros(e * chunk, np.uint8) for _ in range(p)]
    passes, t_enc, t_reb, threads = 0, 0.0, 0.0, 0
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        threads = st.encode_pthreads(lofi, parity, chunk, slice_bytes=MIB)
        t1 = time.perf_counter()
        lf = [x if r not in lost else np.zeros_like(x) for r, x in enumerate(lofi)]
        pr = [x if r not in lost else np.zeros_like(x) for r, x in enumerate(parity)]
        st.rebuild_set(lost, lf, pr, chunk, slice_bytes=MIB)
        t2 = time.perf_counter()
        t_enc += t1 - t0
        t_reb += t2 - t1
        passes += 1
        if time.perf_counter() - t_start >= target_s:
            break
    ok = all(np.array_equal(lf[r], lofi[r]) and np.array_equal(pr[r], parity[r]) for r in lost)
    enc_bytes = p * (d + e) * chunk * passes
    reb_bytes = p * (d + len(lost)) * chunk * passes
    # (ii) of SURVEY.md §8d: one thread of redset_rs_reduce_buffer_multadd's
    # premult loop (src/redset_reedsolomon_common.c:798-811) on 64 MiB slices
    # (the source is the first member's logical file, d cells: at small
    # chunks shorter than 64 MiB, and multadd reads buf.size bytes of it)
    n_ma = min(64 * MIB, lofi[0].size)
    buf = np.zeros(n_ma, np.uint8)
    src = np.ascontiguousarray(lofi[0][:n_ma])
    reps, t_ma = 0, 0.0
    while t_ma < min(3.0, target_s / 3):
        t0 = time.perf_counter()
        st.multadd(buf, 29, src)
        t_ma += time.perf_counter() - t0
        reps += 1
    return {
        "value": round((enc_bytes + reb_bytes) / (t_enc + t_reb) / 1e9, 4),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": (
            f"{passes} x (RS({d}+{e}) full-set encode with {threads} pthreads + serial rebuild of "
            f"members {lost}), p={p}, chunk={chunk / MIB:g} MiB (host buffers, the GPU workload's shape); encode "
            f"{enc_bytes / t_enc / 1e9:.3f} GB/s, rebuild {reb_bytes / t_reb / 1e9:.3f} GB/s"
        ),
        "encode_GBps": round(enc_bytes / t_enc / 1e9, 4),
        "rebuild_GBps": round(reb_bytes / t_reb / 1e9, 4),
        "round_trip_equal": ok,
        "host_cpus": os.cpu_count(),
        "cpu_model": _cpu_model(),
        # input bytes of one multadd (data read; the accumulator's RMW not counted), GB/s
        "multadd_1thread_GBps": round(reps * n_ma / t_ma / 1e9, 4),
    }


def cpu_baseline_xor(p, root, target_s, chunk):
    """XOR CPU baseline beside the XOR leg (BASELINE.json configs[1]):
    redset_xor_encode_pthreads (src/redset_xor_pthreads.c:311-392) for the
    encode and the serial rebuild (src/redset_xor_serial.c:161-275), as
    restated in oracle/, on the XOR leg's own shape (p=8, 64 MiB cells)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib

    oracle_lib.build()
    rng = np.random.default_rng(8)
    lofi = [_host_random((p - 1) * chunk, rng) for _ in range(p)]
    xorc = [np.zeros(chunk, np.uint8) for _ in range(p)]
    passes, t_enc, t_reb, threads = 0, 0.0, 0.0, 0
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        threads = oracle_lib.xor_encode_pthreads(p, lofi, xorc, chunk, slice_bytes=MIB)
        t1 = time.perf_counter()
        lf = [x if r != root else np.zeros_like(x) for r, x in enumerate(lofi)]
        xc = [x if r != root else np.zeros_like(x) for r, x in enumerate(xorc)]
        oracle_lib.xor_rebuild_set(p, root, lf, xc, chunk, slice_bytes=MIB)
        t2 = time.perf_counter()
        t_enc += t1 - t0
        t_reb += t2 - t1
        passes += 1
        if time.perf_counter() - t_start >= target_s:
            break
    ok = np.array_equal(lf[root], lofi[root]) and np.array_equal(xc[root], xorc[root])
    nbytes = p * p * chunk * passes  # p cells per stripe, p stripes, both passes
    return {
        "value": round(2 * nbytes / (t_enc + t_reb) / 1e9, 4),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{passes} x (XOR p={p} full-set encode with {threads} pthreads + serial rebuild of member "
                   f"{root}), chunk={chunk / MIB:g} MiB (host buffers, the XOR leg's shape); encode "
                   f"{nbytes / t_enc / 1e9:.3f} GB/s, rebuild {nbytes / t_reb / 1e9:.3f} GB/s"),
        "encode_GBps": round(nbytes / t_enc / 1e9, 4),
        "rebuild_GBps": round(nbytes / t_reb / 1e9, 4),
        "round_trip_equal": bool(ok),
    }


def load_traffic(path, kernel_prefix):
    """HBM bytes per launch of the dominant kernel from a rocprofv3 PMC pass
    (tools/pmc_traffic.py writes this file); None if absent."""
    try:
        with open(path) as f:
            t = json.load(f)
        return t.get(kernel_prefix)
    except (OSError, ValueError):
        return None


def traffic_source(path):
    """Where the PMC bytes of `path` were measured (its _provenance block):
    another process -- rocprofv3 must wrap the program -- of this bench,
    usually on another box and in another session than this line's."""
    try:
        with open(path) as f:
            prov = json.load(f).get("_provenance") or {}
    except (OSError, ValueError):
        prov = {}
    where = ", ".join(f"{k} {prov[k]}" for k in ("session", "host", "date") if prov.get(k))
    return (f"{os.path.relpath(path, ROOT)} ({where or 'provenance not recorded'}): rocprofv3 --pmc FETCH_SIZE / "
            "WRITE_SIZE in separate runs of this bench, not measured in this process")


def cell_pad(args, chunk):
    """Bytes after every cell: --cell-pad-mib, or (-1) what the library's
    recommended stride adds to the 256-B-aligned chunk (include/redset_hip.h
    redset_hip_cell_stride), the layout INTEGRATION.md advises."""
    import redset_amd

    if args.cell_pad_mib >= 0:
        return int(args.cell_pad_mib * MIB)
    return redset_amd.cell_stride(chunk) - -(-chunk // 256) * 256


def timed(step, steps, warmup, dist_on, before=None):
    """W untimed warmups, then K steps bracketed by barrier + synchronize on
    both sides; returns the max-over-ranks elapsed seconds."""
    import torch

    for _ in range(warmup):
        step(-1)
    torch.cuda.synchronize()
    if before is not None:
        before()
    if dist_on:
        import torch.distributed as dist

        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist_on:
        on_gpu = dist.get_backend() == "nccl"
        t = torch.tensor([elapsed], device="cuda" if on_gpu else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def round_trip(lay, enc_plan, reb_plan, lost, stream):
    """Full-size encode -> erase -> rebuild: the erased members' cells (data
    and the parity the encode just wrote) must come back bit for bit -- the
    size-independent parity property of the timed workload (the oracle
    comparisons themselves live in tests/ at sizes the CPU finishes)."""
    import torch

    enc_plan.execute(stream)
    torch.cuda.synchronize()
    cells = [c for r in lost for c in
             [lay.data_cell(r, s) for s in range(lay.data_cells)] + [lay.parity_cell(r, i) for i in range(lay.parity_cells)]]
    snap = [c.clone() for c in cells]
    for c in cells:
        c.fill_(0xEE)
    reb_plan.execute(stream)
    torch.cuda.synchronize()
    return all(torch.equal(c, s) for c, s in zip(cells, snap))


def copy_probe(stream, nbytes=1 << 30, reps=10):
    """This box's HBM rate for a plain device-to-device copy (torch's copy
    kernel, read + write bytes / time): boxes differ by several percent, so
    the codec's rate is reported beside what the same HBM does for a copy."""
    import torch

    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        for _ in range(3):
            b.copy_(a)
        e0.record(stream)
        for _ in range(reps):
            b.copy_(a)
        e1.record(stream)
    torch.cuda.synchronize()
    return round(2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)


def rebuild_pairs(codec, lay, chunk, stream, reps=5, passes=2):
    """configs[3] over every erasure pair: the rebuild rate of each 2-member
    pattern on the bench's own set (event-timed, `reps` executes after one
    warm-up, mean over `passes` sweeps; one pass alone leaves single pairs
    up to 10% low by noise, profiles/r01_rebuild_pairs.txt). The decode reads
    d survivors per stripe whatever the pair, but which cells (data or
    parity) and their coefficients differ."""
    import itertools

    import torch

    p = lay.ranks
    plans = {pair: codec.plan_rebuild(list(pair), lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
             for pair in itertools.combinations(range(p), 2)}
    sums = dict.fromkeys(plans, 0.0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # the first pair measured ran 5-10% low on every box without this warm-up
    first = next(iter(plans.values()))
    for _ in range(20):
        first.execute(stream)
    for _ in range(passes):
        for pair, plan in plans.items():
            plan.execute(stream)
            e0.record(stream)
            for _ in range(reps):
                plan.execute(stream)
            e1.record(stream)
            torch.cuda.synchronize()
            nbytes = plan.bytes_read + plan.bytes_written
            sums[pair] += nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    rates = {pair: v / passes for pair, v in sums.items()}
    for plan in plans.values():
        plan.close()
    worst = min(rates, key=rates.get)
    best = max(rates, key=rates.get)
    vals = sorted(rates.values())
    return {
        "pairs": len(rates),
        "min_GBps": round(rates[worst], 1), "worst_pair": list(worst),
        "median_GBps": round(vals[len(vals) // 2], 1),
        "max_GBps": round(rates[best], 1), "best_pair": list(best),
    }


def xor_leg(args, chunk, stream):
    """BASELINE.json configs[1]: XOR set of 8 ranks, 64 MiB chunks -- encode
    all 8 parity cells + rebuild one member (xor_kernel<7>), timed with HIP
    events on the launch stream; reported beside the RS line."""
    import torch
    import redset_amd

    p = 8
    lay = redset_amd.SetLayout.allocate(p, p - 1, 1, chunk, pad=cell_pad(args, chunk))
    g = torch.Generator(device="cuda")
    g.manual_seed(77)
    for r in range(p):
        n = lay.lofi(r).numel()
        lay.lofi(r).copy_(torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g))
    enc = redset_amd.xor_plan_encode(p, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    reb = redset_amd.xor_plan_rebuild(p, 3, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(args.warmup):
        enc.execute(stream)
        reb.execute(stream)
    t_enc = t_reb = 0.0
    for _ in range(args.steps):
        ev[0].record(stream)
        enc.execute(stream)
        ev[1].record(stream)
        reb.execute(stream)
        ev[2].record(stream)
        torch.cuda.synchronize()
        t_enc += ev[0].elapsed_time(ev[1])
        t_reb += ev[1].elapsed_time(ev[2])
    eb = enc.bytes_read + enc.bytes_written
    rb = reb.bytes_read + reb.bytes_written
    t_enc, t_reb = t_enc / args.steps, t_reb / args.steps
    ok = round_trip(lay, enc, reb, [3], stream)
    return {
        "workload": f"XOR p={p}, chunk {chunk // MIB} MiB: encode all {p} parity cells + rebuild member 3 "
                    "(BASELINE.json configs[1])",
        "value": round((eb + rb) / ((t_enc + t_reb) * 1e-3) / 1e9, 1),
        "unit": "GB/s",
        "frac": round((eb + rb) / ((t_enc + t_reb) * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "encode_GBps": round(eb / (t_enc * 1e-3) / 1e9, 1),
        "rebuild_GBps": round(rb / (t_reb * 1e-3) / 1e9, 1),
        "launches_per_step": {"encode": enc.launches, "rebuild": reb.launches},
        "avg_launch_ms": {"encode": round(t_enc / enc.launches, 4), "rebuild": round(t_reb / reb.launches, 4)},
        "algorithmic_bytes_per_launch": {"encode": eb // enc.launches, "rebuild": rb // reb.launches},
        "round_trip_bit_exact": ok,
    }


def sharded_leg(args, p, e, chunk, lost, world, rank):
    """BASELINE.json configs[3]: erase members, rebuild them with the set's
    cells spread over the node's GPUs (redset_amd.dist). N sets, member m on
    GPU m mod N; the timed step is the rebuild only -- gather my column slice
    of every decode input over RCCL, gf_mac, return the rebuilt slices to
    their hosts. Parity comes from one untimed sharded encode beforehand.
    After timing every GPU checks that its lost members' slabs are back bit
    for bit (min over ranks). At world 1 (no process group) the transport is
    RCCL over a one-rank communicator with nothing to send, and the step is
    configs[3]'s N=1 point."""
    import torch
    import torch.distributed as dist

    import redset_amd
    from redset_amd import dist as rdist
    from redset_amd._lib import PHASE_ACCUMULATE as L_PHASE_ACCUMULATE, PHASE_COMPUTE as L_PHASE_COMPUTE
    from redset_amd._lib import PHASE_GATHER as L_PHASE_GATHER, PHASE_RETURN as L_PHASE_RETURN

    dist_on = world > 1
    dev = "cuda" if (not dist_on or dist.get_backend() == "nccl") else "cpu"

    def reduce(x, op, dtype):
        t = torch.tensor([x], dtype=dtype, device=dev)
        if dist_on:
            dist.all_reduce(t, op=op)
        return t.item()

    runner = rdist.ShardedSetRunner(p, e, chunk, lost, world=world, rank=rank, shape=args.sharded_shape,
                                    transport=args.sharded_transport or None)
    shape = runner.shape("rebuild")
    runner.encode()
    snap = runner.lost_snapshot()
    runner.erase()
    # the leg starts after a pause in GPU work (planning, the snapshot): its
    # first ~25 steps run ~4% slow however they are split (the same loop
    # right after runs at full rate, profiles/r05s22_sequence.json), so over
    # RCCL it warms up for at least 25 steps whatever --warmup says (gloo
    # rehearsals take seconds per step and keep --warmup)
    warm = args.warmup
    if args.warmup > 0 and dev == "cuda":
        warm = max(args.warmup, SHARDED_MIN_WARMUP)
    s_elapsed = timed(lambda i: runner.rebuild(), args.steps, warm, dist_on, before=runner.reset_timing)
    s_step = s_elapsed / args.steps
    torch.cuda.synchronize()
    hangs = redset_amd.hang_faults()
    ok = reduce(1 if runner.matches(snap) and hangs == 0 else 0, dist.ReduceOp.MIN, torch.int32)
    value = world * runner.algorithmic_bytes("rebuild") / s_step / 1e9
    # bytes each GPU sends over the fabric per rebuild (C planner's count),
    # mean and max over the ranks
    sent_mine = float(runner.exchanged_bytes("rebuild"))
    sent_mean = reduce(sent_mine, dist.ReduceOp.SUM, torch.float64) / world
    sent_max = reduce(sent_mine, dist.ReduceOp.MAX, torch.float64)
    info = runner.info("rebuild")
    recv_max = reduce(float(info["gather_bytes_recv"] + info["return_bytes_recv"]), dist.ReduceOp.MAX, torch.float64)
    # untimed diagnostic: the same rebuild with its four phases one after
    # another (no overlap across sets), timed apart by events on rank 0
    pipelined_event_ms = runner.phase_ms().get("rebuild_start->done")
    runner.phased = True
    timed(lambda i: runner.rebuild(), 3, 1, dist_on, before=runner.reset_timing)
    phases = runner.phase_ms()
    compute_ms = phases.get("rebuild_gathered->computed")
    if compute_ms is not None and phases.get("rebuild_returned->done") is not None:
        compute_ms = round(compute_ms + phases["rebuild_returned->done"], 4)  # + the accumulate
    # BASELINE.md's C4 as it states it: the column-sharded decode on N GPUs
    # with every GPU's slices already in place, and the RCCL exchange (gather
    # + return) timed separately -- each K steps bracketed like the step,
    # max over ranks (partial-sum shape: the combines, and its one exchange)
    d_step = timed(lambda i: runner.run_phases("rebuild", [L_PHASE_COMPUTE, L_PHASE_ACCUMULATE]), args.steps, warm,
                   dist_on) / args.steps
    x_step = timed(lambda i: runner.run_phases("rebuild", [L_PHASE_GATHER, L_PHASE_RETURN]), args.steps,
                   min(warm, args.warmup), dist_on) / args.steps
    decode_value = world * runner.algorithmic_bytes("rebuild") / d_step / 1e9
    # The step's roofline is the fabric, not HBM: every GPU sends its
    # share of the decode inputs' slices to every other GPU and gets the
    # rebuilt slices back (an all-to-all over the node's fully connected
    # xGMI mesh: one link per peer pair, world - 1 links usable per GPU).
    link_peak = (world - 1) * XGMI_LINK_GBPS
    fabric_gbps = sent_mean / s_step / 1e9
    out = {
        "workload": (f"{world} sets of p={p} (RS({p - e}+{e}), chunk {chunk / MIB:g} MiB), members round-robin over "
                     f"{world} GPUs; rebuild of members {lost} of every set, column-sharded (BASELINE.json configs[3])"),
        "value": round(value, 2),
        "unit": "GB/s",
        # north_star: the sharded rebuild "as absolute GB/s and as fraction of HBM peak"
        "frac_of_hbm": round(value / (world * HBM_PEAK_GBPS), 6),
        "hbm_peak_GBps": world * HBM_PEAK_GBPS,
        "ms_per_step": round(s_step * 1e3, 4),
        "bit_exact": bool(ok),
        "transport": type(runner._transport).__name__ + ("" if dist_on else " (world 1: no messages)"),
        # the exchange's shape, chosen by the planner from its byte counts
        # (include/redset_hip.h REDSET_HIP_SHAPE_*): gather the inputs' column
        # slices, or send each GPU's partial sums of its own inputs
        "shape": shape["shape"],
        "schedule": ("sets pipelined: set k+1's gather overlaps set k's gf_mac (redset_hip_sharded_execute)"
                     if shape["shape"] == "gather" else
                     "sets pipelined: set k's partial-sum exchange overlaps set k+1's combines "
                     "(redset_hip_sharded_execute)"),
        "pipelined_event_ms_rank0": pipelined_event_ms,
        "roofline": {
            "bound": "xgmi",
            "achieved": round(fabric_gbps, 2),
            "peak": link_peak,
            "unit": "GB/s per GPU (bytes sent over the fabric / step time)",
            "frac": round(fabric_gbps / link_peak, 4),
            "bytes_sent_per_gpu_per_step": {"mean": int(sent_mean), "max": int(sent_max)},
            "peak_source": (f"{XGMI_LINK_GBPS:g} GB/s per xGMI link and direction x (world - 1) links: one link per "
                            "GPU pair of the node's fully connected mesh, 7 per GPU at 8 GPUs (SURVEY.md §5; "
                            "MI355X platform figure, not measured here)"),
        } if dist_on else {
            # world 1: nothing crosses the fabric and nothing is copied (a
            # process computes its own slice of the members it hosts in
            # place): the step is the gf_mac's, HBM-bound
            "bound": "hbm",
            "achieved": round(runner.algorithmic_bytes("rebuild") / s_step / 1e9, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s (algorithmic bytes / step time)",
            "frac": round(runner.algorithmic_bytes("rebuild") / s_step / 1e9 / HBM_PEAK_GBPS, 4),
        },
        # what the planner's bytes predict for this step (tools/sharded_model.py):
        # the exchange at (N - 1) x 153 GB/s per GPU against the gf_mac at the
        # measured whole-set rebuild rate; the step costs about the larger
        "model": {
            "xgmi_ms": round(max(sent_max, recv_max) / (link_peak * 1e9) * 1e3, 4) if dist_on else 0.0,
            "hbm_ms": round(info["compute_bytes"] / (MODEL_GF_MAC_GBPS * 1e9) * 1e3, 4),
            "value": round(world * runner.algorithmic_bytes("rebuild") / max(
                max(sent_max, recv_max) / (link_peak * 1e9) if dist_on else 0.0,
                info["compute_bytes"] / (MODEL_GF_MAC_GBPS * 1e9)) / 1e9, 1),
            "note": f"{XGMI_LINK_GBPS:g} GB/s per xGMI link (platform figure), gf_mac {MODEL_GF_MAC_GBPS:g} GB/s",
            # both shapes' busiest GPU (max over GPUs of max(sent, received))
            # at the same link rate: what each would cost on the fabric
            "xgmi_ms_by_shape": {
                "gather": round(shape["gather_busiest_bytes"] / (link_peak * 1e9) * 1e3, 4) if dist_on else 0.0,
                "reduce": (round(shape["reduce_busiest_bytes"] / (link_peak * 1e9) * 1e3, 4)
                           if dist_on and shape["reduce_possible"] else None),
            },
        },
        # C4's decode alone, slices in place (all GPUs, max over ranks)
        "decode": {
            "value": round(decode_value, 2),
            "unit": "GB/s",
            "frac_of_hbm": round(decode_value / (world * HBM_PEAK_GBPS), 6),
            "ms_per_step": round(d_step * 1e3, 4),
            "note": "the rebuild's gf_mac on every GPU's column slice, inputs already gathered (no exchange)",
        },
        # C4's RCCL exchange alone: gather + return (no compute)
        "exchange_only": {
            "ms_per_step": round(x_step * 1e3, 4),
            "send_GBps_per_gpu": round(sent_mean / x_step / 1e9, 2) if sent_mean else None,
            "frac_of_xgmi": round(sent_mean / x_step / 1e9 / link_peak, 4) if (sent_mean and dist_on) else None,
        },
        # HBM is the bound of the compute phase alone (phased diagnostic)
        "compute_hbm": {
            "phase_ms_rank0": compute_ms,
            "achieved": (round(runner.algorithmic_bytes("rebuild") / (compute_ms * 1e-3) / 1e9, 1)
                         if compute_ms else None),
            "peak": HBM_PEAK_GBPS,
            "frac": (round(runner.algorithmic_bytes("rebuild") / (compute_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                     if compute_ms else None),
        },
    }
    out.update(runner.report(s_step, "rebuild"))
    # the plans, the codec and the RCCL communicator go before the process
    # group does (every rank is past the same collectives here)
    torch.cuda.synchronize()
    runner.close()
    if dist_on:
        out["one_set"] = one_set(args, p, e, chunk, lost, world, rank, warm, reduce, link_peak)
        # the shape not taken, measured (when the partial sums fit at all)
        if args.sharded_shape == "auto" and shape["reduce_possible"]:
            other = "gather" if shape["shape"] == "reduce" else "reduce"
            out["other_shape"] = other_shape(args, p, e, chunk, lost, world, rank, warm, reduce, link_peak, other)
    else:
        out["one_set"] = "at N = 1 the leg itself: one set on one GPU"
    return out


def runner_loops(runner, args, world, warm, reduce, link_peak):
    """The leg's three loops on a runner whose lost members are erased: the
    step (K rebuilds), the decode on slices in place (COMPUTE + ACCUMULATE)
    and the exchange alone (GATHER + RETURN), K steps each, bracketed and max
    over ranks; bit-exact checked after the step loop."""
    import torch
    import torch.distributed as dist

    import redset_amd
    from redset_amd._lib import PHASE_ACCUMULATE, PHASE_COMPUTE, PHASE_GATHER, PHASE_RETURN

    runner.timing = False
    runner.encode()
    snap = runner.lost_snapshot()
    runner.erase()
    dist_on = world > 1
    step = timed(lambda i: runner.rebuild(), args.steps, warm, dist_on) / args.steps
    torch.cuda.synchronize()
    ok = reduce(1 if runner.matches(snap) and redset_amd.hang_faults() == 0 else 0, dist.ReduceOp.MIN, torch.int32)
    d_step = timed(lambda i: runner.run_phases("rebuild", [PHASE_COMPUTE, PHASE_ACCUMULATE]), args.steps, warm,
                   dist_on) / args.steps
    x_step = timed(lambda i: runner.run_phases("rebuild", [PHASE_GATHER, PHASE_RETURN]), args.steps,
                   min(warm, args.warmup), dist_on) / args.steps
    total = runner.total_algorithmic_bytes("rebuild")
    sent_mean = reduce(float(runner.exchanged_bytes("rebuild")), dist.ReduceOp.SUM, torch.float64) / world
    shape = runner.shape("rebuild")
    torch.cuda.synchronize()
    runner.close()
    peak = world * HBM_PEAK_GBPS
    return {
        "shape": shape["shape"],
        "value": round(total / step / 1e9, 2),
        "frac_of_hbm": round(total / step / 1e9 / peak, 6),
        "ms_per_step": round(step * 1e3, 4),
        "bit_exact": bool(ok),
        "busiest_gpu_bytes_by_shape": {"gather": shape["gather_busiest_bytes"],
                                       "reduce": shape["reduce_busiest_bytes"] if shape["reduce_possible"] else None},
        "decode": {"value": round(total / d_step / 1e9, 2), "frac_of_hbm": round(total / d_step / 1e9 / peak, 6),
                   "ms_per_step": round(d_step * 1e3, 4)},
        "exchange_only": {"ms_per_step": round(x_step * 1e3, 4),
                          "bytes_sent_per_gpu": int(sent_mean),
                          "send_GBps_per_gpu": round(sent_mean / x_step / 1e9, 2) if sent_mean else None,
                          "frac_of_xgmi": round(sent_mean / x_step / 1e9 / link_peak, 4) if sent_mean else None},
    }


def one_set(args, p, e, chunk, lost, world, rank, warm, reduce, link_peak):
    """BASELINE.md's C4 word for word: ONE RS(8+3) set (configs[2]'s data)
    column-sharded over the N GPUs -- strong scaling, member r on GPU r mod N,
    every GPU rebuilding its 1/N column slice of every stripe. The same three
    loops as the leg (the step, the decode on slices in place, the exchange
    alone), K steps each, bracketed and max over ranks; bit-exact checked."""
    from redset_amd import dist as rdist

    runner = rdist.ShardedSetRunner(p, e, chunk, lost, world=world, rank=rank, sets=1, shape=args.sharded_shape,
                                    transport=args.sharded_transport or None)
    out = {"workload": (f"one set of p={p} (RS({p - e}+{e}), chunk {chunk / MIB:g} MiB) over {world} GPUs, member r "
                        f"on GPU r mod {world}; rebuild of {lost} (BASELINE.md C4, strong scaling)")}
    out.update(runner_loops(runner, args, world, warm, reduce, link_peak))
    return out


def other_shape(args, p, e, chunk, lost, world, rank, warm, reduce, link_peak, shape):
    """The leg once more with the exchange shape the planner did NOT take
    (forced), the same three loops: the measured A/B behind the planner's
    byte-count choice (gather = C4's column-sharded decode as BASELINE.md
    states it; reduce = partial sums of each GPU's own inputs)."""
    from redset_amd import dist as rdist

    runner = rdist.ShardedSetRunner(p, e, chunk, lost, world=world, rank=rank, shape=("auto", shape),
                                    transport=args.sharded_transport or None)
    return runner_loops(runner, args, world, warm, reduce, link_peak)


_PRINT_LOCK = threading.Lock()
_PRINTED = threading.Event()
_RESULT_OUT = None


def claim_stdout():
    """Keep stdout for the one JSON line: the process's fd 1 goes to stderr
    from here on (RCCL prints a version banner to stdout when a communicator
    is created, on every rank), and the line is written to a duplicate of
    the original stdout."""
    global _RESULT_OUT
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    _RESULT_OUT = os.fdopen(fd, "w", buffering=1)


def _print_result(result):
    out = _RESULT_OUT or sys.stdout
    print(json.dumps(result), file=out, flush=True)


def emit(result, rank):
    """Rank 0 prints the one JSON line (once, whichever thread gets here first)."""
    with _PRINT_LOCK:
        if rank == 0 and not _PRINTED.is_set():
            _print_result(result)
        _PRINTED.set()


WATCHDOG_EXIT = 3
SHARDED_MIN_WARMUP = 25


def sharded_expired(result, rank, limit):
    """Watchdog of the sharded leg and the final barrier: print the line
    measured so far if it is not out yet, then end this rank with a non-zero
    status (WATCHDOG_EXIT), so a hung exchange or barrier never looks like a
    clean run to the caller (the process group is left hung, not torn down)."""
    with _PRINT_LOCK:
        if not _PRINTED.is_set():
            result["sharded"] = {"error": f"timed out after {limit:g} s"}
            if rank == 0:
                _print_result(result)
            _PRINTED.set()
        print(f"rank {rank}: sharded leg or final barrier timed out after {limit:g} s", file=sys.stderr, flush=True)
        os._exit(WATCHDOG_EXIT)


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relay(lines, out=sys.stdout, err=sys.stderr):
    """Pass the rank processes' output on: the first JSON line carrying
    "metric" (rank 0's result) to `out`, everything else to `err` as it comes
    (so a long run shows progress). Returns whether the line was seen."""
    seen = False
    for ln in lines:
        s = ln.strip()
        if not seen and s.startswith("{"):
            try:
                if "metric" in json.loads(s):
                    print(s, file=out, flush=True)
                    seen = True
                    continue
            except ValueError:
                pass
        print(ln.rstrip("\n"), file=err, flush=True)
    return seen


def self_launch(argv, n, timeout, cmd=None):
    """`--gpus n > 1` without torchrun: start the n ranks as ONE child process
    (torch.distributed.run, rendezvous on 127.0.0.1) before this process makes
    any GPU call -- it never initialises the GPU and never execs -- and relay
    rank 0's line. The child's exit status is returned; a child still running
    after `timeout` seconds is stopped (its whole process group) and counts as
    failed."""
    if cmd is None:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
               os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, text=True, env=env, start_new_session=True)
    killer = threading.Timer(timeout, lambda: os.killpg(proc.pid, 9))
    killer.daemon = True
    killer.start()
    try:
        seen = relay(proc.stdout)
        rc = proc.wait()
    finally:
        killer.cancel()
    if not seen:
        print(json.dumps({"error": f"the {n} rank processes printed no result line (exit status {rc})"}), flush=True)
    return rc if rc != 0 or seen else 1


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(self_launch(sys.argv[1:], args.gpus, args.launch_timeout))
    claim_stdout()
    import torch

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        _print_result({"error": f"--gpus {args.gpus} but WORLD_SIZE={world}"})
        sys.exit(2)
    dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist_on = world > 1
    if dist_on:
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.dist_backend)

    import redset_amd

    redset_amd.load()
    p, e = args.ranks, args.encoding
    d = p - e
    chunk = int(args.chunk_mib * MIB)
    lost = sorted(int(x) for x in args.lost.split(",") if x != "")
    cpu_chunk = int(args.cpu_chunk_mib * MIB) if args.cpu_chunk_mib > 0 else chunk
    stream = torch.cuda.current_stream()

    # this rank's own set, all cells resident in HBM
    codec = redset_amd.RSCodec(p, e)
    lay = redset_amd.SetLayout.allocate(p, d, e, chunk, pad=cell_pad(args, chunk))
    g = torch.Generator(device="cuda")
    g.manual_seed(1234 + rank)
    for r in range(p):
        n = lay.lofi(r).numel()
        lay.lofi(r).copy_(torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g))
    enc_plan = codec.plan_encode(lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    reb_plan = codec.plan_rebuild(lost, lay.lofi_ptrs(), lay.parity_ptrs(), chunk, lay.cell_stride)
    eb = enc_plan.bytes_read + enc_plan.bytes_written
    rb = reb_plan.bytes_read + reb_plan.bytes_written
    bytes_per_step = eb + rb
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]

    def step(i):
        if i >= 0:
            ev[i][0].record(stream)
        enc_plan.execute(stream)
        if i >= 0:
            ev[i][1].record(stream)
        reb_plan.execute(stream)
        if i >= 0:
            ev[i][2].record(stream)

    elapsed = timed(step, args.steps, args.warmup, dist_on)
    ms_per_step = elapsed * 1e3 / args.steps
    # after the timed region: the round trip on this rank's set, and the box's copy rate
    rt_ok = round_trip(lay, enc_plan, reb_plan, lost, stream)
    # every launch so far (timed steps included) completed its loader-ring handshakes
    ring_faults = redset_amd.ring_faults()
    # no kernel wait without a fallback gave up (include/redset_hip.h
    # redset_hip_hang_faults): a nonzero count means wrong bytes somewhere
    hang_faults = redset_amd.hang_faults()
    rt_ok = rt_ok and ring_faults == 0 and hang_faults == 0
    if dist_on:
        flag = torch.tensor([int(rt_ok)], dtype=torch.int32, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        rt_ok = bool(flag.item())
    box_copy = copy_probe(stream)
    value = world * bytes_per_step / (elapsed / args.steps) / 1e9

    result = {
        "metric": "GB/s device-resident RS/XOR encode+rebuild vs HBM peak, 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: uniform random bytes (torch.randint on device), all cells resident in HBM",
        "config": {
            "workload": (f"RS({d}+{e}) p={p} e={e}, chunk {args.chunk_mib:g} MiB: full-set encode of all "
                         f"{p} stripes + rebuild of members {lost}, one set per GPU"),
            "ranks": p,
            "encoding": e,
            "chunk_bytes": chunk,
            "cell_stride_bytes": lay.cell_stride,
            "sets": world,
            "bytes_per_step_per_gpu": bytes_per_step,
            "parallelism": "single GPU" if world == 1 else f"{world} independent sets, one per GPU (no collective)",
            # which number is which: `value` is the independent-sets step
            # (configs[2] + configs[3] on each GPU), comparable from N=1 to
            # N=8; configs[3]'s multi-GPU scaling curve is sharded.value
            "scaling_value": ("sharded.value: configs[3]'s column-sharded rebuild step over RCCL/xGMI "
                              "(gather + gf_mac + return, pipelined over the sets), with sharded.frac_of_hbm; "
                              "sharded.decode and sharded.exchange_only: its decode on slices in place and its "
                              "RCCL exchange timed apart (BASELINE.md C4)" if args.sharded else None),
        },
    }
    step_ms = sorted(ev[k][0].elapsed_time(ev[k][2]) for k in range(args.steps))
    step_ms_median = step_ms[len(step_ms) // 2] if len(step_ms) % 2 else \
        (step_ms[len(step_ms) // 2 - 1] + step_ms[len(step_ms) // 2]) / 2
    enc_ms = sum(ev[k][0].elapsed_time(ev[k][1]) for k in range(args.steps)) / args.steps
    reb_ms = sum(ev[k][1].elapsed_time(ev[k][2]) for k in range(args.steps)) / args.steps
    # one launch = one stripe when a plan runs its jobs one after another (the
    # default for 64 MiB cells), else the whole set; a launch's average
    # duration is the plan's event span / its launches (gaps included)
    el, rl = enc_plan.launches, reb_plan.launches
    eb1, rb1 = eb // el, rb // rl
    achieved = (eb + rb) / ((enc_ms + reb_ms) * 1e-3) / 1e9
    # PMC-measured HBM bytes per gf_mac launch (tools/pmc_traffic.py; gfx950
    # FETCH_SIZE doubled); compare with the algorithmic bytes per launch
    k_enc = f"gf_mac_kernel<{d}, {min(e, 4)}, false>"
    k_reb = f"gf_mac_kernel<{d}, {min(len(lost), 4)}, false>"
    t_enc, t_reb = load_traffic(args.traffic_json, k_enc), load_traffic(args.traffic_json, k_reb)
    # the PMC file is recorded on the default workload; a different set shape
    # or chunk size has different bytes per launch, so it does not apply
    if not (t_enc and t_reb and 0.5 < t_enc / eb1 < 2.0 and 0.5 < t_reb / rb1 < 2.0):
        t_enc = t_reb = None
    traffic = (t_enc * el + t_reb * rl) // (el + rl) if (t_enc and t_reb) else None
    result["roofline"] = {
        "bound": "hbm",
        "kernel": f"{k_enc} (encode) + {k_reb} (rebuild), redset_amd/csrc/codec_device.h",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBPS, 4),
        "traffic": traffic,
        "launches_per_step": {"encode": el, "rebuild": rl},
        "algorithmic_bytes_per_launch": {"encode": eb1, "rebuild": rb1, "mean": (eb + rb) // (el + rl)},
        "traffic_per_launch": {"encode": t_enc, "rebuild": t_reb},
        "traffic_source": traffic_source(args.traffic_json),
        "avg_launch_ms": {"encode": round(enc_ms / el, 4), "rebuild": round(reb_ms / rl, 4)},
    }
    result["breakdown"] = {
        "encode_GBps": round(eb / (enc_ms * 1e-3) / 1e9, 1),
        "encode_read_GBps": round(enc_plan.bytes_read / (enc_ms * 1e-3) / 1e9, 1),
        "rebuild_GBps": round(rb / (reb_ms * 1e-3) / 1e9, 1),
        # SURVEY.md §8d asks for the median of >= 10 event-timed steps beside the mean
        "step_median_GBps": round(bytes_per_step / (step_ms_median * 1e-3) / 1e9, 1),
        "step_event_ms": {"median": round(step_ms_median, 4), "min": round(min(step_ms), 4),
                          "max": round(max(step_ms), 4)},
    }
    result["round_trip_bit_exact"] = rt_ok
    result["ring_faults"] = ring_faults
    result["hang_faults"] = hang_faults
    result["box_reference"] = {
        "torch_copy_GBps": box_copy,
        "codec_vs_copy": round(achieved / box_copy, 4),
        "note": "same box, same process: device-to-device copy of 1 GiB (read + write bytes)",
    }
    if args.pairs and rank == 0:
        result["rebuild_every_pair"] = rebuild_pairs(codec, lay, chunk, stream)
    if args.xor and rank == 0:
        result["xor"] = xor_leg(args, chunk, stream)
        if args.cpu_baseline and not dist_on:
            result["xor"]["cpu_baseline"] = cpu_baseline_xor(8, 3, args.cpu_seconds / 2, cpu_chunk)
    watchdog = None
    if dist_on:
        # A hung exchange or final barrier cannot raise: a watchdog then
        # prints the main line (with the sharded leg marked timed out) and
        # ends every rank with a non-zero status.
        limit = args.sharded_timeout + (3 * args.cpu_seconds + 60 if args.cpu_baseline else 0)
        watchdog = threading.Timer(limit, sharded_expired, (result, rank, limit))
        watchdog.daemon = True
        watchdog.start()
    if args.sharded:
        # second leg: the multi-rank rebuild with its RCCL exchange (at N=1
        # the world-1 transport). It must not cost the main line: a failure
        # is reported in "sharded" (every rank runs the same collectives, so
        # they fail alike).
        try:
            result["sharded"] = sharded_leg(args, p, e, chunk, lost, world, rank)
        except Exception as exc:  # noqa: BLE001 -- reported, not swallowed
            result["sharded"] = {"error": f"{type(exc).__name__}: {exc}"}
        # configs[3]'s scaling number next to `value`: the
        # exchange-bearing step, where SCALE's reader looks first
        sv = result["sharded"].get("value")
        result["config"]["scaling_value_GBps"] = sv
        result["scaling_value_GBps"] = sv
    if args.cpu_baseline and rank == 0:
        # at N > 1 too, after every collective of the legs and under the
        # watchdog (its limit has the CPU leg's seconds added): the other
        # ranks wait in the final barrier meanwhile
        result["cpu_baseline"] = cpu_baseline(p, e, lost, args.cpu_seconds, cpu_chunk)
        if dist_on and args.xor and "xor" in result:
            result["xor"]["cpu_baseline"] = cpu_baseline_xor(8, 3, args.cpu_seconds / 2, cpu_chunk)
    emit(result, rank)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    if watchdog is not None:
        watchdog.cancel()


if __name__ == "__main__":
    main()
