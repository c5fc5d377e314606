#!/usr/bin/env python3
"""Per-rank MPI backends at scale (the drop-in REDSET_ENCODE=HIP path): p
ranks under mpirun sharing the box's GPU, each with one data file of
d * chunk bytes, RS encode then rebuild of two lost ranks (rank_test.c =
redset_apply / redset_recover's calling convention). Prints the slowest
rank's time per call and the algorithmic rate ((d+e)*C per stripe encode,
(d+m)*C rebuild, p stripes), and the slot's roofline: what each rank moved
in the call (redset_hip_rank_last_stats: file reads and writes, MPI or
sharded-exchange bytes, H2D / D2H), the time each resource would need at its
ceiling -- PCIe H2D / D2H at the measured DMA rate, host MPI at the rate
tools/mpi_bw measures in the same pattern on the same box -- and the bound:
the resource whose ceiling time is the largest share of the call."""
import argparse
import json
import os
import re
import shutil
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIB = 1 << 20


# the disjoint classes of a call's blocked host time (include/redset_hip_mpi.h)
BLOCKED = ("read_seconds", "mpi_seconds", "gpu_seconds", "write_seconds", "stage_seconds", "copy_seconds",
           "plan_seconds", "setup_seconds")


def roofline(stats, p, mpi_gbps, pcie_gbps, seconds):
    """The slot's roofline for one call: per-rank bytes (max over ranks), the
    time each would take at its resource's ceiling, the share of the call
    that is, and the bound (largest share)."""
    mx = {k: v[0] for k, v in stats.items()}
    mean = {k: v[1] / p for k, v in stats.items()}
    need = {
        "pcie_h2d": mx["h2d_bytes"] / (pcie_gbps * 1e9),
        "pcie_d2h": mx["d2h_bytes"] / (pcie_gbps * 1e9),
    }
    if mpi_gbps:
        need["host_mpi"] = (mx["sent_bytes"] + mx["recv_bytes"]) / (mpi_gbps * 1e9)
    bound = max(need, key=need.get)
    return {
        "bytes_per_rank_max": {k: int(mx[k]) for k in ("read_bytes", "sent_bytes", "recv_bytes", "h2d_bytes",
                                                          "d2h_bytes", "write_bytes")},
        "blocked_seconds_max": {k: round(mx.get(k, 0.0), 4) for k in BLOCKED},
        "blocked_seconds_mean": {k: round(mean.get(k, 0.0), 4) for k in BLOCKED},
        # the host thread's time the disjoint classes explain, summed over the
        # ranks against the ranks' summed call time (redset_hip_rank_last_stats)
        "blocked_coverage": round(sum(stats[k][1] for k in BLOCKED if k in stats) / stats["seconds"][1], 3),
        "call_seconds_max": round(mx["seconds"], 4),
        "exchange_seconds_max": round(mx.get("exchange_seconds", 0.0), 4),
        "ceilings": {"pcie_GBps_per_direction": pcie_gbps, "host_mpi_GBps_per_rank_send_plus_recv": mpi_gbps},
        "seconds_at_ceiling": {k: round(v, 4) for k, v in need.items()},
        "bound": bound,
        "frac": round(need[bound] / seconds, 3),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scheme", choices=["rs", "xor"], default="rs")
    ap.add_argument("--ranks", type=int, default=11)
    ap.add_argument("--encoding", type=int, default=3)
    ap.add_argument("--chunk-mib", type=int, default=16)
    ap.add_argument("--file-bytes", type=int, default=0,
                    help="each rank's data file size instead (chunk = ceil(size / d), the redset rule)")
    ap.add_argument("--buf-mib", type=float, default=1.0)
    ap.add_argument("--lost", default="1,2")
    ap.add_argument("--dir", default="/tmp/rank_bench")
    ap.add_argument("--repeat", type=int, default=1, help="calls per process; the median of calls 2..N is reported as warm")
    ap.add_argument("--exchange", default="auto", help="exchange: auto, host, sharded-mpi, sharded-host, rccl")
    ap.add_argument("--pcie-gbps", type=float, default=55.0,
                    help="PCIe DMA ceiling per direction (profiles/r01_pcie_probe.json: 55-56 GB/s H2D)")
    a = ap.parse_args()
    p, e = a.ranks, (a.encoding if a.scheme == "rs" else 1)
    d = p - e
    C = -(-a.file_bytes // d) if a.file_bytes else a.chunk_mib * MIB
    size = a.file_bytes if a.file_bytes else d * C
    lost = [int(x) for x in a.lost.split(",")][: 1 if a.scheme == "xor" else None]
    shutil.rmtree(a.dir, ignore_errors=True)
    os.makedirs(a.dir)
    block = np.frombuffer(np.random.default_rng(1).bytes(16 * MIB), np.uint8)
    def content(r):
        left, k = size, 0
        while left > 0:
            n = min(left, block.size)
            yield np.roll(block, r * 131 + k)[:n].tobytes()
            left -= n
            k += 1

    for r in range(p):
        path = os.path.join(a.dir, f"r{r}.dat")
        with open(path, "wb") as f:
            for piece in content(r):
                f.write(piece)
        with open(os.path.join(a.dir, f"manifest_{r}.txt"), "w") as f:
            f.write(f"1\n{path} {size}\n{C}\n4096\n{os.path.join(a.dir, f'r{r}.{a.scheme}.redset')}\n")
    drv = os.path.join(ROOT, "tests", "mpi", "build", "rank_test")
    buf = int(a.buf_mib * MIB)
    out = {}
    # host MPI ceiling in the backends' pattern (every rank to every rank at
    # once, one MPI buffer per message), same box, same rank count
    bw = subprocess.run(["/opt/conda/bin/mpirun", "-np", str(p), "-host", "localhost",
                         os.path.join(ROOT, "tools", "mpi_bw"), str(buf), "5"],
                        capture_output=True, text=True, timeout=300)
    mpi_gbps = json.loads(bw.stdout.strip().splitlines()[-1])["per_rank_send_recv_GBps"] if bw.returncode == 0 else None
    for op, extra in (("encode", []), ("rebuild", lost)):
        if op == "rebuild":
            for r in lost:
                os.unlink(os.path.join(a.dir, f"r{r}.dat"))
                os.unlink(os.path.join(a.dir, f"r{r}.{a.scheme}.redset"))
        cmd = ["/opt/conda/bin/mpirun", "-np", str(p), "-host", "localhost", drv, a.scheme, op, str(e), a.dir, str(buf)] + \
            [str(x) for x in extra]
        res = subprocess.run(cmd, capture_output=True, text=True, timeout=900,
                             env={**os.environ, "RANK_TEST_REPEAT": str(a.repeat), "RANK_TEST_EXCHANGE": a.exchange})
        if res.returncode != 0:
            raise SystemExit(res.stdout + res.stderr)
        t = float(re.search(r": ([0-9.]+) s", res.stdout).group(1))
        alg = p * (d + (e if op == "encode" else len(lost))) * C
        out[op] = {"seconds": t, "GBps": round(alg / t / 1e9, 3)}
        warm = re.search(r"\(warm\): ([0-9.]+) s", res.stdout)
        if warm:
            # every call after the first: the median is the warm figure (one
            # box's shared-memory MPI varies by +-20% from call to call)
            calls = [float(x) for x in re.findall(r"call \d+ of \d+(?: \(warm\))?: ([0-9.]+) s", res.stdout)]
            tw = float(np.median(calls))
            out[op].update(warm_seconds=tw, warm_GBps=round(alg / tw / 1e9, 3), warm_calls=calls)
        ex = re.search(op + r" exchange (\S+)", res.stdout)
        if ex:
            out[op]["exchange"] = ex.group(1)
        tag = "warm" if warm else "first"
        st = re.search(r"rank_stats " + tag + r" (\{.*\})", res.stdout)
        if st:
            out[op]["roofline"] = roofline(json.loads(st.group(1)), p, mpi_gbps, a.pcie_gbps,
                                           out[op].get("warm_seconds", t))
    for r in lost:  # the rebuilt files must be the originals
        with open(os.path.join(a.dir, f"r{r}.dat"), "rb") as f:
            if any(f.read(len(piece)) != piece for piece in content(r)) or f.read(1):
                raise SystemExit(f"rank {r}: rebuilt file differs from the original")
    out["rebuilt_equal"] = True
    shutil.rmtree(a.dir, ignore_errors=True)
    print(json.dumps({"scheme": a.scheme, "ranks": p, "encoding": e, "chunk": C, "buf": buf,
                      "host_mpi_GBps_per_rank": mpi_gbps, **out}))


if __name__ == "__main__":
    main()
