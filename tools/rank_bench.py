#!/usr/bin/env python3
"""Per-rank MPI backends at scale (the drop-in REDSET_ENCODE=HIP path): p
ranks under mpirun sharing the box's GPU, each with one data file of
d * chunk bytes, RS encode then rebuild of two lost ranks (rank_test.c =
redset_apply / redset_recover's calling convention). Prints the slowest
rank's time per call and the algorithmic rate ((d+e)*C per stripe encode,
(d+m)*C rebuild, p stripes)."""
import argparse
import json
import os
import re
import shutil
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIB = 1 << 20


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
    ap.add_argument("--repeat", type=int, default=1, help="calls per process; the last one is reported as warm")
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
    for op, extra in (("encode", []), ("rebuild", lost)):
        if op == "rebuild":
            for r in lost:
                os.unlink(os.path.join(a.dir, f"r{r}.dat"))
                os.unlink(os.path.join(a.dir, f"r{r}.{a.scheme}.redset"))
        cmd = ["/opt/conda/bin/mpirun", "-np", str(p), "-host", "localhost", drv, a.scheme, op, str(e), a.dir, str(buf)] + \
            [str(x) for x in extra]
        res = subprocess.run(cmd, capture_output=True, text=True, timeout=900,
                             env={**os.environ, "RANK_TEST_REPEAT": str(a.repeat)})
        if res.returncode != 0:
            raise SystemExit(res.stdout + res.stderr)
        t = float(re.search(r": ([0-9.]+) s", res.stdout).group(1))
        alg = p * (d + (e if op == "encode" else len(lost))) * C
        out[op] = {"seconds": t, "GBps": round(alg / t / 1e9, 3)}
        warm = re.search(r"\(warm\): ([0-9.]+) s", res.stdout)
        if warm:
            tw = float(warm.group(1))
            out[op].update(warm_seconds=tw, warm_GBps=round(alg / tw / 1e9, 3))
    for r in lost:  # the rebuilt files must be the originals
        with open(os.path.join(a.dir, f"r{r}.dat"), "rb") as f:
            if any(f.read(len(piece)) != piece for piece in content(r)) or f.read(1):
                raise SystemExit(f"rank {r}: rebuilt file differs from the original")
    out["rebuilt_equal"] = True
    shutil.rmtree(a.dir, ignore_errors=True)
    print(json.dumps({"scheme": a.scheme, "ranks": p, "encoding": e, "chunk": C, "buf": buf, **out}))


if __name__ == "__main__":
    main()
