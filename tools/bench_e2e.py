#!/usr/bin/env python3
"""End-to-end (host-resident) RS encode + rebuild rates through the pinned
streaming pipeline, for DESIGN.md (BASELINE.json config 5: RS(16+4)).

  host : cells in page-locked host memory (torch pin_memory) -> pinned staging
         -> HBM -> back; the PCIe-inclusive rate.
  disk : cells in files under --dir (redset logical files + redundancy files
         after a header), disk-to-disk including fsync of what is written.
Prints one JSON object per measurement.
"""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MIB = 1 << 20


def host_case(p, e, chunk, lost, slice_bytes, threads, pinned=True):
    import torch
    import redset_amd
    from redset_amd import stream

    d = p - e
    per = (d + e) * chunk
    t0 = time.time()
    buf = torch.empty(p * per, dtype=torch.uint8, pin_memory=True)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    step = 1 << 30
    for off in range(0, p * per, step):
        n = min(step, p * per - off)
        buf[off:off + n].copy_(torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g))
    setup = time.time() - t0
    base = buf.data_ptr()
    lofi = [base + r * per for r in range(p)]
    parity = [base + r * per + d * chunk for r in range(p)]
    io = stream.HostIO(p, lofi, parity, chunk, keepalive=(buf,), pinned=pinned)
    codec = redset_amd.RSCodec(p, e)
    out = []
    enc = stream.rs_encode_stream(codec, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    alg = p * (d + e) * chunk
    out.append({"case": "host encode" + (" (direct DMA)" if pinned else " (staged)"), "ranks": p, "encoding": e, "chunk": chunk, "GBps": alg / enc["seconds"] / 1e9,
                "stats": enc, "setup_s": setup})
    ref = buf[:per * p].clone() if p * per <= (64 << 30) else None
    for r in lost:
        buf[r * per:(r + 1) * per].zero_()
    reb = stream.rs_rebuild_stream(codec, lost, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    alg_r = p * (d + len(lost)) * chunk
    ok = bool(torch.equal(buf, ref)) if ref is not None else None
    out.append({"case": "host rebuild" + (" (direct DMA)" if pinned else " (staged)"), "ranks": p, "encoding": e, "chunk": chunk, "lost": lost,
                "GBps": alg_r / reb["seconds"] / 1e9, "stats": reb, "round_trip_equal": ok})
    return out


def disk_case(p, e, chunk, lost, slice_bytes, threads, directory):
    import numpy as np
    import redset_amd
    from redset_amd import stream

    d = p - e
    os.makedirs(directory, exist_ok=True)
    rng = np.random.default_rng(3)
    block = rng.integers(0, 256, 64 * MIB, dtype=np.uint8)
    files, reds, headers = [], [], []
    t0 = time.time()
    for r in range(p):
        path = os.path.join(directory, f"ckpt_rank{r}.dat")
        size = d * chunk - 4096 * r  # ragged sizes: the logical files get zero padding
        with open(path, "wb") as f:
            left = size
            while left > 0:
                n = min(left, block.size)
                f.write(np.roll(block, r * 977)[:n].tobytes())
                left -= n
        files.append([(path, size)])
        reds.append(os.path.join(directory, f"ckpt_rank{r}.rs.redset"))
        headers.append(4096)
    write_s = time.time() - t0
    codec = redset_amd.RSCodec(p, e)
    io = stream.FileIO(files, reds, headers, chunk)
    t0 = time.time()
    enc = stream.rs_encode_stream(codec, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    io.close()  # fsync + close
    t_enc = time.time() - t0
    alg = p * (d + e) * chunk
    out = [{"case": "disk encode", "ranks": p, "encoding": e, "chunk": chunk, "GBps": alg / t_enc / 1e9,
            "pipeline_seconds": enc["seconds"], "with_fsync_seconds": t_enc, "stats": enc,
            "files_written_s": write_s, "dir": directory}]
    for r in lost:
        os.unlink(files[r][0][0])
        os.unlink(reds[r])
    io = stream.FileIO(files, reds, headers, chunk, writable=[r in lost for r in range(p)])
    t0 = time.time()
    reb = stream.rs_rebuild_stream(codec, lost, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    io.close()
    t_reb = time.time() - t0
    alg_r = p * (d + len(lost)) * chunk
    out.append({"case": "disk rebuild", "ranks": p, "encoding": e, "chunk": chunk, "lost": lost,
                "GBps": alg_r / t_reb / 1e9, "pipeline_seconds": reb["seconds"], "with_fsync_seconds": t_reb,
                "stats": reb})
    shutil.rmtree(directory, ignore_errors=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["host", "disk", "both"], default="both")
    ap.add_argument("--ranks", type=int, default=20)
    ap.add_argument("--encoding", type=int, default=4)
    ap.add_argument("--chunk-mib", type=int, default=256)
    ap.add_argument("--disk-chunk-mib", type=int, default=64)
    ap.add_argument("--slice-mib", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--lost", default="1,2")
    ap.add_argument("--dir", default="/tmp/redset_e2e")
    a = ap.parse_args()
    lost = [int(x) for x in a.lost.split(",")]
    res = []
    if a.mode in ("host", "both"):
        res += host_case(a.ranks, a.encoding, a.chunk_mib * MIB, lost, a.slice_mib * MIB, a.threads, pinned=True)
        res += host_case(a.ranks, a.encoding, a.chunk_mib * MIB, lost, a.slice_mib * MIB, a.threads, pinned=False)
    if a.mode in ("disk", "both"):
        res += disk_case(a.ranks, a.encoding, a.disk_chunk_mib * MIB, lost, a.slice_mib * MIB, a.threads, a.dir)
    for r in res:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
