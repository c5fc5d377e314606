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


def host_case(p, e, chunk, lost, slice_bytes, threads, mode="zero copy"):
    """mode: "zero copy" (kernels read/write the page-locked cells over PCIe),
    "direct DMA" (staged pipeline, SDMA straight from/to the page-locked cells)
    or "staged" (read/write callbacks through pinned staging buffers)."""
    pinned = mode != "staged"
    if mode == "direct DMA":
        # the staged pipeline over mapped cells is a test-twin knob (the
        # product takes zero copy whenever every cell is mapped)
        os.environ["REDSET_HIP_ZERO_COPY"] = "0"
        os.environ.setdefault("REDSET_HIP_LIBRARY", os.path.join(ROOT, "redset_amd", "lib_test", "libredset_hip.so"))
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
    out.append({"case": f"host encode ({mode})", "ranks": p, "encoding": e, "chunk": chunk, "GBps": alg / enc["seconds"] / 1e9,
                "stats": enc, "setup_s": setup})
    # the lost members' regions (data + parity cells) are what the rebuild
    # must restore: snapshot them, erase, rebuild, compare
    ref = [buf[r * per:(r + 1) * per].clone() for r in lost]
    for r in lost:
        buf[r * per:(r + 1) * per].fill_(0xEE)
    reb = stream.rs_rebuild_stream(codec, lost, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    alg_r = p * (d + len(lost)) * chunk
    ok = all(bool(torch.equal(buf[r * per:(r + 1) * per], x)) for r, x in zip(lost, ref))
    out.append({"case": f"host rebuild ({mode})", "ranks": p, "encoding": e,
                "chunk": chunk, "lost": lost, "GBps": alg_r / reb["seconds"] / 1e9, "stats": reb,
                "round_trip_equal": ok})
    return out


def _drop_cache(paths):
    """fsync + POSIX_FADV_DONTNEED: the next read of these files comes from the
    device, not the page cache (no root needed)."""
    for path in paths:
        fd = os.open(path, os.O_RDONLY)
        try:
            os.fsync(fd)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        finally:
            os.close(fd)


def _crc(path):
    import zlib

    crc = 0
    with open(path, "rb") as f:
        while True:
            b = f.read(64 * MIB)
            if not b:
                return crc
            crc = zlib.crc32(b, crc)


def disk_case(p, e, chunk, lost, slice_bytes, threads, directory, short_mib, cold):
    """Disk to disk (BASELINE.json configs[4]): member r's logical file is one
    data file, member 0's exactly d*chunk bytes (so redset's chunk rule,
    ceil(max/d), gives `chunk`), the others `short_mib` MiB shorter (redset
    pads them with zeros, src/redset_lofi.c:30-173; keeps the set within the
    box's scratch disk). Redundancy files = 4 KiB header + e*chunk. cold: the
    inputs are fsynced and dropped from the page cache before the encode, the
    survivors before the rebuild. Times include fsync of what is written."""
    import numpy as np
    import redset_amd
    from redset_amd import stream

    d = p - e
    os.makedirs(directory, exist_ok=True)
    rng = np.random.default_rng(3)
    block = np.frombuffer(rng.bytes(64 * MIB), np.uint8)
    files, reds, headers = [], [], []
    t0 = time.time()
    for r in range(p):
        path = os.path.join(directory, f"ckpt_rank{r}.dat")
        size = d * chunk - (0 if r == 0 else short_mib * MIB + 4096 * r)
        with open(path, "wb") as f:
            left, k = size, 0
            while left > 0:
                n = min(left, block.size)
                f.write(np.roll(block, r * 977 + k * 131)[:n].tobytes())
                left -= n
                k += 1
        files.append([(path, size)])
        reds.append(os.path.join(directory, f"ckpt_rank{r}.rs.redset"))
        headers.append(4096)
    write_s = time.time() - t0
    assert stream.chunk_size_for(max(f[0][1] for f in files), d) == chunk
    data_bytes = sum(f[0][1] for f in files)
    if cold:
        _drop_cache([f[0][0] for f in files])
    codec = redset_amd.RSCodec(p, e)
    io = stream.FileIO(files, reds, headers, chunk)
    t0 = time.time()
    enc = stream.rs_encode_stream(codec, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    io.close()  # fsync + close
    t_enc = time.time() - t0
    alg = p * (d + e) * chunk
    cache = "cold (fsync + POSIX_FADV_DONTNEED before the call)" if cold else "warm (page cache)"
    out = [{"case": "disk encode", "ranks": p, "encoding": e, "chunk": chunk, "GBps": alg / t_enc / 1e9,
            "file_GBps": (data_bytes + p * e * chunk) / t_enc / 1e9, "data_file_bytes": data_bytes,
            "pipeline_seconds": enc["seconds"], "with_fsync_seconds": t_enc, "stats": enc, "cache": cache,
            "files_written_s": write_s, "dir": directory}]
    crcs = {files[r][0][0]: _crc(files[r][0][0]) for r in lost}
    crcs.update({reds[r]: _crc(reds[r]) for r in lost})
    for r in lost:
        os.unlink(files[r][0][0])
        os.unlink(reds[r])
    if cold:
        _drop_cache([files[r][0][0] for r in range(p) if r not in lost] + [reds[r] for r in range(p) if r not in lost])
    io = stream.FileIO(files, reds, headers, chunk, writable=[r in lost for r in range(p)])
    t0 = time.time()
    reb = stream.rs_rebuild_stream(codec, lost, chunk, io, slice_bytes=slice_bytes, io_threads=threads)
    io.close()
    t_reb = time.time() - t0
    alg_r = p * (d + len(lost)) * chunk
    ok = all(_crc(files[r][0][0]) == crcs[files[r][0][0]] and os.path.getsize(files[r][0][0]) == files[r][0][1]
             for r in lost)
    # whole redundancy files (the 4 KiB header region is a hole of zeros in
    # both: this tool writes no header bytes)
    ok_par = all(_crc(reds[r]) == crcs[reds[r]] for r in lost)
    out.append({"case": "disk rebuild", "ranks": p, "encoding": e, "chunk": chunk, "lost": lost,
                "GBps": alg_r / t_reb / 1e9, "pipeline_seconds": reb["seconds"], "with_fsync_seconds": t_reb,
                "stats": reb, "cache": cache, "round_trip_equal": bool(ok and ok_par),
                "data_files_equal": bool(ok), "redundancy_files_equal": bool(ok_par)})
    return out, files, reds, headers


def cpu_disk_case(p, e, chunk, files, reds, headers, stripes, threads, cold):
    """CPU baseline beside the disk case, same files: the reference's CPU
    path for `stripes` stripes -- read each stripe's d data cells through the
    logical-file rules (zero padding past EOF), redset_rs_reduce_buffer_multadd
    for every (parity row, data cell) pair split over `threads` threads in 1 MiB
    slices (the pthreads backend's job split, src/redset_reedsolomon_pthreads.c:
    459-499, as restated in oracle/), pwrite the e parity cells after the
    header, fsync. A bounded sample: `stripes` of the p stripes."""
    import threading

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    import redset_amd

    d = p - e
    codec = redset_amd.RSCodec(p, e)
    mat = codec.matrix()
    st = oracle_lib.OracleRS(p, e)
    if cold:
        _drop_cache([f[0][0] for f in files])
    t_read = t_comp = t_write = 0.0
    mismatches = [0]  # CPU parity bytes that differ from what the GPU pipeline wrote
    for c in stripes:
        t0 = time.time()
        ins, coefs, outs = [], [], []
        for s in range(p):
            enc = codec.encoding_id(s, c)
            if enc < p:
                k = codec.data_id(s, c)
                buf = np.zeros(chunk, np.uint8)
                path, size = files[s][0]
                lo = k * chunk
                n = max(0, min(chunk, size - lo))
                if n:
                    with open(path, "rb") as f:
                        f.seek(lo)
                        f.readinto(memoryview(buf)[:n])
                ins.append((s, buf))
            else:
                outs.append((s, enc - p))
        t1 = time.time()
        res = {key: np.zeros(chunk, np.uint8) for key in outs}
        tc0 = time.time()
        jobs = []
        for (s, i) in outs:
            for (sd, buf) in ins:
                jobs.append((res[(s, i)], int(mat[p + i, sd]), buf))
        sl = MIB
        nsl = (chunk + sl - 1) // sl

        def work(t):
            for q in range(t, nsl, threads):
                a, b = q * sl, min(chunk, (q + 1) * sl)
                for acc, coef, src in jobs:
                    st.multadd(acc[a:b], coef, src[a:b])

        th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        tc1 = time.time()
        # untimed: the GPU pipeline's parity of this stripe, already in the files
        for (s, i), acc in res.items():
            with open(reds[s], "rb") as f:
                f.seek(headers[s] + i * chunk)
                mismatches[0] += int(np.count_nonzero(np.frombuffer(f.read(chunk), np.uint8) != acc))
        t2 = time.time()
        for (s, i), acc in res.items():
            with open(reds[s], "r+b") as f:
                f.seek(headers[s] + i * chunk)
                f.write(acc.tobytes())
                f.flush()
                os.fsync(f.fileno())
        t3 = time.time()
        t_read += t1 - t0
        t_comp += tc1 - tc0
        t_write += t3 - t2
    alg = len(stripes) * p * chunk  # (d + e) cells per stripe
    tot = t_read + t_comp + t_write
    return {"case": "cpu disk encode (port)", "ranks": p, "encoding": e, "chunk": chunk, "stripes": list(stripes),
            "threads": threads, "GBps": alg / tot / 1e9, "read_s": t_read, "compute_s": t_comp, "write_s": t_write,
            "compute_GBps": alg / t_comp / 1e9, "cache": "cold" if cold else "warm",
            "parity_equal_to_gpu": mismatches[0] == 0,
            "sample": f"{len(stripes)} of {p} stripes; oracle multadd (premult table) over 1 MiB slices"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["host", "disk", "both"], default="both")
    ap.add_argument("--ranks", type=int, default=20)
    ap.add_argument("--encoding", type=int, default=4)
    ap.add_argument("--chunk-mib", type=int, default=256)
    ap.add_argument("--disk-chunk-mib", type=int, default=256)
    ap.add_argument("--short-mib", type=int, default=2048,
                    help="disk case: members 1..p-1 write this much less than d*chunk (zero padded)")
    ap.add_argument("--slice-mib", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--cpu-threads", type=int, default=10)
    ap.add_argument("--cpu-stripes", default="0,1")
    ap.add_argument("--cold", type=int, default=1)
    ap.add_argument("--lost", default="1,2")
    ap.add_argument("--dir", default="/tmp/redset_e2e")
    a = ap.parse_args()
    lost = [int(x) for x in a.lost.split(",")]
    res = []
    if a.mode in ("host", "both"):
        for mode in ("zero copy", "direct DMA", "staged"):
            for r in host_case(a.ranks, a.encoding, a.chunk_mib * MIB, lost, a.slice_mib * MIB, a.threads, mode):
                print(json.dumps(r), flush=True)
    if a.mode in ("disk", "both"):
        out, files, reds, headers = disk_case(a.ranks, a.encoding, a.disk_chunk_mib * MIB, lost, a.slice_mib * MIB,
                                              a.threads, a.dir, a.short_mib, bool(a.cold))
        for r in out:
            print(json.dumps(r), flush=True)
        stripes = [int(x) for x in a.cpu_stripes.split(",") if x != ""]
        if stripes:
            print(json.dumps(cpu_disk_case(a.ranks, a.encoding, a.disk_chunk_mib * MIB, files, reds, headers,
                                           stripes, a.cpu_threads, bool(a.cold))), flush=True)
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
