"""BASELINE.json configs[0]'s shape end to end through the header path:
XOR, 4 members, one 16 MiB file each (chunk 5,592,406 B). apply_set writes
headers + parity; member 2 is lost; rebuild_set (Python) and
redset_hip_rebuild headers (C) rebuild it from the surviving headers.
Files live in a tmpfs directory so the numbers are the pipeline's, not a
disk's. Prints one JSON line per phase.
usage: python tools/config1_e2e.py [dir] [reps] [slice_bytes]"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from redset_amd import setfiles  # noqa: E402

TOOL = os.path.join(ROOT, "redset_amd", "bin", "redset_hip_rebuild")


def crc(path):
    with open(path, "rb") as f:
        return zlib.crc32(f.read())


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else "/dev/shm"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    sb = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    tmp = tempfile.mkdtemp(prefix="redset_c1_", dir=base)
    try:
        p, size, lost = 4, 16 << 20, 2
        rng = np.random.default_rng(0x5EED)
        files = []
        for r in range(p):
            path = os.path.join(tmp, f"testfile_{r}.out")
            rng.integers(0, 256, size, dtype=np.uint8).tofile(path)
            files.append([path])
        want = {f[0]: crc(f[0]) for f in files}
        setfiles.apply_set("XOR", files, os.path.join(tmp, "ckpt."))  # warm-up (first HIP use)
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            res = setfiles.apply_set("XOR", files, os.path.join(tmp, "ckpt."), slice_bytes=sb)
            t.append(time.perf_counter() - t0)
        reds = res["redundancy"]
        chunk = res["chunk"]
        algo = p * (p - 1) * chunk + p * chunk  # read every member's 3 segments, write 4 parity cells
        print(json.dumps({"phase": "apply_set", "chunk": chunk, "slice_bytes": sb, "median_s": float(np.median(t)),
                          "GBps": algo / float(np.median(t)) / 1e9, "reps": reps}), flush=True)
        for mode in ("rebuild_set", "tool_headers"):
            t = []
            for _ in range(reps):
                os.unlink(files[lost][0])
                os.unlink(reds[lost])
                t0 = time.perf_counter()
                if mode == "rebuild_set":
                    out = setfiles.rebuild_set(reds, slice_bytes=sb)
                    ok = out["ok"] and out["missing"] == [lost]
                else:
                    r = subprocess.run([TOOL, "headers", *reds], capture_output=True, text=True, timeout=120)
                    ok = r.returncode == 0 and json.loads(r.stdout)["missing"] == [lost]
                t.append(time.perf_counter() - t0)
                assert ok, mode
                assert all(crc(f) == c for f, c in want.items()), mode
            # survivors' files and parity in, the lost file and its parity out: 16 C
            algo = (p - 1) * (p - 1) * chunk + (p - 1) * chunk + (p - 1) * chunk + chunk
            print(json.dumps({"phase": mode, "slice_bytes": sb, "median_s": float(np.median(t)), "GBps": algo / float(np.median(t)) / 1e9,
                              "reps": reps, "crc_ok": True}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
