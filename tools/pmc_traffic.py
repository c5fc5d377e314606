#!/usr/bin/env python3
"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into HBM bytes per
launch of each kernel, with the gfx950 corrections of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): sizes are in KiB;
FETCH_SIZE counts exactly half of a wide coalesced streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json
"""
import csv
import glob
import json
import os
import re
import socket
import sys
import time


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    sums, counts = {}, {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"]
                m = re.search(r"(\w+<[^>]*>)", name) if "redset_hip" in name else None
                key = m.group(1) if m else name[:60]
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                sums[key] = sums.get(key, 0.0) + float(row["Counter_Value"])
                counts.setdefault(key, set()).add(disp)
    return {k: sums[k] / max(1, len(counts[k])) for k in sums}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in fetch:
        if k in write:
            out[k] = int((2.0 * fetch[k] + write[k]) * 1024)
            out[k + ":detail"] = {"FETCH_SIZE_KiB_raw": fetch[k], "fetch_bytes_corrected": int(2 * fetch[k] * 1024),
                                  "WRITE_SIZE_KiB": write[k], "write_bytes": int(write[k] * 1024)}
    # where these bytes were measured: the session (gpurun_out/<session>/...),
    # the box and the date -- bench.py names them in its traffic_source
    parts = os.path.normpath(os.path.abspath(sys.argv[1])).split(os.sep)
    session = parts[parts.index("gpurun_out") + 1] if "gpurun_out" in parts[:-1] else os.path.basename(sys.argv[1])
    out["_provenance"] = {"session": session, "host": socket.gethostname(),
                          "date": time.strftime("%Y-%m-%d %H:%M:%S %Z"),
                          "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate runs of "
                                    "bench.py --steps 4 --warmup 1 on that box"}
    with open(sys.argv[3], "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
