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
import sys


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
    with open(sys.argv[3], "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
