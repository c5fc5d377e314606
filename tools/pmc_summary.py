#!/usr/bin/env python3
"""Mean per dispatch of every counter in rocprofv3 --pmc output directories,
for the codec kernels (gf_mac / xor), as a table.

usage: pmc_summary.py LABEL=DIR [LABEL=DIR ...]
"""
import csv
import glob
import os
import re
import sys

from collections import defaultdict


def collect(d):
    sums, disp = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                if "redset_hip" not in name:
                    continue
                m = re.search(r"(\w+<[^>]*>)", name)
                k = (m.group(1) if m else name[:40], row["Counter_Name"])
                sums[k] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    return {k: sums[k] / len(disp[k]) for k in sums}


def main():
    rows = {}
    for arg in sys.argv[1:]:
        label, d = arg.split("=", 1)
        for (kern, ctr), v in collect(d).items():
            rows.setdefault((label, kern), {})[ctr] = v
    ctrs = sorted({c for r in rows.values() for c in r})
    print(f"{'build':10s} {'kernel':28s} " + " ".join(f"{c:>22s}" for c in ctrs))
    for (label, kern), r in sorted(rows.items()):
        print(f"{label:10s} {kern:28s} " + " ".join(f"{r.get(c, float('nan')):22,.0f}" for c in ctrs))


if __name__ == "__main__":
    main()
