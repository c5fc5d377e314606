#!/bin/bash
# widths check + RS(16+4) device-resident bench A/B (memory skeleton, ring size)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIBS="FD2 FD3 new" ROUNDS=1 GF3="1 2 9 10 11 12" GF2="16" XW="9 10 11 12 13 14 15 16" bash tools/ab_probe_widths.sh || exit 1
cp gpurun_out/widths.jsonl gpurun_out/widths_check.jsonl
BENCH_ARGS="--ranks 20 --encoding 4 --lost 1,2,3,4 --xor 0" LIBS="new memonly kib144" ROUNDS=2 bash tools/ab_abx.sh > /dev/null 2>&1
cp gpurun_out/abx/ab.jsonl gpurun_out/rs164_bench.jsonl
echo done
