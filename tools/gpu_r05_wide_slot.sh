#!/bin/bash
# The drop-in slot's RS encode at a wider set than RS(8+3): RS(10+4), 14
# ranks sharing the box's GPU (the box allows 16 GPU processes), 32 MiB
# chunks, host ring against host slabs (tools/rank_bench.py). The ring sends
# d*e = 40 cells per member, the host slabs (d + e)(p - 1)/p = 13.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-wide_slot}; mkdir -p "$OUT"
for ex in host sharded-host; do
  echo "== rs10+4 $ex" | tee -a "$OUT/progress.txt"
  timeout -k 10 400 python tools/rank_bench.py --ranks 14 --encoding 4 --chunk-mib 32 --buf-mib 16 --repeat 5 \
    --lost 1,2,3,4 --exchange $ex --dir /tmp/rank_wide_$ex > "$OUT/rank_rs10p4_$ex.out" 2> "$OUT/rank_rs10p4_$ex.err"
  s=$?; echo "exit $s" | tee -a "$OUT/progress.txt"; [ $s -eq 0 ] || exit $s
  rm -rf /tmp/rank_wide_$ex
done
