#!/bin/bash
# A/B of the plans' job order (REDSET_HIP_SEQUENTIAL: 1 = one launch per stripe,
# 2 = one launch whose blocks loop over the stripes, 3 = one launch streaming
# every stripe through one continuous ring), fresh processes, alternating:
# tools/ab_env_seq.sh [modes...] (default: 1 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MODES=${*:-1 2}
OUT=gpurun_out/seq; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2 3; do
  for m in $MODES; do
    REDSET_HIP_SEQUENTIAL=$m timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2> $OUT/b.err || exit 1
    echo "seq$m $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
echo done
