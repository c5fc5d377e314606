#!/bin/bash
# Mid-size cells: stripes side by side (g=all) vs in sequence g per launch
# (REDSET_HIP_SEQUENTIAL=1, REDSET_HIP_STRIPES_PER_LAUNCH=g); fresh process per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/grpchunk; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2; do
  for cg in ${CGS:-16:0 16:2 16:3 8:0 8:3 8:4 8:6 4:0 4:6 24:0 24:1 24:2}; do
    c=${cg%%:*}; g=${cg##*:}
    if [ $g = 0 ]; then s=0; g=1; else s=1; fi
    REDSET_HIP_SEQUENTIAL=$s REDSET_HIP_STRIPES_PER_LAUNCH=$g timeout -k 10 120 python bench.py --steps 40 --warmup 5 \
      --cpu-baseline 0 --pairs 0 --xor 0 --chunk-mib $c > $OUT/b.tmp 2>&1 || exit 1
    echo "chunk=$c seq=$s/g=$g $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/grpchunk/ab.jsonl"):
    t1, t2, js = line.split(" ", 2)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t1:9s} {t2:9s} step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  launches {r['roofline']['launches_per_step']['encode']}")
PY
