#!/bin/bash
# A/B of stripes per launch in sequence mode (REDSET_HIP_STRIPES_PER_LAUNCH,
# side by side within a launch): 1 (default), 2, 3; fresh process per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/group; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2; do
  for g in ${GROUPS_LIST:-1 2 3}; do
    REDSET_HIP_STRIPES_PER_LAUNCH=$g timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $OUT/b.tmp 2>&1 || exit 1
    echo "g=$g $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/group/ab.jsonl"):
    t, js = line.split(" ", 1)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t}  step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  copy {r['box_reference']['torch_copy_GBps']:7.1f}  rt {r['round_trip_bit_exact']}")
PY
