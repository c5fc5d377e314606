#!/bin/bash
# A/B: plan jobs side by side (REDSET_HIP_SEQUENTIAL=0) vs one after another
# on the whole grid (1, default) or in one launch whose blocks loop over the
# stripes (2); alternating fresh processes. MODES="2 1" picks the orders.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/seq; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2 3; do
  for s in ${MODES:-1 0}; do
    REDSET_HIP_SEQUENTIAL=$s timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $OUT/b.tmp 2>&1 || exit 1
    echo "seq=$s $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/seq/ab.jsonl"):
    tag, js = line.split(" ", 1)
    r = json.loads(js); b = r["breakdown"]
    print(f"{tag}  step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f} (enc {r['xor']['encode_GBps']:7.1f} reb {r['xor']['rebuild_GBps']:7.1f})"
          f"  copy {r['box_reference']['torch_copy_GBps']:7.1f}  rt {r['round_trip_bit_exact']} {r['xor']['round_trip_bit_exact']}")
PY
