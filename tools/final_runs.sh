#!/bin/bash
# N fresh bench processes of the in-tree build with the driver's defaults
# (the spread a single driver run samples from). usage: tools/final_runs.sh <tag> [n]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-final}; mkdir -p "$OUT"; rm -f "$OUT/final_runs.jsonl"
for i in $(seq 1 ${2:-5}); do
  timeout -k 10 300 python bench.py > "$OUT/b.tmp" 2> "$OUT/b.err" || exit $?
  tail -1 "$OUT/b.tmp" >> "$OUT/final_runs.jsonl"
done
python3 - "$OUT/final_runs.jsonl" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    r = json.loads(line); b = r["breakdown"]
    print(f"value {r['value']:7.1f}  frac {r['roofline']['frac']:.4f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  rt {r['round_trip_bit_exact']}  ring_faults {r['ring_faults']}")
PY
