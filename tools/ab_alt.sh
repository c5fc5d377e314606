#!/bin/bash
# alternating A/B: in-tree build vs abx/lib_<name>.so (copy variants from ab/,
# which does not travel), fresh process per run: tools/ab_alt.sh <name>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abx; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2 3; do
  for lib in new "$@"; do
    if [ $lib = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/abx/lib_$lib.so; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2>&1 || exit 1
    echo "$lib $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/abx/ab.jsonl"):
    t1, js = line.split(" ", 1)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t1:5s} step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  copy {r['box_reference']['torch_copy_GBps']:7.1f}  rt {r['round_trip_bit_exact']}")
PY
