#!/bin/bash
# A/B of threads per block: in-tree build vs ab/lib_b256.so (256 threads, 2 blocks/CU);
# fresh process per run, three rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/block; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2 3; do
  for lib in new b256; do
    if [ $lib = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/ab/lib_$lib.so; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2>&1 || exit 1
    echo "$lib $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/block/ab.jsonl"):
    t, js = line.split(" ", 1)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t:5s} step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  copy {r['box_reference']['torch_copy_GBps']:7.1f}  rt {r['round_trip_bit_exact']} {r['xor']['round_trip_bit_exact']}")
PY
