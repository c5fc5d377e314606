#!/bin/bash
# A/B of library builds x blocks per CU: CFGS="lib:bpc ..." (lib "new" = the
# in-tree build, else ab/lib_<lib>.so); fresh process per run, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/libs; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2; do
  for cfg in $CFGS; do
    lib=${cfg%%:*}; b=${cfg##*:}
    if [ $lib = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/ab/lib_$lib.so; fi
    REDSET_HIP_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2>&1 || exit 1
    echo "$lib bpc=$b $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/libs/ab.jsonl"):
    t1, t2, js = line.split(" ", 2)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t1:5s} {t2}  step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  copy {r['box_reference']['torch_copy_GBps']:7.1f}  rt {r['round_trip_bit_exact']}")
PY
