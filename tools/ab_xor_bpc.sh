#!/bin/bash
# A/B of resident XOR blocks per CU (REDSET_HIP_XOR_BLOCKS_PER_CU = 1 vs the
# default 2), bench.py's XOR leg (configs[1]); fresh process per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/xorbpc; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2 3; do
  for b in ${XBPC:-1 8}; do
    REDSET_HIP_XOR_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2>&1 || exit 1
    echo "xbpc=$b $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/xorbpc/ab.jsonl"):
    t, js = line.split(" ", 1)
    r = json.loads(js); x = r["xor"]
    print(f"{t:7s} xor {x['value']:7.1f} (enc {x['encode_GBps']:7.1f} reb {x['rebuild_GBps']:7.1f})  rs step {r['value']:7.1f}"
          f"  copy {r['box_reference']['torch_copy_GBps']:7.1f}  rt {x['round_trip_bit_exact']}")
PY
