#!/bin/bash
# blocks-per-CU x cell padding with sequential job launches (fresh process each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/seqsweep; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2; do
  for b in ${BPC_LIST:-1 2 3 4}; do
    for pad in ${PADS:-0 16}; do
      REDSET_HIP_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --cell-pad-mib $pad > $OUT/b.tmp 2>&1 || exit 1
      echo "bpc=$b pad=$pad $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
    done
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/seqsweep/ab.jsonl"):
    t1, t2, js = line.split(" ", 2)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t1} {t2:6s} step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  copy {r['box_reference']['torch_copy_GBps']:7.1f}")
PY
