#!/bin/bash
# Where does one launch per stripe start to pay? RS(8+3) step at several cell
# sizes with stripes side by side (REDSET_HIP_SEQUENTIAL=0) vs in sequence (1);
# fresh process per run, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/seqchunk; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2; do
  for c in ${CHUNKS:-1 4 8 16 32}; do
    for s in 0 1; do
      REDSET_HIP_SEQUENTIAL=$s timeout -k 10 120 python bench.py --steps 40 --warmup 5 --cpu-baseline 0 --pairs 0 --xor 0 \
        --chunk-mib $c > $OUT/b.tmp 2>&1 || exit 1
      echo "chunk=$c seq=$s $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
    done
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/seqchunk/ab.jsonl"):
    t1, t2, js = line.split(" ", 2)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t1:9s} {t2}  step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  launches {r['roofline']['launches_per_step']['encode']}")
PY
