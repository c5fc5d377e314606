#!/bin/bash
# Does the bench number depend on how long the HBM has been under load?
# Prints the clocks, then the same bench at increasing warm-up lengths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/warm; mkdir -p $OUT
(rocm-smi --showclocks; rocm-smi --showpower --showtemp) > $OUT/smi_before.txt 2>&1 || true
for W in 3 3 100 400 3; do
  timeout -k 10 200 python bench.py --steps 50 --warmup $W --xor 0 --cpu-baseline 0 > $OUT/w$W.json 2>/dev/null || exit $?
  python - $OUT/w$W.json $W <<'PY'
import json,sys; r=json.load(open(sys.argv[1])); b=r["breakdown"]
print(f"warmup {sys.argv[2]:>4}: step {r['value']:.0f}  encode {b['encode_GBps']:.0f}  rebuild {b['rebuild_GBps']:.0f}")
PY
done | tee $OUT/summary.txt
(rocm-smi --showclocks) > $OUT/smi_after.txt 2>&1 || true
