#!/bin/bash
# A/B of environment settings on the in-tree build: ENVS="name:VAR=val,VAR2=val ..." ;
# parity first (GPU tests under each setting), then ROUNDS alternating bench processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/abenv}; mkdir -p $OUT; rm -f $OUT/ab.jsonl
run_env() { local spec=$1; shift; ( IFS=','; for kv in $spec; do export "$kv"; done; "$@" ); }
for cfg in $ENVS; do
  name=${cfg%%:*}; spec=${cfg#*:}
  run_env "$spec" timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_doc_examples.py -k "rs_ or xor_ or job_order or graph or full_size or doc" \
    > $OUT/parity_$name.log 2>&1
  s=$?; echo "$name parity exit $s: $(tail -1 $OUT/parity_$name.log)"; [ $s -eq 0 ] || exit $s
done
for r in $(seq 1 ${ROUNDS:-3}); do
  for cfg in $ENVS; do
    name=${cfg%%:*}; spec=${cfg#*:}
    run_env "$spec" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2>&1 || exit $?
    echo "$name $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    t1, js = line.split(" ", 1)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t1:12s} step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  frac {r['roofline']['frac']}  rt {r['round_trip_bit_exact']}")
PY
