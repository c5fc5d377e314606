#!/bin/bash
# Variant libraries (abx/lib_<name>.so, built by tools/build_ab_variant.sh and
# copied to abx/, which travels) x blocks per CU: CFGS="name:bpc ..." ("new" =
# the in-tree build; bpc 0 = the library's default). For each variant first a
# parity check (GPU tests through REDSET_HIP_LIBRARY), then ROUNDS alternating
# bench processes (main line only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/abcfg}; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for cfg in $CFGS; do
  lib=${cfg%%:*}; b=${cfg##*:}
  [ $lib = new ] && continue
  REDSET_HIP_LIBRARY=$PWD/abx/lib_$lib.so REDSET_HIP_BLOCKS_PER_CU=$b timeout -k 10 300 python -m pytest -x -q \
    --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "rs_encode_set or every_pattern or full_size or doc" \
    tests/test_doc_examples.py > $OUT/parity_${lib}_${b}.log 2>&1
  s=$?; echo "$cfg parity exit $s: $(tail -1 $OUT/parity_${lib}_${b}.log)"; [ $s -eq 0 ] || exit $s
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in $CFGS; do
    lib=${cfg%%:*}; b=${cfg##*:}
    if [ $lib = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/abx/lib_$lib.so; fi
    if [ $b = 0 ]; then unset REDSET_HIP_BLOCKS_PER_CU; else export REDSET_HIP_BLOCKS_PER_CU=$b; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2>&1 || exit $?
    echo "$cfg $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
unset REDSET_HIP_LIBRARY REDSET_HIP_BLOCKS_PER_CU
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    t1, js = line.split(" ", 1)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t1:16s} step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  copy {r['box_reference']['torch_copy_GBps']:7.1f}  rt {r['round_trip_bit_exact']}")
PY
