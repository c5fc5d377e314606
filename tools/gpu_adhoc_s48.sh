# loaders publish with every lane (puball) vs lane 0 (in-tree), default orders and a launch per stripe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03s48; mkdir -p $OUT; rm -f $OUT/ab.jsonl
REDSET_HIP_LIBRARY=$PWD/abx/lib_puball.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_puball.log 2>&1; s=$?; tail -2 $OUT/tests_puball.log; [ $s -eq 0 ] || exit $s
for r in 1 2 3; do
  for m in "new def" "puball def" "new 1" "puball 1"; do
    set -- $m
    if [ $1 = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/abx/lib_$1.so; fi
    if [ $2 = def ]; then unset REDSET_HIP_SEQUENTIAL; else export REDSET_HIP_SEQUENTIAL=$2; fi
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2> $OUT/b.err || exit 1
    echo "$1/$2 $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
unset REDSET_HIP_LIBRARY REDSET_HIP_SEQUENTIAL
python3 - <<'PY'
import json
for line in open("gpurun_out/r03s48/ab.jsonl"):
    t, js = line.split(" ", 1); r = json.loads(js); b = r["breakdown"]
    print(f"{t:11s} step {r['value']:7.1f} encode {b['encode_GBps']:7.1f} rebuild {b['rebuild_GBps']:7.1f} xor {r['xor']['value']:7.1f} rt {r['round_trip_bit_exact']} faults {r['ring_faults']}")
PY
