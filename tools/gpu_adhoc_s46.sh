# claimed order as the default (+ batched FREE check): full session, then A/B of the claimed kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh r03s46 || exit $?
OUT=gpurun_out/r03s46; rm -f $OUT/ab.jsonl
for r in 1 2 3; do
  for m in "new 4 0" "prev 4 0" "new 3 2"; do
    set -- $m
    if [ $1 = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/abx/lib_$1.so; fi
    REDSET_HIP_SEQUENTIAL=$2 REDSET_HIP_STREAM_JOBS=$3 timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2> $OUT/b.err || exit 1
    echo "$1/seq$2/sj$3 $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/r03s46/ab.jsonl"):
    t, js = line.split(" ", 1); r = json.loads(js); b = r["breakdown"]
    print(f"{t:14s} step {r['value']:7.1f} encode {b['encode_GBps']:7.1f} rebuild {b['rebuild_GBps']:7.1f} xor {r['xor']['value']:7.1f} rt {r['round_trip_bit_exact']} faults {r['ring_faults']}")
PY
