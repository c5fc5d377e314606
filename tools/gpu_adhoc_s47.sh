# default = claimed encode + streamed-pair rebuild: full session, then A/B against all-pairs and all-claimed
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh r03s47 || exit $?
OUT=gpurun_out/r03s47; rm -f $OUT/ab.jsonl
for r in 1 2 3; do
  for m in "def x" "3 2" "4 0"; do
    set -- $m
    if [ $1 = def ]; then unset REDSET_HIP_SEQUENTIAL REDSET_HIP_STREAM_JOBS; else export REDSET_HIP_SEQUENTIAL=$1 REDSET_HIP_STREAM_JOBS=$2; fi
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2> $OUT/b.err || exit 1
    echo "$1/$2 $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
unset REDSET_HIP_SEQUENTIAL REDSET_HIP_STREAM_JOBS
python3 - <<'PY'
import json
for line in open("gpurun_out/r03s47/ab.jsonl"):
    t, js = line.split(" ", 1); r = json.loads(js); b = r["breakdown"]
    print(f"{t:6s} step {r['value']:7.1f} encode {b['encode_GBps']:7.1f} rebuild {b['rebuild_GBps']:7.1f} xor {r['xor']['value']:7.1f} rt {r['round_trip_bit_exact']} faults {r['ring_faults']}")
PY
