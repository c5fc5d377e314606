# claimed order: claimer look-ahead 2 (in-tree) / 4 / 8 batches, against streamed pairs (the default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03s44; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2; do
  for m in "3 new" "4 new" "4 b4l4" "4 b4l8"; do
    set -- $m
    if [ $2 = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/abx/lib_$2.so; fi
    REDSET_HIP_SEQUENTIAL=$1 REDSET_HIP_STREAM_JOBS=$([ $1 = 3 ] && echo 2 || echo 0) timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2> $OUT/b.err || exit 1
    echo "seq$1/$2 $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/r03s44/ab.jsonl"):
    t, js = line.split(" ", 1); r = json.loads(js); b = r["breakdown"]
    print(f"{t:12s} step {r['value']:7.1f} encode {b['encode_GBps']:7.1f} rebuild {b['rebuild_GBps']:7.1f} xor {r['xor']['value']:7.1f} rt {r['round_trip_bit_exact']} faults {r['ring_faults']}")
PY
