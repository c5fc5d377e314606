# XOR streamed pairs on/off A/B, then the full session
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03s42; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2 3; do
  for m in 1 0; do
    REDSET_HIP_XOR_STREAM=$m timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2> $OUT/b.err || exit 1
    echo "xorstream$m $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/r03s42/ab.jsonl"):
    t, js = line.split(" ", 1); r = json.loads(js); b = r["breakdown"]; x = r["xor"]
    print(f"{t:11s} step {r['value']:7.1f} encode {b['encode_GBps']:7.1f} rebuild {b['rebuild_GBps']:7.1f} xor {x['value']:7.1f} (enc {x['encode_GBps']:7.1f} reb {x['rebuild_GBps']:7.1f}) rt {r['round_trip_bit_exact']} {x['round_trip_bit_exact']} faults {r['ring_faults']}")
PY
bash tools/gpu_session.sh r03s42s
