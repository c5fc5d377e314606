# claimed order without the per-item position record: correctness (normal + spin-cap twin), then A/B vs streamed pairs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03s45; mkdir -p $OUT; rm -f $OUT/ab.jsonl
REDSET_HIP_SEQUENTIAL=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_digests.py tests/test_gpu_redset_sequence.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_seq4.log 2>&1; s=$?; tail -2 $OUT/tests_seq4.log; [ $s -eq 0 ] || exit $s
REDSET_RING_FALLBACK_RUN=1 REDSET_HIP_LIBRARY=$PWD/redset_amd/lib_spincap/libredset_hip.so REDSET_HIP_SEQUENTIAL=4 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_digests.py tests/test_gpu_redset_sequence.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests_seq4_twin.log 2>&1; s=$?; tail -2 $OUT/tests_seq4_twin.log; [ $s -eq 0 ] || exit $s
for r in 1 2 3; do
  for m in 3 4; do
    REDSET_HIP_SEQUENTIAL=$m REDSET_HIP_STREAM_JOBS=$([ $m = 3 ] && echo 2 || echo 0) timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > $OUT/b.tmp 2> $OUT/b.err || exit 1
    echo "seq$m $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/r03s45/ab.jsonl"):
    t, js = line.split(" ", 1); r = json.loads(js); b = r["breakdown"]
    print(f"{t:6s} step {r['value']:7.1f} encode {b['encode_GBps']:7.1f} rebuild {b['rebuild_GBps']:7.1f} xor {r['xor']['value']:7.1f} rt {r['round_trip_bit_exact']} faults {r['ring_faults']}")
PY
