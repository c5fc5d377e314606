# streamed stripes (REDSET_HIP_SEQUENTIAL=3): parity suites forced to it, then A/B against 1 and 2
mkdir -p gpurun_out/r03s35
REDSET_HIP_SEQUENTIAL=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_digests.py tests/test_gpu_redset_sequence.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s35/tests_seq3.log 2>&1; s=$?; tail -5 gpurun_out/r03s35/tests_seq3.log; [ $s -eq 0 ] || exit $s
timeout -k 10 900 bash tools/ab_env_seq.sh 1 3 2 > gpurun_out/r03s35/seq.txt 2>&1; s=$?
python3 - <<'PY'
import json
for line in open("gpurun_out/seq/ab.jsonl"):
    t, js = line.split(" ", 1); r = json.loads(js); b = r["breakdown"]
    print(f"{t} step {r['value']:7.1f} encode {b['encode_GBps']:7.1f} rebuild {b['rebuild_GBps']:7.1f} xor {r['xor']['value']:7.1f} rt {r['round_trip_bit_exact']} faults {r['ring_faults']}")
PY
exit $s
