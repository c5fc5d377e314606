# in-kernel stripe loop (REDSET_HIP_SEQUENTIAL=2) vs launch per stripe, with the wait fix
mkdir -p gpurun_out/r03s34
timeout -k 10 900 bash tools/ab_env_seq.sh > gpurun_out/r03s34/seq.txt 2>&1; s=$?
python3 - <<'PY'
import json
for line in open("gpurun_out/seq/ab.jsonl"):
    t, js = line.split(" ", 1); r = json.loads(js); b = r["breakdown"]
    print(f"{t} step {r['value']:7.1f} encode {b['encode_GBps']:7.1f} rebuild {b['rebuild_GBps']:7.1f} xor {r['xor']['value']:7.1f} rt {r['round_trip_bit_exact']} faults {r['ring_faults']}")
PY
exit $s
