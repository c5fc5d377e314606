#!/bin/bash
# A short GPU check after a change to the sharded path: the sharded and bench
# tests (full-size digests of configs[3] at world 1, the world-1 runner, the
# bench's N=1 and self-launched N=2 flows), then the N=1 bench without the
# CPU baseline and pair sweep. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}; mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_full_digests.py tests/test_gpu_parity.py tests/test_gpu_bench.py \
  -k "sharded or bench" -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || \
  { tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 > "$OUT/bench.json" 2> "$OUT/bench.err" || \
  { tail -5 "$OUT/bench.err"; exit 2; }
python -c "
import json; d = json.load(open('$OUT/bench.json'))
s = d['sharded']
print('bench', d['value'], d['roofline']['frac'], 'sharded', s['value'], s['frac_of_hbm'], s['bit_exact'], s['compute_hbm'])"
