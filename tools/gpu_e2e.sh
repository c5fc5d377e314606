#!/bin/bash
# GPU tests of the streaming pipeline + end-to-end rates. usage: tools/gpu_e2e.sh <tag> [chunk_mib] [disk_chunk_mib]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-e2e}; CH=${2:-64}; DCH=${3:-64}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ok() { local s=$1; [ "$s" -eq 0 ] || [ "$s" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py -m gpu -q -x > "$OUT/gpu_tests.log" 2>&1
s=$?; echo "gpu tests exit $s"; tail -3 "$OUT/gpu_tests.log"; ok $s || exit $s
timeout -k 10 900 python tools/bench_e2e.py --mode both --chunk-mib $CH --disk-chunk-mib $DCH > "$OUT/e2e.jsonl" 2> "$OUT/e2e.err"
s=$?; echo "e2e exit $s"; cat "$OUT/e2e.jsonl"; tail -5 "$OUT/e2e.err"
exit $s
