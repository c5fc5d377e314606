#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first step that faults / aborts / times out (exit >= 2 or
# signal), per the pool rules; an ordinary test failure (exit 1) continues.
# usage: tools/gpu_session.sh <tag> [pytest-args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ok() { local s=$1; [ "$s" -eq 0 ] || [ "$s" -eq 1 ]; }

echo "== gpu tests" | tee "$OUT/progress.txt"
REDSET_TEST_PROGRESS_DIR="$OUT" timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread "$@" > "$OUT/gpu_tests.log" 2>&1
s=$?; echo "gpu tests exit $s" | tee -a "$OUT/progress.txt"; tail -3 "$OUT/gpu_tests.log"
ok $s || exit $s

echo "== smoke" | tee -a "$OUT/progress.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
s=$?; echo "smoke exit $s" | tee -a "$OUT/progress.txt"; tail -2 "$OUT/smoke.log"
ok $s || exit $s

echo "== bench" | tee -a "$OUT/progress.txt"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
s=$?; echo "bench exit $s" | tee -a "$OUT/progress.txt"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
ok $s || exit $s

echo "== rocprofv3 kernel stats" | tee -a "$OUT/progress.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
  python3 bench.py --steps 20 --warmup 3 --cpu-baseline 0 --pairs 0 > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
s=$?; echo "rocprof exit $s" | tee -a "$OUT/progress.txt"
ok $s || exit $s
echo "== rocprofv3 PMC FETCH_SIZE / WRITE_SIZE (separate passes)" | tee -a "$OUT/progress.txt"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
  python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --pairs 0 > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
s=$?; echo "pmc fetch exit $s" | tee -a "$OUT/progress.txt"; ok $s || exit $s
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write -- \
  python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --pairs 0 > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
s=$?; echo "pmc write exit $s" | tee -a "$OUT/progress.txt"; ok $s || exit $s
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/traffic.json" > /dev/null
echo "== done" | tee -a "$OUT/progress.txt"
echo "== N=2 gloo rehearsal of bench.py --gpus 2 (both ranks on the one GPU)" | tee -a "$OUT/progress.txt"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --chunk-mib 2 --steps 3 --warmup 1 \
  --cpu-baseline 0 --pairs 0 > "$OUT/n2_gloo.json" 2> "$OUT/n2_gloo.err"
s=$?; echo "n2 gloo exit $s" | tee -a "$OUT/progress.txt"; ok $s || exit $s
echo "== done (gloo)" | tee -a "$OUT/progress.txt"
