#!/bin/bash
# Round 6's GPU session: the round's new tests first (the RCCL transport at
# world > 1 over tests/rcclstub, the partial-sum shape with the HIP combine
# plans, the bench's N > 1 line), then, unless NEW_ONLY is set, the whole GPU
# suite with per-test durations, smoke, the driver's
# bench command, a rocprofv3 kernel-stats run and separate PMC FETCH_SIZE /
# WRITE_SIZE passes. Stops at the first step that faults / aborts / times
# out. usage: gpu_r06_check.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06check}; mkdir -p "$OUT"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
echo "== new tests" | tee "$OUT/progress.txt"
timeout -k 10 900 $PYT --durations=0 tests/test_gpu_rccl_stub.py tests/test_gpu_bench.py > "$OUT/new_tests.log" 2>&1
s=$?; echo "new tests exit $s" | tee -a "$OUT/progress.txt"; tail -5 "$OUT/new_tests.log"; ok $s || exit $s
[ -n "$NEW_ONLY" ] && { echo "== done (new tests only)" | tee -a "$OUT/progress.txt"; exit 0; }
echo "== gpu suite" | tee -a "$OUT/progress.txt"
PYTEST_ADDOPTS="--durations=60" REDSET_TEST_PROGRESS_DIR="$OUT" timeout -k 10 1000 python -u -m pytest tests -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1
s=$?; echo "gpu suite exit $s" | tee -a "$OUT/progress.txt"; tail -3 "$OUT/gpu_tests.log"; ok $s || exit $s
echo "== smoke" | tee -a "$OUT/progress.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
s=$?; echo "smoke exit $s" | tee -a "$OUT/progress.txt"; ok $s || exit $s
echo "== bench" | tee -a "$OUT/progress.txt"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
s=$?; echo "bench exit $s" | tee -a "$OUT/progress.txt"; head -c 600 "$OUT/bench.json"; echo; ok $s || exit $s
[ -n "$NO_PROF" ] && { echo "== done (no profiles)" | tee -a "$OUT/progress.txt"; exit 0; }
echo "== rocprofv3 kernel stats" | tee -a "$OUT/progress.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 --sharded 0 > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
s=$?; echo "rocprof exit $s" | tee -a "$OUT/progress.txt"; ok $s || exit $s
echo "== rocprofv3 PMC FETCH_SIZE / WRITE_SIZE (separate passes)" | tee -a "$OUT/progress.txt"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
  python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --pairs 0 --sharded 0 > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
s=$?; echo "pmc fetch exit $s" | tee -a "$OUT/progress.txt"; ok $s || exit $s
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write -- \
  python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --pairs 0 --sharded 0 > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
s=$?; echo "pmc write exit $s" | tee -a "$OUT/progress.txt"; ok $s || exit $s
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/traffic.json" > /dev/null
echo "== done" | tee -a "$OUT/progress.txt"
