set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s4
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_stream.py > $OUT/tests.log 2>&1; s=$?; tail -4 $OUT/tests.log; [ $s -le 1 ] || exit $s
timeout -k 10 900 python -u tools/bench_e2e.py --mode both > $OUT/e2e.jsonl 2> $OUT/e2e.err; s=$?; cat $OUT/e2e.jsonl | cut -c1-400; tail -3 $OUT/e2e.err; exit $s
