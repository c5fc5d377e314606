set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s15
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_stream.py tests/test_gpu_setfiles.py > $OUT/tests.log 2>&1; s=$?; tail -3 $OUT/tests.log; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python -u tools/bench_e2e.py --mode host > $OUT/e2e.jsonl 2> $OUT/e2e.err; s=$?; cut -c1-330 $OUT/e2e.jsonl; exit $s
