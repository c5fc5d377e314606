set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02s2
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_doc_examples.py tests/test_gpu_stream.py > gpurun_out/r02s2/tests.log 2>&1; s=$?; tail -3 gpurun_out/r02s2/tests.log; [ $s -le 1 ] || exit $s
OUT=gpurun_out/r02s2 bash tools/ab_pad.sh || exit $?
start=$(date +%s); timeout -k 10 400 python bench.py > gpurun_out/r02s2/bench_default.json 2> gpurun_out/r02s2/bench_default.err || exit $?
cat gpurun_out/r02s2/bench_default.json; echo "bench wall $(( $(date +%s) - start )) s"
