set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s42
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_stream.py -k random > $O/tests.log 2>&1; s=$?
grep -E "PASSED|FAILED|passed|failed|Error|assert" $O/tests.log | tail -20
exit $s
