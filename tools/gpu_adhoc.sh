set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s29
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_mpi.py -k "sharded" > $O/tests.log 2>&1; s=$?
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -12
exit $s
