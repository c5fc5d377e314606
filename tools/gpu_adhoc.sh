set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s39
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_mpi.py -k repeated > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED" $O/tests.log
bash tools/gpu_asan.sh r02s39_san
