set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s33
mkdir -p $O
export TSAN_OPTIONS="halt_on_error=0:exitcode=66:report_signal_unsafe=0:suppressions=$PWD/tests/asan/tsan.supp"
REDSET_HIP_REBUILD_TOOL=$PWD/tests/asan/build_tsan/redset_hip_rebuild timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_rebuild_tool.py > $O/tsan_tests.log 2>&1; s=$?
grep -E "PASSED|FAILED|passed|failed" $O/tsan_tests.log | tail -8
exit $s
