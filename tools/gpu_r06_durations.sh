cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06s1; mkdir -p $OUT
PYTEST_ADDOPTS="--durations=80" REDSET_TEST_PROGRESS_DIR="$OUT" timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
echo "exit $?"; tail -3 $OUT/gpu_tests.log
