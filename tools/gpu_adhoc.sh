set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mpi.py tests/test_gpu_parity.py::test_sharded_runner_world1_hip tests/test_doc_examples.py > $OUT/tests.log 2>&1; s=$?; tail -5 $OUT/tests.log; [ $s -le 1 ] || exit $s
exit $s
