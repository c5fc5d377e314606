set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s19
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mpi.py > $OUT/tests.log 2>&1; s=$?; tail -2 $OUT/tests.log; [ $s -eq 0 ] || exit $s
for args in "--scheme xor --ranks 8 --chunk-mib 64 --buf-mib 1" "--scheme xor --ranks 8 --chunk-mib 64 --buf-mib 8"; do
  timeout -k 10 600 python tools/rank_bench.py $args 2>&1 | tee -a $OUT/rank_bench.jsonl || exit $?
done
