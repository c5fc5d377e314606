# session script (round 4, s21): XOR host decode orders (chain vs gather,
# twin-forced) over chunk sizes; then the MPI GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04s21; mkdir -p $O
echo start > $O/progress.txt
run() { # name order args...
  local name=$1 order=$2; shift 2
  LD_LIBRARY_PATH=$PWD/redset_amd/lib_test REDSET_HIP_TEST_XOR_DECODE=$order timeout -k 10 300 \
    python tools/rank_bench.py --scheme xor --buf-mib 1 --repeat 5 --exchange host --dir /tmp/rb "$@" > $O/${name}_$order.json 2> $O/${name}_$order.err || exit 1
}
for order in chain gather; do
  run p4_c0 $order --ranks 4 --file-bytes 16777216 --lost 2
  run p4_16m $order --ranks 4 --chunk-mib 16 --lost 2
  run p4_64m $order --ranks 4 --chunk-mib 64 --lost 2
  run p8_8m $order --ranks 8 --chunk-mib 8 --lost 3
  run p8_32m $order --ranks 8 --chunk-mib 32 --lost 3
  run p8_64m $order --ranks 8 --chunk-mib 64 --lost 3
  echo "$order ok" >> $O/progress.txt
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_mpi.py -x -v --timeout 150 --timeout-method thread > $O/t.log 2>&1 || exit 1
echo done >> $O/progress.txt
