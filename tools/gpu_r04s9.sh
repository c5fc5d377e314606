# session script (round 4, s9): the host-MPI slice rule against the caller's
# raw buffer (twin: REDSET_HIP_TEST_RANK_SLICE=raw), alternating, median of 6
# warm calls each; then the MPI / adapter GPU tests on the new rule
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04s9; mkdir -p $O
echo start > $O/progress.txt
TW="env LD_LIBRARY_PATH=$PWD/redset_amd/lib_test REDSET_HIP_TEST_RANK_SLICE=raw"
run() { # name args...
  local name=$1; shift
  for k in 1 2; do
    timeout -k 10 300 python tools/rank_bench.py --repeat 7 --dir /tmp/rb "$@" > $O/${name}_new$k.json 2> $O/${name}_new$k.err || exit 1
    timeout -k 10 300 $TW python tools/rank_bench.py --repeat 7 --dir /tmp/rb "$@" > $O/${name}_raw$k.json 2> $O/${name}_raw$k.err || exit 1
  done
  echo "$name ok" >> $O/progress.txt
}
run rs64_buf1 --ranks 11 --encoding 3 --chunk-mib 64 --buf-mib 1 --exchange host
run xor64_buf1 --scheme xor --ranks 8 --chunk-mib 64 --buf-mib 1 --exchange host --lost 3
run rs16_buf16 --ranks 11 --encoding 3 --chunk-mib 16 --buf-mib 16 --exchange host
timeout -k 10 600 python -u -m pytest tests/test_gpu_mpi.py tests/test_gpu_adapter.py -x -v --timeout 120 --timeout-method thread > $O/mpi_tests.log 2>&1 || exit 1
echo done >> $O/progress.txt
