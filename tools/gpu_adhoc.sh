set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s10
mkdir -p $OUT
for args in "--chunk-mib 16 --buf-mib 1" "--chunk-mib 64 --buf-mib 1" "--chunk-mib 64 --buf-mib 8"; do
  timeout -k 10 600 python tools/rank_bench.py $args 2>&1 | tee -a $OUT/rank_bench.jsonl || exit $?
done
