set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s12
mkdir -p $OUT
cat gpurun_out/r02s12/rank_bench.jsonl 2>/dev/null
for args in "--scheme xor --ranks 8 --chunk-mib 64 --buf-mib 1" "--scheme xor --ranks 8 --chunk-mib 64 --buf-mib 8"; do
  timeout -k 10 600 python tools/rank_bench.py $args 2>&1 | tee -a $OUT/rank_bench.jsonl || exit $?
done
