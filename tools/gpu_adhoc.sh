set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s31
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_mpi.py tests/test_gpu_rebuild_tool.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_asan.sh r02s31_asan || exit 1
for c in 1 0; do
for b in 1; do
REDSET_HIP_SCRATCH_CACHE=$c timeout -k 10 300 python -u tools/rank_bench.py --scheme xor --ranks 4 --file-bytes 16777216 --lost 2 --buf-mib $b --repeat 4 | sed "s/^/cache=$c /" >> $O/rank.jsonl || exit 2
done
REDSET_HIP_SCRATCH_CACHE=$c timeout -k 10 300 python -u tools/rank_bench.py --scheme rs --ranks 11 --encoding 3 --chunk-mib 16 --repeat 3 | sed "s/^/cache=$c /" >> $O/rank.jsonl || exit 3
done
cat $O/rank.jsonl
