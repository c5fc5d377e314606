set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s38
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_mpi.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_asan.sh r02s38_san || exit 2
for ch in 16 64; do
timeout -k 10 400 python -u tools/rank_bench.py --scheme rs --ranks 11 --encoding 3 --chunk-mib $ch --repeat 3 >> $O/rank.jsonl || exit 3
done
cat $O/rank.jsonl
