set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s37
mkdir -p $O
timeout -k 10 400 python -u tools/rank_bench.py --scheme xor --ranks 8 --chunk-mib 64 --lost 3 --repeat 3 >> $O/rank.jsonl || exit 1
for b in 4 16; do
timeout -k 10 400 python -u tools/rank_bench.py --scheme rs --ranks 11 --encoding 3 --chunk-mib 64 --buf-mib $b --repeat 3 >> $O/rank.jsonl || exit 2
done
cat $O/rank.jsonl
