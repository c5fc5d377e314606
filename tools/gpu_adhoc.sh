set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s22
mkdir -p $O
for b in 1 4; do
timeout -k 10 300 python -u tools/rank_bench.py --scheme xor --ranks 4 --file-bytes 16777216 --lost 2 --buf-mib $b --repeat 3 >> $O/rank_cfg0.json 2>&1 || exit 1
done
timeout -k 10 600 python -u tools/rank_bench.py --scheme rs --ranks 11 --encoding 3 --chunk-mib 16 --repeat 3 >> $O/rank_rs.json 2>&1
