set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s44
mkdir -p $O
for i in 1 2 3 4 5; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 --xor 0 > $O/run$i.json 2>> $O/err.log || exit 1
python -c "import json; d=json.load(open('$O/run$i.json')); print($i, d['value'], d['roofline']['frac'], d['breakdown']['encode_GBps'], d['breakdown']['rebuild_GBps'])" | tee -a $O/runs.txt
done
