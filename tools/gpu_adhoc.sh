set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s9
mkdir -p $OUT
: > $OUT/pads.jsonl
for r in 1 2; do
  for pad in 0 0.00390625 0.0625 1 2 3 6 16 17 24 40; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 --xor 0 --cell-pad-mib $pad > $OUT/p.tmp 2> $OUT/p.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/p.tmp')); b=d['breakdown']; print(json.dumps({'round': $r, 'pad_mib': $pad, 'value': d['value'], 'encode': b['encode_GBps'], 'rebuild': b['rebuild_GBps'], 'stride': d['config']['cell_stride_bytes']}))" | tee -a $OUT/pads.jsonl
  done
done
