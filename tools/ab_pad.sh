#!/bin/bash
# A/B of the bench's cell padding with stripes in sequence: alternating
# processes, pad 0 vs 16 MiB, ROUNDS rounds (bench.py, main line only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/ab_pad}
mkdir -p "$OUT"
: > "$OUT/ab_pad.jsonl"
for r in $(seq 1 ${ROUNDS:-3}); do
  for pad in ${PADS:-0 16}; do
    timeout -k 10 180 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 --xor 0 \
      --cell-pad-mib $pad > "$OUT/pad.tmp" 2> "$OUT/pad.err" || exit $?
    python3 -c "import json,sys; d=json.load(open('$OUT/pad.tmp')); b=d['breakdown']; print(json.dumps({'round': $r, 'pad_mib': $pad, 'value': d['value'], 'frac': d['roofline']['frac'], 'encode_GBps': b['encode_GBps'], 'rebuild_GBps': b['rebuild_GBps'], 'stride': d['config']['cell_stride_bytes']}))" >> "$OUT/ab_pad.jsonl"
    tail -1 "$OUT/ab_pad.jsonl"
  done
done
