#!/bin/bash
# A/B of the kernels' register budget (REDSET_WAVES_PER_EU, codec_device.h):
# in-tree build vs ab/lib_<name>.so variants (CFGS="lib:mode ..."), stripes
# one launch each (1) and in-kernel loop (2); fresh process per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wpe; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2; do
  for cfg in ${CFGS:-new:1 wpe0:1 wpe2pipe:1}; do
    lib=${cfg%%:*}; mode=${cfg##*:}
    if [ $lib = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/ab/lib_$lib.so; fi
    REDSET_HIP_SEQUENTIAL=$mode timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $OUT/b.tmp 2>&1 || exit 1
    echo "$lib seq=$mode $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/wpe/ab.jsonl"):
    t1, t2, js = line.split(" ", 2)
    r = json.loads(js); b = r["breakdown"]
    print(f"{t1:5s} {t2}  step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  copy {r['box_reference']['torch_copy_GBps']:7.1f}  rt {r['round_trip_bit_exact']}")
PY
