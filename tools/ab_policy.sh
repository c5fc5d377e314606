#!/bin/bash
# A/B of cache-policy builds of the codec (ab/lib_*.so, tools/build_ab_variant.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -f gpurun_out/ab.jsonl
LIBS="${LIBS:-new stnt stall ldnt both}" BPC_LIST="${BPC_LIST:-2}" bash tools/ab_bench.sh || exit $?
python3 - <<'PY'
import json
for line in open("gpurun_out/ab.jsonl"):
    tag, js = line.split(" ", 2)[:2], line.split(" ", 2)[2]
    r = json.loads(js); b = r["breakdown"]
    print(f"{tag[0]:6s} {tag[1]}  step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  copy {r['box_reference']['torch_copy_GBps']:7.1f}  rt {r['round_trip_bit_exact']}")
PY
