#!/bin/bash
# A/B of library builds in fresh processes, alternating: LIBS="r02 new ..."
# (new = the in-tree build, else abx/lib_<name>.so), ROUNDS rounds (3).
# Extra bench.py flags in BENCH_ARGS. Summary in gpurun_out/abx/summary.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abx; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in $(seq ${ROUNDS:-3}); do
  for lib in ${LIBS:-r02 new}; do
    if [ $lib = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/abx/lib_$lib.so; fi
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pairs 0 $BENCH_ARGS > $OUT/b.tmp 2> $OUT/b.err || exit 1
    echo "$lib $(tail -1 $OUT/b.tmp)" >> $OUT/ab.jsonl
    echo "round $r $lib done"
  done
done
python3 - <<'PY' | tee gpurun_out/abx/summary.txt
import json, collections
rows = collections.defaultdict(list)
for line in open("gpurun_out/abx/ab.jsonl"):
    name, js = line.split(" ", 1)
    r = json.loads(js); b = r["breakdown"]
    rows[name].append((r["value"], b["encode_GBps"], b["rebuild_GBps"], r["xor"]["value"]))
    print(f"{name:8s} step {r['value']:7.1f}  encode {b['encode_GBps']:7.1f}  rebuild {b['rebuild_GBps']:7.1f}"
          f"  xor {r['xor']['value']:7.1f}  faults {r.get('ring_faults')}  rt {r['round_trip_bit_exact']}")
for name, v in rows.items():
    m = [sum(x[i] for x in v) / len(v) for i in range(4)]
    print(f"mean {name:8s} step {m[0]:7.1f}  encode {m[1]:7.1f}  rebuild {m[2]:7.1f}  xor {m[3]:7.1f}")
PY
