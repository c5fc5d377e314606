#!/bin/bash
# A/B of the host-resident pipeline builds (ab/lib_<name>.so vs the in-tree
# library) on the end-to-end host case, RS(16+4) p=20, fresh process per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abe2e; mkdir -p $OUT; rm -f $OUT/ab.jsonl
for r in 1 2; do
  for lib in ${LIBS:-new h2d1}; do
    if [ $lib = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/ab/lib_$lib.so; fi
    timeout -k 10 300 python tools/bench_e2e.py --mode host --chunk-mib ${CH:-64} > $OUT/b.tmp 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
    sed "s/^/$lib /" $OUT/b.tmp >> $OUT/ab.jsonl
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/abe2e/ab.jsonl"):
    lib, js = line.split(" ", 1)
    r = json.loads(js)
    print(f"{lib:5s} {r['case']:28s} {r['GBps']:6.1f} GB/s  {r['stats']['seconds']:.3f} s")
PY
