#!/bin/bash
# gf_mac / xor widths on one box, alternating library builds (LIBS: "new" =
# in-tree, else abx/lib_<name>.so), ROUNDS rounds: tools/gf_width_probe.py
# and tools/xor_wide_probe.py. Output gpurun_out/widths.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; rm -f gpurun_out/widths.jsonl
for r in $(seq ${ROUNDS:-2}); do
  for l in ${LIBS:-prev new}; do
    if [ $l = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/abx/lib_$l.so; fi
    timeout -k 10 300 python tools/gf_width_probe.py 3 ${GF3:-2 4 6 8 12 16} >> gpurun_out/widths.jsonl || exit 1
    timeout -k 10 300 python tools/gf_width_probe.py 2 ${GF2:-8 16} >> gpurun_out/widths.jsonl || exit 1
    timeout -k 10 300 python tools/xor_wide_probe.py ${XW:-3 7 12 16} | sed 's/"lib"/"xor": 1, "lib"/' >> gpurun_out/widths.jsonl || exit 1
  done
done
echo done
