#!/bin/bash
# One rocprofv3 --pmc pass per counter group for library builds, bench.py
# --steps 4, its own run each (never combined with trace domains; at most 8
# SQ counters per pass). LIBS entries: "new" = in-tree, "twin" = the test twin
# (redset_amd/lib_test), else abx/lib_<name>.so; ":VAR=val[,VAR=val]" adds
# environment for that build's runs ("twin:REDSET_HIP_XOR_CLAIM=1").
# BENCH_ARGS adds bench flags; PMC_XOR (default "--xor 0") the XOR leg's.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmcsq}; mkdir -p $OUT
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --pairs 0 ${PMC_XOR:---xor 0} ${BENCH_ARGS:-}"
G1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM"
args=()
for spec in ${LIBS:-new}; do
  lib=${spec%%:*}
  envs=()
  [ "$spec" != "$lib" ] && IFS=, read -r -a envs <<< "${spec#*:}"
  case $lib in
    new) libpath= ;;
    twin) libpath=$PWD/redset_amd/lib_test/libredset_hip.so ;;
    *) libpath=$PWD/abx/lib_$lib.so ;;
  esac
  label=$lib
  for e in "${envs[@]}"; do label+="_${e##*_}"; done
  label=${label//=/-}  # pmc_summary.py takes LABEL=DIR
  for g in 1 2; do
    eval "ctrs=\$G$g"
    env ${libpath:+REDSET_HIP_LIBRARY=$libpath} "${envs[@]}" timeout -s KILL 120 \
      rocprofv3 --pmc $ctrs --output-format csv -d $OUT/$label/g$g -o run -- $B > /dev/null 2> $OUT/$label.g$g.err ||
      { echo "pmc $label g$g failed"; tail -3 $OUT/$label.g$g.err; exit 1; }
  done
  args+=("$label=$OUT/$label")
  echo "$label done"
done
python3 tools/pmc_summary.py "${args[@]}" | tee $OUT/summary.txt
