#!/bin/bash
# One rocprofv3 --pmc pass per counter group for library builds (LIBS: "new"
# = in-tree, else abx/lib_<name>.so), bench.py --steps 4, its own run each
# (never combined with trace domains; at most 8 SQ counters per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmcsq}; mkdir -p $OUT
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --pairs 0 --xor 0 ${BENCH_ARGS:-}"
G1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM"
args=()
for lib in ${LIBS:-new}; do
  if [ $lib = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/abx/lib_$lib.so; fi
  for g in 1 2; do
    eval "ctrs=\$G$g"
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/$lib/g$g -o run -- $B > /dev/null 2> $OUT/$lib.g$g.err || { echo "pmc $lib g$g failed"; tail -3 $OUT/$lib.g$g.err; exit 1; }
  done
  args+=("$lib=$OUT/$lib")
  echo "$lib done"
done
python3 tools/pmc_summary.py "${args[@]}" | tee $OUT/summary.txt
