#!/bin/bash
# rocprofv3 passes for one library build (LIB = "new" or abx/lib_<LIB>.so):
# kernel stats, FETCH_SIZE, WRITE_SIZE and one SQ pass, each its own run
# (MI355X_MICROARCH.md HBM section; counters never combined with trace domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LIB=${1:-new}; OUT=${OUT:-gpurun_out/pmc}/$LIB; mkdir -p $OUT
if [ $LIB != new ]; then export REDSET_HIP_LIBRARY=$PWD/abx/lib_$LIB.so; fi
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --pairs 0 --xor 0"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $B > $OUT/stats.json 2> $OUT/stats.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > /dev/null 2> $OUT/fetch.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > /dev/null 2> $OUT/write.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc ${SQ:-SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU} \
  --output-format csv -d $OUT/sq -o run -- $B > /dev/null 2> $OUT/sq.err || exit $?
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write $OUT/traffic.json > /dev/null
echo "$LIB done"
