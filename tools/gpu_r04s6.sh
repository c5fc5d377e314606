# session script (round 4, s6): wide-stripe job order A/B; XOR claimed vs
# default SQ counters and HBM traffic (the claimed negative's counters)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04s6; mkdir -p $O
echo start > $O/progress.txt
W="--ranks 20 --encoding 4 --lost 1,2,3,4 --xor 0"
bash tools/ab_run.sh 3 "--steps 10 --warmup 3 $W" twin twin:REDSET_HIP_SEQUENTIAL=2 > $O/ab_wide_order.txt 2>&1 || exit 1
echo ab_wide ok >> $O/progress.txt
OUT=$O/xor_sq PMC_XOR="--xor 1" LIBS="twin twin:REDSET_HIP_XOR_CLAIM=1" timeout -k 10 500 bash tools/pmc_sq.sh > $O/xor_sq.out 2>&1 || exit 1
echo xor_sq ok >> $O/progress.txt
for spec in default claim; do
  e=(); [ $spec = claim ] && e=(REDSET_HIP_XOR_CLAIM=1)
  env REDSET_HIP_LIBRARY=$PWD/redset_amd/lib_test/libredset_hip.so "${e[@]}" timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/xf_$spec -o f -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --pairs 0 > /dev/null 2> $O/xf_$spec.err || exit 1
  env REDSET_HIP_LIBRARY=$PWD/redset_amd/lib_test/libredset_hip.so "${e[@]}" timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/xw_$spec -o w -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --pairs 0 > /dev/null 2> $O/xw_$spec.err || exit 1
  python3 tools/pmc_traffic.py $O/xf_$spec $O/xw_$spec $O/xor_traffic_$spec.json > /dev/null || exit 1
  env REDSET_HIP_LIBRARY=$PWD/redset_amd/lib_test/libredset_hip.so "${e[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xs_$spec -o s -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --pairs 0 > $O/xs_$spec.out 2> $O/xs_$spec.err || exit 1
done
echo done >> $O/progress.txt
