mkdir -p gpurun_out/r03s18
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_digests.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03s18/parity.log 2>&1; s=$?; tail -2 gpurun_out/r03s18/parity.log; [ $s -eq 0 ] || exit $s
LIBS="prev new" ROUNDS=2 bash tools/ab_abx.sh > /dev/null 2>&1; cp gpurun_out/abx/ab.jsonl gpurun_out/r03s18/ab_rs83.jsonl
BENCH_ARGS="--ranks 20 --encoding 4 --lost 1,2,3,4 --xor 0" LIBS="prev b512 new" ROUNDS=2 bash tools/ab_abx.sh > /dev/null 2>&1; cp gpurun_out/abx/ab.jsonl gpurun_out/r03s18/ab_rs164.jsonl
for l in prev new; do if [ $l = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/abx/lib_$l.so; fi; timeout -k 10 120 python tools/xor_wide_probe.py 7 12 16 || exit 1; done > gpurun_out/r03s18/xor_wide.jsonl
echo done
