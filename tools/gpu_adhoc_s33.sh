# A/B: compiler-visible wait before the ring loops (new) vs HEAD (old); block clock of the new build
mkdir -p gpurun_out/r03s33
timeout -k 10 600 bash tools/ab_alt.sh old > gpurun_out/r03s33/ab.txt 2>&1; s=$?; cat gpurun_out/r03s33/ab.txt; [ $s -eq 0 ] || exit $s
REDSET_HIP_LIBRARY=$PWD/abx/lib_clock.so timeout -k 10 200 python -u tools/block_clock.py 10 > gpurun_out/r03s33/block_clock.jsonl 2>&1; s=$?
cat gpurun_out/r03s33/block_clock.jsonl; exit $s
