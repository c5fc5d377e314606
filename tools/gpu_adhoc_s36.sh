# block clock with per-CU persistence (current tree's clock build)
mkdir -p gpurun_out/r03s36
REDSET_HIP_LIBRARY=$PWD/abx/lib_clock.so timeout -k 10 200 python -u tools/block_clock.py 10 > gpurun_out/r03s36/block_clock.jsonl 2>&1; s=$?
cat gpurun_out/r03s36/block_clock.jsonl; exit $s
