mkdir -p gpurun_out/r03s31
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r03s31/gpu_dist.log 2>&1; s=$?; tail -8 gpurun_out/r03s31/gpu_dist.log; [ $s -le 1 ] || exit $s
REDSET_HIP_LIBRARY=$PWD/abx/lib_clock.so timeout -k 10 200 python -u tools/block_clock.py 10 > gpurun_out/r03s31/block_clock.jsonl 2>&1; s=$?; cat gpurun_out/r03s31/block_clock.jsonl; exit $s
