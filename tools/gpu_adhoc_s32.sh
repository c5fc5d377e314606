# block-clock study: event times with the default library, then the clock build
mkdir -p gpurun_out/r03s32
timeout -k 10 200 python -u tools/block_clock.py 10 > gpurun_out/r03s32/block_clock.jsonl 2>&1 || exit $?
REDSET_HIP_LIBRARY=$PWD/abx/lib_clock.so timeout -k 10 200 python -u tools/block_clock.py 10 >> gpurun_out/r03s32/block_clock.jsonl 2>&1; s=$?
cat gpurun_out/r03s32/block_clock.jsonl; exit $s
