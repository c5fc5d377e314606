# bench.py with extra padding after every cell (relative placement of a stripe's cells in HBM)
mkdir -p gpurun_out
for r in 1 2; do
  for pad in ${PADS:-0 16 32}; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --cell-pad-mib $pad > gpurun_out/pad.tmp 2>&1 || exit 1
    echo "pad=$pad $(tail -1 gpurun_out/pad.tmp)" >> gpurun_out/pad.jsonl
  done
done
