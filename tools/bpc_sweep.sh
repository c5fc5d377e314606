# blocks-per-CU sweep of the production bench (interleaved to expose drift)
mkdir -p gpurun_out
for b in ${BPC_LIST:-1 2 4 2 1 4}; do
  REDSET_HIP_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/sweep.tmp 2>&1 || exit 1
  echo "bpc=$b $(tail -1 gpurun_out/sweep.tmp)" >> gpurun_out/sweep.jsonl
done
