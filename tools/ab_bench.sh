# A/B of two library builds on the same box: ab/lib_old.so vs the in-tree one
mkdir -p gpurun_out
for r in 1 2; do
  for b in ${BPC_LIST:-2 4}; do
    for lib in old new; do
      if [ $lib = old ]; then export REDSET_HIP_LIBRARY=$PWD/ab/lib_old.so; else unset REDSET_HIP_LIBRARY; fi
      REDSET_HIP_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/ab.tmp 2>&1 || exit 1
      echo "$lib bpc=$b $(tail -1 gpurun_out/ab.tmp)" >> gpurun_out/ab.jsonl
    done
  done
done
