# A/B of library builds on one box: ab/lib_<name>.so for each name in LIBS
# ("new" = the in-tree build), for each blocks-per-CU in BPC_LIST, twice.
mkdir -p gpurun_out
for r in 1 2; do
  for b in ${BPC_LIST:-2 4}; do
    for lib in ${LIBS:-old new}; do
      if [ $lib = new ]; then unset REDSET_HIP_LIBRARY; else export REDSET_HIP_LIBRARY=$PWD/ab/lib_$lib.so; fi
      REDSET_HIP_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/ab.tmp 2>&1 || exit 1
      echo "$lib bpc=$b $(tail -1 gpurun_out/ab.tmp)" >> gpurun_out/ab.jsonl
    done
  done
done
