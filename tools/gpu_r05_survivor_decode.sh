#!/bin/bash
# The host-slab decode computing on the survivors only: the slot's GPU tests,
# then the slot roofline of the host exchange against the host slabs for
# RS(8+3) (11 ranks, 64 MiB) and RS(10+4) (14 ranks, 32 MiB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-survivor}; mkdir -p "$OUT"
echo "== slot tests" | tee -a "$OUT/progress.txt"
timeout -k 10 700 python -u -m pytest tests/test_gpu_mpi.py tests/test_gpu_adapter.py -m gpu -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/slot_tests.log" 2>&1
s=$?; echo "slot tests exit $s" | tee -a "$OUT/progress.txt"; tail -2 "$OUT/slot_tests.log"; [ $s -eq 0 ] || exit $s
for ex in host sharded-host; do
  echo "== rs8+3 $ex" | tee -a "$OUT/progress.txt"
  timeout -k 10 400 python tools/rank_bench.py --ranks 11 --encoding 3 --chunk-mib 64 --buf-mib 16 --repeat 5 \
    --exchange $ex --dir /tmp/rank_s_$ex > "$OUT/rank_rs8p3_$ex.out" 2> "$OUT/rank_rs8p3_$ex.err"
  s=$?; echo "exit $s" | tee -a "$OUT/progress.txt"; [ $s -eq 0 ] || exit $s
  rm -rf /tmp/rank_s_$ex
  echo "== rs10+4 $ex" | tee -a "$OUT/progress.txt"
  timeout -k 10 400 python tools/rank_bench.py --ranks 14 --encoding 4 --chunk-mib 32 --buf-mib 16 --repeat 5 \
    --lost 1,2,3,4 --exchange $ex --dir /tmp/rank_w_$ex > "$OUT/rank_rs10p4_$ex.out" 2> "$OUT/rank_rs10p4_$ex.err"
  s=$?; echo "exit $s" | tee -a "$OUT/progress.txt"; [ $s -eq 0 ] || exit $s
  rm -rf /tmp/rank_w_$ex
done
