#!/bin/bash
# The drop-in slot's GPU tests (per-rank backends under mpirun, the adapter).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-slot}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "== slot tests" | tee -a "$OUT/progress.txt"
timeout -k 10 900 python -u -m pytest tests/test_gpu_mpi.py tests/test_gpu_adapter.py -m gpu -v --timeout 120 \
  --timeout-method thread > "$OUT/slot_tests.log" 2>&1
s=$?
echo "slot tests exit $s" | tee -a "$OUT/progress.txt"
tail -3 "$OUT/slot_tests.log"
exit $s
