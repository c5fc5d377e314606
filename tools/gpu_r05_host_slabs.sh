#!/bin/bash
# Round 5, sessions r05s10 and r05s12: the sharded slot over host slabs
# (REDSET_HIP_EXCHANGE_SHARDED_HOST): its GPU tests, then the slot's
# roofline for every exchange (tools/gpu_probes.sh rank).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05s10}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "== host-slab tests" | tee -a "$OUT/progress.txt"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mpi.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "sharded-host or sharded_host" > "$OUT/host_slab_tests.log" 2>&1
s=$?
echo "host-slab tests exit $s" | tee -a "$OUT/progress.txt"
tail -3 "$OUT/host_slab_tests.log"
[ $s -eq 0 ] || exit $s
bash tools/gpu_probes.sh "$TAG" rank
