#!/bin/bash
# Quick GPU-box check after a change: GPU tests, N=1 bench, and the N=2
# exchange path rehearsed with gloo on the one GPU (RCCL needs 2 devices).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
s=$?; tail -3 $OUT/gpu_tests.log; [ $s -le 1 ] || exit $s
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 3; }
cat $OUT/bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --chunk-mib 2 --steps 3 --warmup 1 \
  > $OUT/n2_gloo.json 2> $OUT/n2_gloo.err || { tail $OUT/n2_gloo.err; exit 4; }
grep metric $OUT/n2_gloo.json
