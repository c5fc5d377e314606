set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s43
mkdir -p $O
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 4 --dist-backend gloo --chunk-mib 2 --steps 3 --warmup 1 --pairs 0 \
  > $O/n4_gloo.json 2> $O/n4_gloo.err || { tail $O/n4_gloo.err; exit 4; }
tail -1 $O/n4_gloo.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], json.dumps(d.get('sharded'))[:600])"
