set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s24
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_mpi.py::test_mpi_sharded_gpu tests/test_gpu_parity.py::test_sharded_runner_world1_hip \
  tests/test_gpu_full_digests.py::test_full_size_sharded_rebuild_digests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for np in 2 4; do
SHARDED_TEST_REPS=5 timeout -k 10 300 /opt/conda/bin/mpirun -np $np -host localhost tests/mpi/build/sharded_test --gpu 11 3 4194304 1 2 > $O/timing_np$np.log 2>&1 || { tail $O/timing_np$np.log; exit 2; }
grep timing $O/timing_np$np.log
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --chunk-mib 2 --steps 3 --warmup 1 --pairs 0 \
  > $O/n2_gloo.json 2> $O/n2_gloo.err || { tail $O/n2_gloo.err; exit 4; }
tail -1 $O/n2_gloo.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get('sharded')))"
