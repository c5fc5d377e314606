set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02s32
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_setfiles.py tests/test_gpu_rebuild_tool.py tests/test_gpu_mpi.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in 1 0; do
REDSET_HIP_SCRATCH_CACHE=$c timeout -k 10 200 python -u tools/config1_e2e.py /dev/shm 5 | sed "s/^/cache=$c /" >> $O/c1.jsonl || exit 2
done
cat $O/c1.jsonl
