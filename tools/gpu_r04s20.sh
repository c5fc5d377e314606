set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04s20; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mpi.py tests/test_gpu_adapter.py -x -v --timeout 150 --timeout-method thread -k "xor" > $O/t.log 2>&1 || exit 1
for k in 1 2; do
timeout -k 10 300 python tools/rank_bench.py --scheme xor --ranks 8 --chunk-mib 64 --buf-mib 1 --repeat 5 --exchange host --lost 3 --dir /tmp/rb > $O/xor64_$k.json 2> $O/xor64_$k.err || exit 1
timeout -k 10 300 python tools/rank_bench.py --scheme xor --ranks 4 --file-bytes 16777216 --buf-mib 1 --repeat 5 --exchange host --lost 2 --dir /tmp/rb > $O/c0_$k.json 2> $O/c0_$k.err || exit 1
done
