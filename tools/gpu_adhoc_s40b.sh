# claimed mode correctness (normal + spin-cap twin), then the A/B in gpu_adhoc_s40.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03s40; mkdir -p $OUT
REDSET_HIP_SEQUENTIAL=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_digests.py tests/test_gpu_redset_sequence.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_seq4.log 2>&1; s=$?; tail -2 $OUT/tests_seq4.log; [ $s -eq 0 ] || exit $s
REDSET_RING_FALLBACK_RUN=1 REDSET_HIP_LIBRARY=$PWD/redset_amd/lib_spincap/libredset_hip.so REDSET_HIP_SEQUENTIAL=4 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_digests.py tests/test_gpu_redset_sequence.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests_seq4_twin.log 2>&1; s=$?; tail -2 $OUT/tests_seq4_twin.log; [ $s -eq 0 ] || exit $s
bash tools/gpu_adhoc_s40.sh
