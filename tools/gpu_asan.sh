#!/bin/bash
# Host-code AddressSanitizer (then ThreadSanitizer) on the GPU box: the offline rebuild tool (the
# streaming pipeline + file I/O), the per-rank MPI backends and the sharded
# driver, built by tests/asan/Makefile with -Xarch_host ASan only (no GPU
# instrumentation), driven by their own GPU tests.
# Leak checking is off by default here (DETECT_LEAKS=1 turns it on): at exit
# LeakSanitizer's stop-the-world intermittently hung processes that had the
# HIP runtime's threads running (twice in two runs, a different test each
# time; never without it). The CPU-only runs (tests/test_asan_host.py) keep it.
# usage: tools/gpu_asan.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-asan}; mkdir -p "$OUT"
B=tests/asan/build
export ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=${DETECT_LEAKS:-0}:exitcode=86"
export LSAN_OPTIONS="suppressions=$PWD/tests/asan/lsan.supp"
export REDSET_HIP_REBUILD_TOOL=$PWD/$B/redset_hip_rebuild RANK_TEST_BIN=$PWD/$B/rank_test SHARDED_TEST_BIN=$PWD/$B/sharded_test
# ASAN_KEEP_GOING=1: no -x, so one test's failure does not hide the rest
# (round 6: a CHECK of ASan's device allocator at process exit, inside the
# HIP runtime's own teardown, failed one sharded-mpi run once)
X=-x; [ -n "$ASAN_KEEP_GOING" ] && X=
timeout -k 10 900 python -u -m pytest $X -v --timeout 100 --timeout-method thread \
  tests/test_gpu_rebuild_tool.py tests/test_gpu_mpi.py "tests/test_gpu_rccl_stub.py::test_sharded_rccl_transport_with_hip_kernels" \
  "tests/test_gpu_rccl_stub.py::test_sharded_reduce_shape_over_mpi" "tests/test_gpu_rccl_stub.py::test_rank_backends_forced_rccl" \
  > "$OUT/asan_tests.log" 2>&1
s=$?
tail -5 "$OUT/asan_tests.log"
echo "ASan reports (real errors): $(grep -c "ERROR: AddressSanitizer\|ERROR: LeakSanitizer" "$OUT/asan_tests.log")"
echo "ASan runtime CHECK failures at exit: $(grep -c "CHECK failed: sanitizer_allocator_device" "$OUT/asan_tests.log")"
[ -n "$ASAN_ONLY" ] && exit $s
[ $s -eq 0 ] || exit $s
# ThreadSanitizer (make -C tests/asan SANITIZER=thread B=build_tsan): the
# offline tool's streaming pipeline -- reader, writer, I/O pool and feeder
# threads -- with the uninstrumented ROCm runtime's interceptors suppressed
export TSAN_OPTIONS="halt_on_error=0:exitcode=66:report_signal_unsafe=0:suppressions=$PWD/tests/asan/tsan.supp"
REDSET_HIP_REBUILD_TOOL=$PWD/tests/asan/build_tsan/redset_hip_rebuild timeout -k 10 400 python -u -m pytest -x -v \
  --timeout 100 --timeout-method thread tests/test_gpu_rebuild_tool.py > "$OUT/tsan_tests.log" 2>&1
s=$?
tail -3 "$OUT/tsan_tests.log"
exit $s
