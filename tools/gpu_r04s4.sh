set -o pipefail
O=gpurun_out/r04s4; mkdir -p $O
(timeout -k 10 60 /opt/conda/bin/mpirun -np 4 -host localhost tools/mpi_bw 1048576 5 > $O/mpi_bw4.out 2>&1; echo "exit $?" >> $O/mpi_bw4.out)
(timeout -k 10 200 python -u tools/rank_bench.py --scheme xor --ranks 4 --file-bytes 16777216 --buf-mib 1 --repeat 3 --exchange host --lost 2 --dir /tmp/rc0 > $O/rank_c0.out 2> $O/rank_c0.err; echo "exit $?" >> $O/rank_c0.out)
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpi.py -x -q --timeout 120 --timeout-method thread -k "config0 or repeated" > $O/mpi_tests.log 2>&1; echo "tests exit $?" >> $O/mpi_tests.log
REDSET_HIP_LIBRARY=$PWD/redset_amd/lib_test/libredset_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m "gpu and knobs" > $O/knob_parity.log 2>&1 || exit 1
timeout -k 10 200 tools/ringbench_16x4 10 rand > $O/ringbench_16x4.txt 2>&1 || exit 1
timeout -k 10 200 tools/ringbench_8x3 10 rand > $O/ringbench_8x3.txt 2>&1 || exit 1
bash tools/ab_run.sh 3 "--steps 10 --warmup 3" twin twin:REDSET_HIP_XOR_CLAIM=1 > $O/ab_xor_claim.txt 2>&1 || exit 1
for pad in 0 4 8 16 24; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --ranks 20 --encoding 4 --lost 1,2,3,4 --xor 0 --pairs 0 --cpu-baseline 0 --cell-pad-mib $pad 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($pad, d['value'], d['breakdown']['encode_GBps'], d['breakdown']['rebuild_GBps'])" >> $O/wide_pad.txt || exit 1; done
echo done >> $O/wide_pad.txt
