#!/bin/bash
# Measurement probes on a GPU box, each under its own time limit; results
# under gpurun_out/<tag>/. Stops at the first step that faults / aborts /
# times out. usage: tools/gpu_probes.sh <tag> <probe>...
#   gloo   torch gloo P2P rate at world 2, CPU and GPU tensors (what the N>1
#          rehearsals' callback transport pays; tools/gloo_p2p_probe.py)
#   n2     bench.py --gpus 2 rehearsal over gloo on the one GPU
#   rank   the per-rank slot's roofline (tools/rank_bench.py): RS(8+3) 64 MiB
#          and configs[0] (XOR, 4 x 16 MiB files), host and sharded exchanges
#          (RANK_EXCHANGES, default "host sharded-mpi sharded-host")
#   stubn  bench.py --gpus 3 / 4 self-launched, sharded leg over the RCCL transport on
#          the test stand-in (tests/rcclstub), 4 MiB chunks
#   stubfull bench.py --gpus 2 at 64 MiB chunks over the RCCL stand-in: both shapes'
#          decode loops on the real kernels
#   slotab the slot's RS(8+3) 64 MiB encode / rebuild, host ring vs host slabs at the
#          default 1 MiB buffer, alternating, twice each
#   slotbuf  the slot's RS(8+3) 64 MiB encode / rebuild over the host ring and the
#          host slabs at the reference's default 1 MiB MPI buffer and at 16 MiB
#          (round 6: the sharded window no longer grows with the buffer)
#   wide   RS(16+4) (configs[4]'s stripe) device-resident: kernel stats, PMC
#          FETCH/WRITE and SQ counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-probe}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a "$OUT/progress.txt"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local s=$?
  echo "$name exit $s" | tee -a "$OUT/progress.txt"
  tail -2 "$OUT/$name.out"
  [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s
}
for probe in "$@"; do
  case $probe in
    gloo)
      run gloo_cpu 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29541 tools/gloo_p2p_probe.py --device cpu
      run gloo_cuda 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29542 tools/gloo_p2p_probe.py --device cuda --reps 1 ;;
    n2)
      run n2_gloo 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29543 bench.py --gpus 2 --dist-backend gloo --chunk-mib 2 --steps 3 --warmup 1 \
        --cpu-baseline 0 --pairs 0 ;;
    rank)
      for ex in ${RANK_EXCHANGES:-host sharded-mpi sharded-host}; do
        run rank_rs_64m_$ex 400 python tools/rank_bench.py --ranks 11 --encoding 3 --chunk-mib 64 --buf-mib 16 \
          --repeat 5 --exchange $ex --dir /tmp/rank_bench_$ex
        run rank_config0_$ex 200 python tools/rank_bench.py --scheme xor --ranks 4 --file-bytes 16777216 \
          --buf-mib 1 --repeat 5 --exchange $ex --lost 2 --dir /tmp/rank_c0_$ex
      done ;;
    slotbuf)
      for buf in ${SLOT_BUFS:-1 16}; do
        for ex in host sharded-host; do
          run rank_rs_64m_${ex}_buf$buf 400 python tools/rank_bench.py --ranks 11 --encoding 3 --chunk-mib 64 \
            --buf-mib $buf --repeat 5 --exchange $ex --dir /tmp/rank_bench_$ex
        done
      done ;;
    slotwin)
      # the host-slab encode at the default 1 MiB buffer with the test twin's
      # window override: the window's effect alone (bytes per window per cell)
      for win in ${SLOT_WINS:-4194304 8388608 16777216}; do
        LD_LIBRARY_PATH=$PWD/redset_amd/lib_test${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} REDSET_HIP_TEST_SHARDED_WINDOW=$win \
          run rank_rs_64m_sharded-host_win$win 400 python tools/rank_bench.py --ranks 11 --encoding 3 --chunk-mib 64 \
            --buf-mib 1 --repeat 5 --exchange sharded-host --dir /tmp/rank_bench_win
      done
      run rank_rs_64m_host_buf1_again 400 python tools/rank_bench.py --ranks 11 --encoding 3 --chunk-mib 64 \
        --buf-mib 1 --repeat 5 --exchange host --dir /tmp/rank_bench_host ;;
    slotab)
      # host ring against host slabs at the default 1 MiB buffer, alternating
      # (one box's shared-memory MPI drifts by +-20% between calls)
      for rep in 1 2; do
        for ex in host sharded-host; do
          run rank_rs_64m_${ex}_ab$rep 400 python tools/rank_bench.py --ranks 11 --encoding 3 --chunk-mib 64 \
            --buf-mib 1 --repeat 5 --exchange $ex --dir /tmp/rank_bench_$ex
        done
      done ;;
    stubn)
      # the bench's self-launched N = 3 / 4 flow with the sharded leg over the
      # RCCL transport (test twin + tests/rcclstub: any number of ranks per
      # GPU), 4 MiB chunks: AUTO's shape, the shape not taken, one set over N
      for n in ${STUB_NS:-3 4}; do
        REDSET_HIP_LIBRARY=$PWD/redset_amd/lib_test/libredset_hip.so \
          REDSET_HIP_TEST_RCCL_LIBRARY=$PWD/tests/rcclstub/lib/librccl.so.1 \
          run bench_stub_n$n 500 python bench.py --gpus $n --dist-backend gloo --sharded-transport rccl \
            --chunk-mib 4 --steps 3 --warmup 1 --cpu-baseline 1 --cpu-seconds 1 --pairs 0 --xor 0 \
            --sharded-timeout 300
      done ;;
    stubfull)
      # the bench's N = 2 sharded leg at full size (64 MiB chunks) over the
      # RCCL stand-in: the step's rate is the stand-in's (shared-memory
      # copies), but the decode loops (COMPUTE + ACCUMULATE, no exchange) run
      # the real kernels of both shapes: the partial sums' combine plans
      # against the gather shape's gf_mac plans (two ranks sharing one GPU)
      REDSET_HIP_LIBRARY=$PWD/redset_amd/lib_test/libredset_hip.so \
        REDSET_HIP_TEST_RCCL_LIBRARY=$PWD/tests/rcclstub/lib/librccl.so.1 \
        run bench_stub_full_n2 900 python bench.py --gpus 2 --dist-backend gloo --sharded-transport rccl \
          --steps 3 --warmup 1 --cpu-baseline 0 --pairs 0 --xor 0 --sharded-timeout 800 ;;
    wide)
      W="--ranks 20 --encoding 4 --lost 1,2,3,4 --cpu-baseline 0 --pairs 0 --xor 0"
      run wide_bench 300 python bench.py --steps 10 --warmup 3 $W
      run wide_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wide_prof" -o wide -- \
        python3 bench.py --steps 10 --warmup 3 $W
      run wide_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/wide_fetch" -o fetch -- \
        python3 bench.py --steps 4 --warmup 1 $W
      run wide_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/wide_write" -o write -- \
        python3 bench.py --steps 4 --warmup 1 $W
      python3 tools/pmc_traffic.py "$OUT/wide_fetch" "$OUT/wide_write" "$OUT/wide_traffic.json" > /dev/null
      OUT=$OUT/wide_sq BENCH_ARGS="$W" timeout -k 10 400 bash tools/pmc_sq.sh > "$OUT/wide_sq.out" 2>&1
      echo "wide_sq exit $?" | tee -a "$OUT/progress.txt" ;;
  esac
done
echo "== done" | tee -a "$OUT/progress.txt"
