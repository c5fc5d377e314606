set -o pipefail
mkdir -p gpurun_out/r05s9
for n in 3 4; do
  echo "== gloo self-launch N=$n"
  timeout -k 10 420 python bench.py --gpus $n --dist-backend gloo --chunk-mib 1 --steps 3 --warmup 1 --cpu-baseline 0 --pairs 0 --xor 0 > gpurun_out/r05s9/bench_gloo_n$n.json 2> gpurun_out/r05s9/bench_gloo_n$n.err || { echo "N=$n exit $?"; exit 1; }
  echo "N=$n exit 0"
  cat gpurun_out/r05s9/bench_gloo_n$n.json
done
