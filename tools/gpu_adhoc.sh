set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s8
mkdir -p $OUT
timeout -k 10 200 python tools/size_sweep.py > $OUT/size_sweep.jsonl 2>&1 || exit $?
cat $OUT/size_sweep.jsonl
OUT=$OUT ENVS="one:REDSET_HIP_STREAMS=1 two:REDSET_HIP_STREAMS=2" ROUNDS=3 bash tools/ab_env.sh
