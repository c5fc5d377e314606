set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s20 CFGS="new:0 sb2:0 sb4:0" ROUNDS=3 bash tools/ab_cfg.sh
