set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s6 CFGS="new:0 glds1:0 glds2:0" ROUNDS=2 bash tools/ab_cfg.sh || exit $?
for lib in new glds2; do OUT=gpurun_out/r02s6/pmc bash tools/pmc_lib.sh $lib || exit $?; done
