# session script (round 4, s12): loader horizon A/B (one LDS read for all FREE
# words) on the XOR leg and RS(16+4); then the slot roofline probes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04s12; mkdir -p $O
echo start > $O/progress.txt
bash tools/ab_run.sh 3 "--steps 10 --warmup 3" tree hz > $O/ab_hz.txt 2>&1 || exit 1
echo ab ok >> $O/progress.txt
bash tools/ab_run.sh 2 "--steps 10 --warmup 3 --ranks 20 --encoding 4 --lost 1,2,3,4 --xor 0" tree hz > $O/ab_hz_wide.txt 2>&1 || exit 1
echo ab wide ok >> $O/progress.txt
bash tools/gpu_probes.sh r04s12/probes rank > $O/probes.out 2>&1 || exit 1
echo done >> $O/progress.txt
