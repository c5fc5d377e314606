set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r02s17
mkdir -p $OUT
for od in 1 0; do
  for cfg in "--slice-mib 8 --threads 16" "--slice-mib 32 --threads 16"; do
    REDSET_HIP_ODIRECT=$od timeout -k 10 600 python -u tools/bench_e2e.py --mode disk --cpu-stripes "" $cfg > $OUT/e.tmp 2> $OUT/e.err || exit $?
    python3 -c "
import json
for l in open('$OUT/e.tmp'):
    d=json.loads(l); print(json.dumps({'odirect': $od, 'cfg': '$cfg', 'case': d['case'], 'GBps': round(d['GBps'],2), 'rt': d.get('round_trip_equal')}))" | tee -a $OUT/sweep.jsonl
  done
done
