# the driver's default command, three fresh processes, final tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03s50; mkdir -p $OUT
for i in 1 2 3; do timeout -k 10 300 python bench.py > $OUT/default_$i.json 2> $OUT/default_$i.err || exit $?; echo "run $i done"; done
python3 -c "
import json
for i in (1,2,3):
    d=json.load(open(f'gpurun_out/r03s50/default_{i}.json')); r=d['roofline']; b=d['breakdown']
    print('default', i, d['value'], r['frac'], b['encode_GBps'], b['rebuild_GBps'], d['xor']['value'], d['ring_faults'], d['round_trip_bit_exact'])
"
