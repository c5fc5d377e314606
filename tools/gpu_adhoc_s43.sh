# final tree: full session, then two runs of the driver's default bench command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_session.sh r03s43 || exit $?
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/r03s43/default_$i.json 2> gpurun_out/r03s43/default_$i.err || exit $?; tail -c 400 gpurun_out/r03s43/default_$i.json | head -c 0; done
python3 -c "
import json
for i in (1,2):
    d=json.load(open(f'gpurun_out/r03s43/default_{i}.json')); print('default', i, d['value'], d['roofline']['frac'], d['xor']['value'])
"
