#!/bin/bash
# A/B of library builds on one box: alternating fresh bench.py processes, one
# per (round, build); each line gives the step rate and the encode / rebuild
# rates and launch times. Builds: "base" etc. = ab/lib_<name>.so
# (tools/build_variant.sh), "tree" = the in-tree product library.
# usage: tools/ab_run.sh <rounds> "<bench args>" <build>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1 args=$2; shift 2
# A build may carry environment settings for its process: "twin:REDSET_HIP_XOR_CLAIM=1"
# ("twin" = the test twin library redset_amd/lib_test/).
for r in $(seq "$rounds"); do
  for spec in "$@"; do
    b=${spec%%:*}
    envs=()
    [ "$spec" != "$b" ] && IFS=, read -r -a envs <<< "${spec#*:}"
    case $b in
      tree) lib= ;;
      twin) lib=$PWD/redset_amd/lib_test/libredset_hip.so ;;
      *) lib=$PWD/ab/lib_$b.so ;;
    esac
    out=$(env ${lib:+REDSET_HIP_LIBRARY=$lib} "${envs[@]}" timeout -k 10 300 python bench.py --cpu-baseline 0 --pairs 0 \
          $args 2>/dev/null | tail -1)
    s=$?
    [ $s -eq 0 ] || { echo "$b: bench exit $s"; exit $s; }
    echo "$out" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
b = d['breakdown']; x = d.get('xor') or {}
print(f\"$spec round $r: step {d['value']:8.1f}  encode {b['encode_GBps']:8.1f}  rebuild {b['rebuild_GBps']:8.1f}  \"
      f\"launch_ms {d['roofline']['avg_launch_ms']}  xor {x.get('value')}  rt {d['round_trip_bit_exact']}  faults {d['ring_faults']}\")"
  done
done
