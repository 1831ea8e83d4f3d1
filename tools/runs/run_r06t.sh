#!/bin/bash
# round 6 A/B on one box, alternating order: chain_split 0 / 1 on the Zipf configs
set -o pipefail
mkdir -p gpurun_out
one() {  # rep cfg v
  timeout -k 10 200 python -u bench.py --config $2 --steps 20 --warmup 3 --no-extra --no-cpu-baseline --tune chain_split=$3 > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $2 $3"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$1 $2 split=$3', round(d['ms_per_step'],3), 'region', s['region'], 'scatter0', s['scatter0'], 'group', s.get('group'), d['status'])"
}
for rep in 1 2 3; do
  for cfg in sw_zipf zipf_1b; do
    if [ $((rep % 2)) = 1 ]; then one $rep $cfg 0 && one $rep $cfg 1 || exit 1
    else one $rep $cfg 1 && one $rep $cfg 0 || exit 1; fi
  done
done
echo done
