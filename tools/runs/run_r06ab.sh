#!/bin/bash
# round 6: upsweep grid 8 workgroups per CU (one tile each) vs 4: does scatter0's mode follow?
set -o pipefail
mkdir -p gpurun_out
one() {  # tag tune...
  local tag=$1; shift
  local t=""; for kv in "$@"; do t="$t --tune $kv"; done
  timeout -k 10 200 python -u bench.py --config sw_zipf --steps 10 --warmup 3 --no-extra --no-cpu-baseline $t > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $tag"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$tag', round(d['ms_per_step'],3), 'upsweep0', s.get('upsweep0'), 'scatter0', s['scatter0'], 'group', s.get('group'), d['status'])"
}
for rep in 1 2 3 4; do
  one up8 upsweep_per_cu=8 && one base || exit 1
done
one up8-z1b upsweep_per_cu=8 && one base-tb || exit 1
echo done
