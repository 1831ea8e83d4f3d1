#!/bin/bash
# round 6: persistent-grid sizes after the 128K-request tiles (sw_zipf): scatter / upsweep /
# unpermute workgroups per CU
set -o pipefail
mkdir -p gpurun_out
one() {  # tag tune...
  local tag=$1; shift
  local t=""; for kv in "$@"; do t="$t --tune $kv"; done
  timeout -k 10 200 python -u bench.py --config sw_zipf --steps 10 --warmup 3 --no-extra --no-cpu-baseline $t > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $tag"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$tag', round(d['ms_per_step'],3), 'upsweep0', s.get('upsweep0'), 'scatter0', s['scatter0'], 'unpermute', s.get('unpermute'), d['status'])"
}
for rep in 1 2; do
  one base && one sc2 scatter_per_cu=2 && one up8 upsweep_per_cu=8 && one up2 upsweep_per_cu=2 && one un2 unpermute_per_cu=2 || exit 1
done
echo done
