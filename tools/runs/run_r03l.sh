#!/bin/bash
# split_hot 1 vs 0 with the greedy scan; mixed_tenants with / without routing
set -o pipefail
mkdir -p gpurun_out
for cfg in sw_zipf zipf_1b mixed_tenants; do
for v in "S1" "S0 --tune split_hot=0" "R0 --tune route=0"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --steps 6 "$@" > gpurun_out/b_l_${cfg}_$tag.log 2>&1 || { echo "bench $cfg $tag failed"; tail -5 gpurun_out/b_l_${cfg}_$tag.log; exit 1; }
  tail -1 gpurun_out/b_l_${cfg}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('region','region_offsets','unpermute','scatter0','scatter1')})"
done; done
