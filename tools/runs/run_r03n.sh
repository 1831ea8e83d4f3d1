#!/bin/bash
# mixed_tenants: region_order / hot chain stream priority effects on the chains
set -o pipefail
mkdir -p gpurun_out
for v in "base" "O0 --tune region_order=0" "O0R --tune region_order=0 --tune sw_rounds=1" "P0 --tune order_prefix=0"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --config mixed_tenants --no-cpu-baseline --no-extra --steps 6 "$@" > gpurun_out/b_n_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/b_n_$tag.log; exit 1; }
  tail -1 gpurun_out/b_n_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('region','region_offsets','unpermute','scatter0','scatter1')})"
done
