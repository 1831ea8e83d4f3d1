#!/bin/bash
# mixed_tenants regression hunt: region timeline over 9 batches, thresholds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 9 > gpurun_out/rd_m.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_m.log; exit 1; }
grep -E "batch|quantile 1.0|latest|normal: sum" gpurun_out/rd_m.log
for v in "T16 --tune hot_threshold=16384" "T32 --tune hot_threshold=32768"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --config mixed_tenants --no-cpu-baseline --no-extra --steps 6 "$@" > gpurun_out/b_m_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/b_m_$tag.log; exit 1; }
  tail -1 gpurun_out/b_m_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('region','region_offsets','unpermute','scatter0','scatter1')})"
done
