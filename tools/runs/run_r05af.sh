#!/bin/bash
# round 5: region dispatch-order prefix (the smallest regions first, for the chains' slots) now
# that the chains launch before k_regions: order_prefix 4096 (default) vs 0 vs 1024 vs 16384
# result: no difference beyond run-to-run noise (sw_zipf 12.2-12.96 ms for the same setting): default kept
set -o pipefail
mkdir -p gpurun_out
for cfg in sw_zipf zipf_1b mixed_tenants; do
for rep in 1 2; do
for op in 4096 0 1024 16384; do
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline --tune order_prefix=$op > gpurun_out/b_r05af.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05af.log; exit 1; }
tail -1 gpurun_out/b_r05af.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg order_prefix=$op', round(d['ms_per_step'],3), 'region', round(s.get('region'),3), d['status'])"
done
done
done
echo done
