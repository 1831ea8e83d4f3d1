#!/bin/bash
# round 5: walk_min 0 (every dense-enough key walked) vs the default 4000 on the headline
# configs, now that the walk's common path is an inner loop and the chains start on time
set -o pipefail
mkdir -p gpurun_out
for cfg in sw_zipf zipf_1b; do
for rep in 1 2; do
for wm in 4000 0; do
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline --tune walk_min=$wm > gpurun_out/b_r05w.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05w.log; exit 1; }
tail -1 gpurun_out/b_r05w.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg walk_min=$wm', round(d['ms_per_step'],3), 'offs', round(s.get('region_offsets'),3), 'region', round(s.get('region'),3), 'fill', round(s.get('hot_fill'),3), d['status'])"
done
done
done
timeout -k 10 300 python -u tools/region_debug.py --config sw_zipf --batches 3 --tune walk_min=0 > gpurun_out/rd_r05w_sw_zipf.txt 2>&1 || { echo "region_debug failed"; exit 1; }
grep -E "^batch|quantile 1.0|latest" gpurun_out/rd_r05w_sw_zipf.txt | cut -c1-250
echo done
