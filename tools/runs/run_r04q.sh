#!/bin/bash
# region slice statistics (greedy steps, probe passes) for sw_zipf / zipf_1b; mid_xcd A/B on sw_zipf
set -o pipefail
mkdir -p gpurun_out
for c in sw_zipf zipf_1b; do
timeout -k 10 300 python -u tools/region_debug.py --config $c --batches 2 > gpurun_out/rd_${c}_r04q.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_${c}_r04q.log; exit 1; }
grep -E "^batch 1|regions [0-9]+: mean|quantile 1.0" gpurun_out/rd_${c}_r04q.log | tail -4
done
for x in 1 0 1 0; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --tune mid_xcd=$x > gpurun_out/b_r04q_$x.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04q_$x.log; exit 1; }
tail -1 gpurun_out/b_r04q_$x.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('mid_xcd $x', '%.3e'%d['value'], round(d['ms_per_step'],3), 'region', d['stage_ms']['region'], 'unpermute', d['stage_ms']['unpermute'])"
done
echo done
