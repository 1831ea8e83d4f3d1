#!/bin/bash
# how the mixed_tenants step evolves over the batches (stage events in the timed steps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config mixed_tenants --steps 6 --warmup 2 --no-cpu-baseline --stage-timing > gpurun_out/b_aa.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_aa.log; exit 1; }
tail -1 gpurun_out/b_aa.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('mixed last step', 'ms/step %.2f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.2}, d['batch_stats'])"
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_aa.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd_aa.log; exit 1; }
grep -E "^batch|quantile 1.0|normal:" gpurun_out/rd_aa.log
