#!/bin/bash
# route table built in parallel after the region stage; A/B of hot_threshold on the Zipf configs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_g.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_g.log | head -20; tail -20 gpurun_out/t_g.log; exit 1; }
tail -1 gpurun_out/t_g.log
for cfg in sw_zipf zipf_1b mixed_tenants; do
for thr in 16384 32768 65536 131072; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --steps 6 --tune hot_threshold=$thr > gpurun_out/b_g_${cfg}_$thr.log 2>&1 || { echo "bench $cfg $thr failed"; tail -5 gpurun_out/b_g_${cfg}_$thr.log; exit 1; }
  tail -1 gpurun_out/b_g_${cfg}_$thr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $thr', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('scatter1','region_offsets','region','hot_fill','upsweep1')})"
done; done
