#!/bin/bash
# single-wave chains for one-key hot regions (3-wave only for two-key regions, second side stream)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_q.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_q.log | head -20; tail -20 gpurun_out/t_q.log; exit 1; }
tail -1 gpurun_out/t_q.log
for cfg in sw_zipf zipf_1b mixed_tenants; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --steps 6 > gpurun_out/b_q_${cfg}.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/b_q_${cfg}.log; exit 1; }
  tail -1 gpurun_out/b_q_${cfg}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
timeout -k 10 200 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_q.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_q.log; exit 1; }
grep -E "batch|quantile 1.0|latest" gpurun_out/rd_q.log
