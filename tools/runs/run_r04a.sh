#!/bin/bash
# round 4 start: the new steady-state config tests (mixed_tenants 6 batches, zipf_1b full batch
# + 4 batches, sw_zipf 3 routed batches), then the default bench line (now with zipf_1b)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py -v -s --timeout 600 --timeout-method thread \
  -k "steady_state or full_batch or routed" > gpurun_out/t_r04a.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error|batch" gpurun_out/t_r04a.log | head -40; tail -20 gpurun_out/t_r04a.log; exit 1; }
grep -E "batch [0-9]|passed|failed" gpurun_out/t_r04a.log | tail -30
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_r04a.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04a.log; exit 1; }
tail -1 gpurun_out/b_r04a.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'), 'cpu %.3e'%d['cpu_baseline']['value'])
for x in ('tb_uniform','zipf_1b'): print(x, '%.3e'%d[x]['value'], 'ms %.3f'%d[x]['ms_per_step'], 'frac %.4f'%d[x]['roofline_frac'], d[x]['parity'], 'cpu %.3e'%d[x]['cpu_baseline']['value'])
print('config1', d['config1']['parity'], '%.3e'%d['config1']['engine_value'])"
echo done
