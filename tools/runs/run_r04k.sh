#!/bin/bash
# region stage: LDS peer match, reference-window geometry, verified fast window fraction; solo
# pass. Whole GPU suite, then the default bench line, then the mixed hot-chain timeline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r04k.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04k.log | head -20; tail -20 gpurun_out/t_r04k.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r04k.log | tail -2
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_r04k.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04k.log; exit 1; }
tail -1 gpurun_out/b_r04k.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'), 'cpu %.3e'%d['cpu_baseline']['value'])
for x in ('tb_uniform','zipf_1b'): print(x, '%.3e'%d[x]['value'], 'ms %.3f'%d[x]['ms_per_step'], 'frac %.4f'%d[x]['roofline_frac'], d[x]['parity'], 'cpu %.3e'%d[x]['cpu_baseline']['value'])
print('config1', d['config1']['parity'], '%.3e'%d['config1']['engine_value'], 'cpu %.3e'%d['config1']['cpu_port_value'])"
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04k.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04k.log; exit 1; }
grep -E "^batch 5|hot:" gpurun_out/rd_r04k.log | tail -3
echo done
