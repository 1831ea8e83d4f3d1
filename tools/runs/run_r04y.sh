#!/bin/bash
# claim losers adopt their own key's slot: whole suite, bench, slice stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r04y.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04y.log | head -20; tail -20 gpurun_out/t_r04y.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r04y.log | tail -1
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_r04y.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04y.log; exit 1; }
tail -1 gpurun_out/b_r04y.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], d.get('parity')[:30], 'region', d['stage_ms']['region'])
for x in ('tb_uniform','zipf_1b'): print(x, '%.3e'%d[x]['value'], 'ms %.3f'%d[x]['ms_per_step'], d[x]['parity'][:30], 'region', d[x]['stage_ms']['region'])"
for c in sw_zipf zipf_1b; do
timeout -k 10 300 python -u tools/region_debug.py --config $c --batches 2 > gpurun_out/rd_${c}_r04y.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_${c}_r04y.log; exit 1; }
grep -E "^batch 1|regions [0-9]+: mean" gpurun_out/rd_${c}_r04y.log | tail -3
done
echo done
