#!/bin/bash
# tile unpermute (u16 tile-local pass-0 positions): whole GPU suite, then A/B on the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r04t.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04t.log | head -20; tail -20 gpurun_out/t_r04t.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r04t.log | tail -2
for x in 1 0 1 0; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --tune tile_unpermute=$x > gpurun_out/b_r04t_$x.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04t_$x.log; exit 1; }
tail -1 gpurun_out/b_r04t_$x.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tile $x', '%.3e'%d['value'], round(d['ms_per_step'],3), 'unpermute', d['stage_ms']['unpermute'], 'scatter0', d['stage_ms']['scatter0'], '| tb', round(d['tb_uniform']['ms_per_step'],3), d['tb_uniform']['stage_ms']['unpermute'], '| z1b', round(d['zipf_1b']['ms_per_step'],3), d['zipf_1b']['stage_ms']['unpermute'], d['zipf_1b']['parity'][:9])"
done
echo done
