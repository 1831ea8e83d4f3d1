#!/bin/bash
# growth threshold 208: growth tests, then table sizing A/B on tb_uniform, large configs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_growth.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_s.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/t_s.log | head -20; tail -30 gpurun_out/t_s.log; exit 1; }
tail -1 gpurun_out/t_s.log
for rep in 1 2; do
 for ts in 1 2 4; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --table-scale $ts > gpurun_out/b_s_${ts}_$rep.log 2>&1 || { echo "bench $ts failed"; tail -5 gpurun_out/b_s_${ts}_$rep.log; exit 1; }
  tail -1 gpurun_out/b_s_${ts}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ts$ts $rep', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], d['batch_stats'], {k:v for k,v in d['stage_ms'].items() if v>0.1})"
 done
done
for c in mixed_tenants zipf_1b sw_zipf; do
  timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b_s_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/b_s_$c.log; exit 1; }
  tail -1 gpurun_out/b_s_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], d['batch_stats'], {k:v for k,v in d['stage_ms'].items() if v>0.3})"
done
