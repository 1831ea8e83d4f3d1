#!/bin/bash
# growth + split hot launch: full GPU suite, benches, mixed_tenants timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_j.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_j.log | head -20; tail -30 gpurun_out/t_j.log; exit 1; }
tail -1 gpurun_out/t_j.log
for c in tb_uniform mixed_tenants zipf_1b sw_zipf; do
  timeout -k 10 300 python -u bench.py --config $c --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/b_j_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/b_j_$c.log; exit 1; }
  tail -1 gpurun_out/b_j_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.1})"
done
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 2 > gpurun_out/rd_j_mixed.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd_j_mixed.log; exit 1; }
head -20 gpurun_out/rd_j_mixed.log | grep -E "batch|quantile 1.0|normal:"
