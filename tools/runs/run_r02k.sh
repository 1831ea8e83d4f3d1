#!/bin/bash
# TB micro-opts: parity (KATs, hot, configs, regression), benches, mixed_tenants timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hot.py tests/test_gpu_regression.py tests/test_gpu_configs.py tests/test_gpu_sparse.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_k.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/t_k.log | head -20; tail -30 gpurun_out/t_k.log; exit 1; }
tail -1 gpurun_out/t_k.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_k_tb.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_k_tb.log; exit 1; }
tail -1 gpurun_out/b_k_tb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tb_uniform', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.02})"
for c in mixed_tenants zipf_1b; do
  timeout -k 10 300 python -u bench.py --config $c --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/b_k_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/b_k_$c.log; exit 1; }
  tail -1 gpurun_out/b_k_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.3})"
done
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 2 > gpurun_out/rd_k_mixed.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd_k_mixed.log; exit 1; }
head -8 gpurun_out/rd_k_mixed.log; grep -E "quantile 1.0|normal:" gpurun_out/rd_k_mixed.log | head -2
