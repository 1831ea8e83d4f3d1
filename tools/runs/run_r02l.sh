#!/bin/bash
# per-key chains in wave_apply: parity, then benches with and without --pipeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hot.py tests/test_gpu_regression.py tests/test_gpu_configs.py tests/test_gpu_sparse.py tests/test_gpu_growth.py tests/test_gpu_state.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_m.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/t_m.log | head -20; tail -30 gpurun_out/t_m.log; exit 1; }
tail -1 gpurun_out/t_m.log
for c in tb_uniform mixed_tenants zipf_1b sw_zipf; do
 for v in "" "--pipeline"; do
  timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline $v > gpurun_out/b_m_$c$v.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/b_m_$c$v.log; exit 1; }
  tail -1 gpurun_out/b_m_$c$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.3})"
 done
done
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 2 > gpurun_out/rd_m_mixed.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd_m_mixed.log; exit 1; }
head -4 gpurun_out/rd_m_mixed.log; grep -E "quantile 1.0|normal:" gpurun_out/rd_m_mixed.log | head -2
timeout -k 10 300 python -u tools/region_debug.py --config zipf_1b --batches 2 > gpurun_out/rd_m_zipf.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd_m_zipf.log; exit 1; }
head -3 gpurun_out/rd_m_zipf.log; grep -E "quantile 1.0|normal:" gpurun_out/rd_m_zipf.log | head -2
