#!/bin/bash
# exact T1 fallback / re-search in the hot chains: parity, shard model, timelines, benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_regression.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ee.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/t_ee.log | head -20; tail -30 gpurun_out/t_ee.log; exit 1; }
tail -1 gpurun_out/t_ee.log
timeout -k 10 400 python -u tools/shard_model.py --config zipf_1b --gpus 8 --debug --steps 1 > gpurun_out/sm_ee.log 2>&1 || { echo "sm failed"; tail -8 gpurun_out/sm_ee.log; exit 1; }
tail -5 gpurun_out/sm_ee.log
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_ee.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd_ee.log; exit 1; }
grep -E "^batch" gpurun_out/rd_ee.log
for c in mixed_tenants zipf_1b sw_zipf tb_uniform; do
  timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b_ee_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/b_ee_$c.log; exit 1; }
  tail -1 gpurun_out/b_ee_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'])"
done
