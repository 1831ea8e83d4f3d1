#!/bin/bash
# hot chains: parity, timelines, benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_parity.py tests/test_gpu_sparse.py tests/test_gpu_configs.py tests/test_gpu_regression.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_thr.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_thr.log; exit 1; }
tail -1 gpurun_out/t_thr.log
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 3 > gpurun_out/rd9_mixed.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd6_mixed.log; exit 1; }
for c in mixed_tenants zipf_1b sw_zipf; do
    timeout -k 10 300 python -u bench.py --config $c --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/b9_$c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b6_$c.log; exit 1; }
    tail -1 gpurun_out/b9_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'region %.2f'%d['stage_ms'].get('region',0))"
done
