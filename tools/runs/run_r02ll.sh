#!/bin/bash
# validation of a hot-chain change: hot / config / parity / router GPU tests, then mixed_tenants steady state and the hot configs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_router.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ll.log 2>&1 || { echo "tests failed"; tail -15 gpurun_out/t_ll.log; exit 1; }
tail -1 gpurun_out/t_ll.log
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_ll.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd_ll.log; exit 1; }
grep -E "^batch" gpurun_out/rd_ll.log
timeout -k 10 300 python -u bench.py --config mixed_tenants --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b_ll.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 gpurun_out/b_ll.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('mixed', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'])"
for c in zipf_1b sw_zipf; do
  timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b_ll_$c.log 2>&1 || { echo "bench $c failed"; exit 1; }
  tail -1 gpurun_out/b_ll_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'])"
done
