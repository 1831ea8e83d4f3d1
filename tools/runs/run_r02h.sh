#!/bin/bash
# pipelined batches: parity, then default bench with / without the pipeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_router.py tests/test_router_cpp.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_h.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_h.log; exit 1; }
tail -1 gpurun_out/t_h.log
for v in "" "--no-pipeline"; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline $v > gpurun_out/b_h$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_h$v.log; exit 1; }
tail -1 gpurun_out/b_h$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default $v', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], {k:v for k,v in d['stage_ms'].items() if v>0.02})"
done
