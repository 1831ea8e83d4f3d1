#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sparse.py tests/test_gpu_growth.py tests/test_gpu_regression.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_y.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/t_y.log | head -20; tail -30 gpurun_out/t_y.log; exit 1; }
tail -1 gpurun_out/t_y.log
timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --cpu-sample 4194304 > gpurun_out/b_y.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_y.log; exit 1; }
tail -1 gpurun_out/b_y.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], d['parity']); print(d['config1'])"
