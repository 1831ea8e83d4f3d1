#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_router.py -x -v --timeout 400 --timeout-method thread > gpurun_out/t_w.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/t_w.log | head -20; tail -30 gpurun_out/t_w.log; exit 1; }
grep -E "PASSED|passed" gpurun_out/t_w.log
