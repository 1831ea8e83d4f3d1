#!/bin/bash
# hot chains: greedy scan in allow/deny runs + SW run stamps; mixed timeline, then the hot and
# config tests for parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04l.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04l.log; exit 1; }
grep -E "^batch|latest" gpurun_out/rd_r04l.log | tail -4; grep -A3 "^batch 5" gpurun_out/rd_r04l.log | tail -3
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -v --timeout 600 --timeout-method thread > gpurun_out/t_r04l.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04l.log | head -20; tail -20 gpurun_out/t_r04l.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r04l.log | tail -2
echo done
