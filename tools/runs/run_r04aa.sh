#!/bin/bash
# hot chains: remaining from readlane of the few table entries in play; hot parity + mixed timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py -x -v --timeout 600 --timeout-method thread -k "hot or mixed" > gpurun_out/t_r04aa.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04aa.log | head -20; tail -30 gpurun_out/t_r04aa.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r04aa.log | tail -1
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04aa.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04aa.log; exit 1; }
grep -E "^batch" gpurun_out/rd_r04aa.log | tail -3; grep -A3 "^batch 5" gpurun_out/rd_r04aa.log | grep dur | head -3 | cut -c1-100
echo done
