#!/bin/bash
# hot chains: a second (guessed) prefetch slot; hot + mixed steady-state parity, mixed timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py -x -v --timeout 600 --timeout-method thread -k "hot or mixed or zipf_1b" > gpurun_out/t_r04v.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04v.log | head -20; tail -30 gpurun_out/t_r04v.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r04v.log | tail -2
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04v.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04v.log; exit 1; }
grep -E "^batch" gpurun_out/rd_r04v.log | tail -3; grep -A5 "^batch 5" gpurun_out/rd_r04v.log | grep dur | head -5 | cut -c1-100; grep -A5 "^batch 5" gpurun_out/rd_r04v.log | grep -o "prefetched [0-9]*" | head -5
echo done
