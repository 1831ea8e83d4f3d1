#!/bin/bash
# SW group sweep in the hot chains: hot + config parity tests, then mixed timeline with/without
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot.py -x -v --timeout 600 --timeout-method thread > gpurun_out/t_r04s.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04s.log | head -20; tail -30 gpurun_out/t_r04s.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r04s.log | tail -2
for sw in 1 0; do
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 --tune sw_sweep=$sw > gpurun_out/rd_r04s_$sw.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04s_$sw.log; exit 1; }
echo "sw_sweep=$sw"; grep -E "^batch|hot: sweeps" gpurun_out/rd_r04s_$sw.log | tail -3; grep -A4 "^batch 5" gpurun_out/rd_r04s_$sw.log | grep dur | head -4 | cut -c1-120
done
echo done
