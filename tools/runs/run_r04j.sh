#!/bin/bash
# solo allow runs (cache-on SW): parity (cache tests, KATs, config 1) + config 1 timing; then
# the hot-chain timeline (lean TB, noinline SW estimates)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_ref_scenarios.py tests/test_gpu_parity.py tests/test_gpu_growth.py tests/test_gpu_state.py -x -v --timeout 300 --timeout-method thread -k "solo or config1 or cache or kat or ref or growth or state" > gpurun_out/t_r04j.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04j.log | head -20; tail -20 gpurun_out/t_r04j.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r04j.log | tail -3
timeout -k 10 200 python -u -c "
import torch, json, bench
print(json.dumps(bench.config1_line(torch.device('cuda', 0))))" > gpurun_out/c1_r04j.log 2>&1 || { echo "config1 failed"; tail -5 gpurun_out/c1_r04j.log; exit 1; }
tail -1 gpurun_out/c1_r04j.log
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04j.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04j.log; exit 1; }
grep -E "^batch 5|hot:" gpurun_out/rd_r04j.log | tail -3; grep -A8 "^batch 5" gpurun_out/rd_r04j.log | grep "dur" | head -8
echo done
