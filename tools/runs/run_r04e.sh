#!/bin/bash
# windowed hot-chain detail (kDet chunks per window): region timeline of mixed_tenants over 6
# batches, then parity: hot tests + the steady-state config tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04e.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04e.log; exit 1; }
grep -E "^batch|dur" gpurun_out/rd_r04e.log | tail -14
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -v --timeout 600 --timeout-method thread > gpurun_out/t_r04e.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04e.log | head -20; tail -20 gpurun_out/t_r04e.log; exit 1; }
grep -E "region stage|passed|failed" gpurun_out/t_r04e.log | tail -10
echo done
