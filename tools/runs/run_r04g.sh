#!/bin/bash
# lean TB acquire rounds + SW window cache: region timeline of mixed over 6 batches + hot parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04g.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04g.log; exit 1; }
grep -E "^batch|dur" gpurun_out/rd_r04g.log | tail -14
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py -x -v --timeout 600 --timeout-method thread -k "hot or steady or mixed" > gpurun_out/t_r04g.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04g.log | head -20; tail -20 gpurun_out/t_r04g.log; exit 1; }
grep -E "region stage|passed|failed" gpurun_out/t_r04g.log | tail -10
echo done
