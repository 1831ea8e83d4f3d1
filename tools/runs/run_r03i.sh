#!/bin/bash
# which router bench-config tests fail with routing on
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "tests/test_gpu_router.py" -q --timeout 250 --timeout-method thread > gpurun_out/t_i_all.log 2>&1; echo "rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/t_i_all.log | tail -8
