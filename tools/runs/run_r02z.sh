#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "cache" --timeout 300 --timeout-method thread > gpurun_out/t_z.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/t_z.log | head -20; tail -20 gpurun_out/t_z.log; exit 1; }
tail -1 gpurun_out/t_z.log
