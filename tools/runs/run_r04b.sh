#!/bin/bash
# router rework (receive capacity + split rounds, buffers reserved at create, engine failure
# test) + the bench rehearsal of the N>1 path, then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_router_cpp.py tests/test_gpu_bench_multi.py tests/test_gpu_router.py -v -s --timeout 250 --timeout-method thread > gpurun_out/t_r04b_router.log 2>&1 || { echo "router tests failed"; grep -E "FAILED|Error|error|CHECK" gpurun_out/t_r04b_router.log | head -40; tail -30 gpurun_out/t_r04b_router.log; exit 1; }
grep -E "rounds|reserve|engine failure|passed|failed|mismatches" gpurun_out/t_r04b_router.log | tail -30
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/t_r04b.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/t_r04b.log | head -20; tail -20 gpurun_out/t_r04b.log; exit 1; }
tail -1 gpurun_out/t_r04b.log
echo done
