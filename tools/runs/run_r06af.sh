#!/bin/bash
# round 6: the whole GPU suite and smoke on the final code
set -o pipefail
mkdir -p gpurun_out/r06af
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06af/gpu_suite.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/r06af/gpu_suite.log | head -20; tail -20 gpurun_out/r06af/gpu_suite.log; exit 1; }
grep -E "passed|failed" gpurun_out/r06af/gpu_suite.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06af/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06af/smoke.log; exit 1; }
tail -1 gpurun_out/r06af/smoke.log
echo done
