#!/bin/bash
# round-4 closing check on the committed tree: GPU suite and smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r04af.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r04af.log | head -20; tail -20 gpurun_out/t_r04af.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r04af.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r04af.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r04af.log; exit 1; }
tail -1 gpurun_out/smoke_r04af.log
echo done
