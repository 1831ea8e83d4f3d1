#!/bin/bash
# round 6: the hot tests (one-wave chains now behind chain_split 0) and the default line
set -o pipefail
mkdir -p gpurun_out/r06ah
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_walk.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06ah/t.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/r06ah/t.log | head; tail -20 gpurun_out/r06ah/t.log; exit 1; }
grep -E "passed|failed" gpurun_out/r06ah/t.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06ah/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06ah/smoke.log; exit 1; }
tail -1 gpurun_out/r06ah/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06ah/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r06ah/bench.log; exit 1; }
tail -1 gpurun_out/r06ah/bench.log > gpurun_out/r06ah/bench_default.json
python tools/show_line.py gpurun_out/r06ah/bench_default.json | grep -v "stages\|io_frac"
echo done
