#!/bin/bash
# round 6: local grouping (k_group) replaces the global second pass + k_bin_bounds: the whole
# GPU suite, smoke, the default line with extras
set -o pipefail
T=${1:-r06b}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_$T.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|CHECK" gpurun_out/t_$T.log | head -20; tail -30 gpurun_out/t_$T.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$T.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_$T.json 2> gpurun_out/b_$T.err || { echo "bench failed"; tail -20 gpurun_out/b_$T.err; exit 1; }
python tools/show_line.py gpurun_out/b_$T.json
echo done
