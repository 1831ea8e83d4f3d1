#!/bin/bash
# routing of the previous batch's hot regions in pass 0: full GPU suite, default bench, region timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_b.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_b.log; exit 1; }
tail -1 gpurun_out/smoke_b.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_b.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_b.log | head -20; tail -20 gpurun_out/t_b.log; exit 1; }
tail -1 gpurun_out/t_b.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-extra > gpurun_out/b_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_b.log; exit 1; }
tail -1 gpurun_out/b_b.log | cut -c1-1500
timeout -k 10 200 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_b.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_b.log; exit 1; }
grep -E "batch|quantile 1.0" gpurun_out/rd_b.log
