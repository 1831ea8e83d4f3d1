#!/bin/bash
# round 6: smoke + default bench line after the upsweep grid default for 128K tiles
set -o pipefail
mkdir -p gpurun_out/r06ae
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "sw_zipf_routed or tb_uniform" > gpurun_out/r06ae/t.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r06ae/t.log; exit 1; }
grep -E "passed|failed" gpurun_out/r06ae/t.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06ae/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06ae/smoke.log; exit 1; }
tail -1 gpurun_out/r06ae/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06ae/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r06ae/bench.log; exit 1; }
tail -1 gpurun_out/r06ae/bench.log > gpurun_out/r06ae/bench_default.json
python tools/show_line.py gpurun_out/r06ae/bench_default.json
echo done
