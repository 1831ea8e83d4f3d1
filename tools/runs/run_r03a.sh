#!/bin/bash
# round-3 first checkpoint: smoke, default bench (sw_zipf headline + tb_uniform + config1),
# rocprofv3 trace + PMC of sw_zipf, region timeline of sw_zipf
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_a.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_a.log; exit 1; }
tail -1 gpurun_out/smoke_a.log
timeout -k 10 400 python -u bench.py > gpurun_out/b_a_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_a_default.log; exit 1; }
tail -1 gpurun_out/b_a_default.log | cut -c1-400
bash tools/profile.sh r03_sw_zipf --steps 3 --warmup 1 --no-cpu-baseline --no-extra || exit 1
timeout -k 10 200 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_a_sw_zipf.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_a_sw_zipf.log; exit 1; }
tail -30 gpurun_out/rd_a_sw_zipf.log
