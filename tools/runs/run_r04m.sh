#!/bin/bash
# hot chains at issue priority 3 (s_setprio): mixed timeline, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04m.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04m.log; exit 1; }
grep -E "^batch|latest|quantile 1.0" gpurun_out/rd_r04m.log | tail -5; grep -A3 "^batch 5" gpurun_out/rd_r04m.log | tail -3
timeout -k 10 300 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rdz_r04m.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rdz_r04m.log; exit 1; }
grep -E "^batch|latest|quantile 1.0" gpurun_out/rdz_r04m.log | tail -4
timeout -k 10 300 python -u tools/region_debug.py --config zipf_1b --batches 3 > gpurun_out/rdb_r04m.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rdb_r04m.log; exit 1; }
grep -E "^batch|latest|quantile 1.0" gpurun_out/rdb_r04m.log | tail -4
echo done
