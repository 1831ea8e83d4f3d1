#!/bin/bash
# hot chain cycle breakdown with the finer stamps (pre = load wait + decode + fast check)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04d_nostore.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04d_nostore.log; exit 1; }
grep -E "^batch|dur" gpurun_out/rd_r04d_nostore.log | tail -28
echo done
