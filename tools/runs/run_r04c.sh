#!/bin/bash
# steady state of mixed_tenants: per-region timeline over 6 batches (hot chain cycle breakdown)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04c_mixed.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04c_mixed.log; exit 1; }
grep -E "^batch|dur" gpurun_out/rd_r04c_mixed.log | head -80
echo done
