#!/bin/bash
# round 5: mixed_tenants region timeline on the inner-loop walk (which chains are longest)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 4 > gpurun_out/rd_r05y_mixed.txt 2>&1 || { echo "region_debug failed"; exit 1; }
grep -E "^batch|quantile 1.0" gpurun_out/rd_r05y_mixed.txt
echo done
