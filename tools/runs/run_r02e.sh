#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 3 > gpurun_out/rd8_mixed.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd8_mixed.log; exit 1; }
echo ok
