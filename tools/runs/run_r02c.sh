#!/bin/bash
# region timelines (hot-chain counters) of mixed_tenants and zipf_1b
set -o pipefail
mkdir -p gpurun_out
for c in mixed_tenants zipf_1b sw_zipf; do
  timeout -k 10 300 python -u tools/region_debug.py --config $c --batches 3 > gpurun_out/rd2_${c}.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd2_${c}.log; exit 1; }
done
echo ok
