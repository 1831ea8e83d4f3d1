#!/bin/bash
# large-table configs: region timelines + rocprofv3 kernel trace and PMC byte counters
set -o pipefail
mkdir -p gpurun_out
for c in mixed_tenants zipf_1b; do
  timeout -k 10 300 python -u tools/region_debug.py --config $c --batches 3 > gpurun_out/rd_i_$c.log 2>&1 || { echo "region_debug $c failed"; tail -5 gpurun_out/rd_i_$c.log; exit 1; }
  head -20 gpurun_out/rd_i_$c.log | grep -E "batch|quantile 1.0|normal:" 
done
for c in mixed_tenants zipf_1b; do
  bash tools/profile.sh r02i_$c --config $c --steps 2 --warmup 1 --no-cpu-baseline || exit 1
done
