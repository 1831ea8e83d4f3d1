#!/bin/bash
# region timelines of mixed_tenants / zipf_1b with and without sparse regions
set -o pipefail
mkdir -p gpurun_out
for c in mixed_tenants zipf_1b; do
for sm in 0 96; do
  timeout -k 10 300 python -u tools/region_debug.py --config $c --batches 4 --tune sparse_max=$sm > gpurun_out/rd_${c}_$sm.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_${c}_$sm.log; exit 1; }
done
done
echo ok
