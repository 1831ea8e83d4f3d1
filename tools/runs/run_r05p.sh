#!/bin/bash
# round 5: sw_zipf / zipf_1b region timelines (chains vs normal-region drain), walk_min default
# and 0; mixed_tenants timeline at HEAD
set -o pipefail
mkdir -p gpurun_out
for cfg in sw_zipf zipf_1b; do
for wm in 4000 0; do
timeout -k 10 300 python -u tools/region_debug.py --config $cfg --batches 3 --tune walk_min=$wm > gpurun_out/rd_r05p_${cfg}_wm$wm.txt 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_r05p_${cfg}_wm$wm.txt; exit 1; }
echo "$cfg walk_min=$wm"; grep -E "^batch|quantile 1.0|latest" gpurun_out/rd_r05p_${cfg}_wm$wm.txt | cut -c1-250
done
done
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 4 > gpurun_out/rd_r05p_mixed.txt 2>&1 || { echo "region_debug failed"; exit 1; }
grep -E "^batch|quantile 1.0" gpurun_out/rd_r05p_mixed.txt
echo done
