#!/bin/bash
# chain_lds A/B: LDS reserved beside each hot chain (fewer normal-region waves on its CU)
set -o pipefail
mkdir -p gpurun_out
for v in 0 49152 98304; do
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 4 --tune chain_lds=$v > gpurun_out/rd_r04w_$v.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04w_$v.log; exit 1; }
echo "chain_lds=$v"; grep -E "^batch|quantile 1.0" gpurun_out/rd_r04w_$v.log | tail -2
timeout -k 10 300 python -u tools/region_debug.py --config sw_zipf --batches 2 --tune chain_lds=$v > gpurun_out/rdz_r04w_$v.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rdz_r04w_$v.log; exit 1; }
grep -E "^batch" gpurun_out/rdz_r04w_$v.log | tail -1
done
echo done
