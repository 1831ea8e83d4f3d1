#!/bin/bash
# round 6: the walk's verdict bookkeeping cost (ablation kAblWalkNoClose, results wrong by
# design) on mixed_tenants' chains; the PMC counter list of the box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || echo "counter list rc=$?"
for v in 0 8192; do
  timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 3 --tune ablate=$v > gpurun_out/rdbg_r06u_mixed_$v.log 2>&1 || { echo "rdbg failed"; exit 1; }
  grep "batch" gpurun_out/rdbg_r06u_mixed_$v.log
done
echo done
