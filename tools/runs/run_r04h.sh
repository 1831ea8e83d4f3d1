#!/bin/bash
# PC sampling (stochastic, cycles) of the mixed_tenants steady state: where the hot chains spend
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 -s KILL 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d gpurun_out/pcs_r04h -o pcs --output-format csv -- python3 tools/region_debug.py --config mixed_tenants --batches 5 > gpurun_out/pcs_r04h.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 gpurun_out/pcs_r04h.log; ls -la gpurun_out/pcs_r04h/* | head
echo done
