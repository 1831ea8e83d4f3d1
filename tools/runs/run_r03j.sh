#!/bin/bash
# router capacity error: the two owners' engines fed directly, in two concurrent processes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/repro_router_cap.py mixed_tenants 0 > gpurun_out/repro0.log 2>&1 &
p0=$!
timeout -k 10 400 python -u tools/repro_router_cap.py mixed_tenants 1 > gpurun_out/repro1.log 2>&1
r1=$?
wait $p0; r0=$?
echo "rc $r0 $r1"; grep owner gpurun_out/repro0.log gpurun_out/repro1.log
