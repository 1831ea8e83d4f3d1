#!/bin/bash
# calibration again (u16 gathers kept), then tb_uniform / zipf_1b / mixed_tenants profiles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 bash tools/calib_fetch.sh gpurun_out/calib2 > gpurun_out/calib2.log 2>&1 || { echo "calib failed"; tail -20 gpurun_out/calib2.log; exit 1; }
grep -E "gather|stream16|scatter<" gpurun_out/calib2.log
for c in tb_uniform zipf_1b mixed_tenants; do
  timeout -k 10 1200 bash tools/profile.sh r04_$c --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-extra || { echo "profile $c failed"; exit 1; }
done
echo done
