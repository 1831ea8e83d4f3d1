#!/bin/bash
# round 5: rocprofv3 kernel trace + PMC passes (tools/profile.sh) for the given configs
# usage: run_r05u.sh <cfg>...
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
timeout -k 10 1100 bash tools/profile.sh r05_$cfg --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-extra || { echo "profile $cfg failed"; exit 1; }
done
echo done
