#!/bin/bash
# FETCH/WRITE_SIZE calibration, then the sw_zipf profile (trace + PMC passes) on this build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 bash tools/calib_fetch.sh gpurun_out/calib > gpurun_out/calib.log 2>&1 || { echo "calib failed"; tail -20 gpurun_out/calib.log; exit 1; }
cat gpurun_out/calib.log | tail -8
timeout -k 10 1500 bash tools/profile.sh r04_sw_zipf --config sw_zipf --steps 3 --warmup 1 --no-cpu-baseline --no-extra || { echo "profile failed"; exit 1; }
echo done
