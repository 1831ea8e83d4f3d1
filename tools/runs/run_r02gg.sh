#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/shard_model.py --config zipf_1b --gpus 8 --debug --steps 1 > gpurun_out/sm_gg.log 2>&1 || { echo "sm failed"; tail -8 gpurun_out/sm_gg.log; exit 1; }
grep -E "top key|region dur" gpurun_out/sm_gg.log | head -4
timeout -k 10 300 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_gg.log 2>&1 || { echo "rd failed"; tail -5 gpurun_out/rd_gg.log; exit 1; }
grep -E "^batch|quantile 1.0" gpurun_out/rd_gg.log; grep -A3 "^batch 2" gpurun_out/rd_gg.log
