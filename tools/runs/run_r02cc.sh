#!/bin/bash
# busiest-shard model of the G-GPU configs (tools/shard_model.py)
set -o pipefail
mkdir -p gpurun_out
for a in "--config zipf_1b --gpus 8" "--config zipf_1b --gpus 8 --directory 4096" "--config mixed_tenants --gpus 4" "--config mixed_tenants --gpus 4 --directory 4096"; do
  timeout -k 10 400 python -u tools/shard_model.py $a > gpurun_out/sm.log 2>&1 || { echo "shard_model $a failed"; tail -8 gpurun_out/sm.log; exit 1; }
  tail -1 gpurun_out/sm.log | tee -a gpurun_out/shard_model.jsonl
done
