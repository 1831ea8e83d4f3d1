#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/shard_model.py --config zipf_1b --gpus 8 --debug --steps 1 > gpurun_out/sm_ff.log 2>&1 || { echo "sm failed"; tail -8 gpurun_out/sm_ff.log; exit 1; }
grep -E "top key|stages|region dur" gpurun_out/sm_ff.log | head -4
