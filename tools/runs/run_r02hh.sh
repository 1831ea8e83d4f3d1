#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/shard_model.py --config zipf_1b --gpus 8 --steps 1 --verify-top > gpurun_out/sm_hh.log 2>&1 || { echo "sm failed"; tail -8 gpurun_out/sm_hh.log; exit 1; }
grep -E "verify_top" gpurun_out/sm_hh.log
