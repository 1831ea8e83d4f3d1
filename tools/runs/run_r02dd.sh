#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/shard_model.py --config zipf_1b --gpus 8 --debug --steps 1 > gpurun_out/sm_dbg.log 2>&1 || { echo "failed"; tail -8 gpurun_out/sm_dbg.log; exit 1; }
tail -9 gpurun_out/sm_dbg.log
timeout -k 10 400 python -u tools/shard_model.py --config zipf_1b --gpus 8 --directory 4096 --steps 1 > gpurun_out/sm_dir.log 2>&1 || { echo "failed"; tail -8 gpurun_out/sm_dir.log; exit 1; }
tail -1 gpurun_out/sm_dir.log
