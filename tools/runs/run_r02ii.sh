set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/shard_model.py --config zipf_1b --gpus 8 --steps 1 --warmup 0 --debug > gpurun_out/sm_ii.log 2>&1
