set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/shard_model.py --config zipf_1b --gpus 8 --steps 2 --warmup 1 --debug --verify-top > gpurun_out/sm_jj_hash.log 2>&1 &&
timeout -k 10 300 python -u tools/shard_model.py --config zipf_1b --gpus 8 --steps 2 --warmup 1 --directory 4096 > gpurun_out/sm_jj_dir.log 2>&1 &&
timeout -k 10 300 python -u tools/shard_model.py --config mixed_tenants --gpus 8 --steps 2 --warmup 1 > gpurun_out/sm_jj_mixed.log 2>&1
