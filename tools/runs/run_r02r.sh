#!/bin/bash
# N>1 bench path rehearsal on one GPU (gloo exchange, every rank on cuda:0), then the
# current build's rocprofv3 profile of the default bench line
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
RL_BENCH_REHEARSE=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch 4194304 > gpurun_out/rehearse2.log 2>&1 || { echo "rehearsal failed"; tail -20 gpurun_out/rehearse2.log; exit 1; }
tail -1 gpurun_out/rehearse2.log | cut -c1-300
bash tools/profile.sh r02r_tb_uniform --steps 3 --warmup 1 --no-cpu-baseline || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/b_r_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r_default.log; exit 1; }
tail -1 gpurun_out/b_r_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'), d['cpu_baseline']['value'])"
