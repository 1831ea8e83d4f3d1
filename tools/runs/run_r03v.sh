#!/bin/bash
# unpermute work units (16K requests) vs 64K tiles (variant un128), interleaved, per config;
# hot-chain grid hint on tb_uniform (hot on/off); full GPU suite first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t_v_all.log 2>&1 || { tail -30 gpurun_out/t_v_all.log; exit 1; }
tail -2 gpurun_out/t_v_all.log
V=distributed-rate-limiter_amd/variants/un128/librl_engine.so
b() {  # tag config args...
  tag=$1; cfg=$2; shift 2
  timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-extra "$@" > gpurun_out/b_v_${tag}.log 2>&1 || { tail -5 gpurun_out/b_v_${tag}.log; exit 1; }
  tail -1 gpurun_out/b_v_${tag}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline'].get('kernels',{}); print('$tag', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'])"
}
for rep in 1 2; do
  for cfg in sw_zipf zipf_1b tb_uniform; do
    b ${cfg}_new_$rep $cfg || exit 1
    RL_ENGINE_LIB=$V b ${cfg}_old_$rep $cfg || exit 1
  done
  b tb_off_$rep tb_uniform --tune hot_threshold=0 || exit 1
done
timeout -k 10 200 python -u bench.py --config sw_zipf --steps 5 --warmup 3 --no-cpu-baseline --no-extra --stage-timing > gpurun_out/b_v_stages.log 2>&1 || exit 1
tail -1 gpurun_out/b_v_stages.log | cut -c1-1500
echo done
