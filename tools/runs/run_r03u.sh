#!/bin/bash
# chain-launch size hint: hot-path parity tests, tb_uniform hot on/off; scatter / unpermute
# workgroups per CU on sw_zipf (interleaved)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hot.py > gpurun_out/t_u_hot.log 2>&1 || { tail -30 gpurun_out/t_u_hot.log; exit 1; }
tail -2 gpurun_out/t_u_hot.log
b() {  # tag config args...
  tag=$1; cfg=$2; shift 2
  timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-extra "$@" > gpurun_out/b_u_${tag}.log 2>&1 || { tail -5 gpurun_out/b_u_${tag}.log; exit 1; }
  tail -1 gpurun_out/b_u_${tag}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'])"
}
for rep in 1 2; do
  b tb_on_$rep tb_uniform || exit 1
  b tb_off_$rep tb_uniform --tune hot_threshold=0 || exit 1
done
for rep in 1 2; do
  b sw_base_$rep sw_zipf || exit 1
  b sw_sc2_$rep sw_zipf --tune scatter_per_cu=2 || exit 1
  b sw_un2_$rep sw_zipf --tune unpermute_per_cu=2 || exit 1
  b sw_un4_$rep sw_zipf --tune unpermute_per_cu=4 || exit 1
done
echo done
