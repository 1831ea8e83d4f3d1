#!/bin/bash
# scatter: vmcnt fixes (unconditional input loads, offset-selected output array) in k_scatter
# (scatter_split=0) and the split loader/ranker scatter (default), vs the previous build (head);
# partition + hot parity tests first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hot.py tests/test_gpu_configs.py > gpurun_out/t_w.log 2>&1 || { tail -30 gpurun_out/t_w.log; exit 1; }
tail -2 gpurun_out/t_w.log
V=distributed-rate-limiter_amd/variants/head/librl_engine.so
b() {  # tag config args...
  tag=$1; cfg=$2; shift 2
  timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-extra --stage-timing "$@" > gpurun_out/b_w_${tag}.log 2>&1 || { tail -5 gpurun_out/b_w_${tag}.log; exit 1; }
  tail -1 gpurun_out/b_w_${tag}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('stage_ms',{}); print('$tag', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'sc0 %.3f sc1 %.3f'%(s.get('scatter0',0), s.get('scatter1',0)))"
}
for rep in 1 2; do
  for cfg in sw_zipf tb_uniform; do
    b ${cfg}_split_$rep $cfg || exit 1
    b ${cfg}_fix_$rep $cfg --tune scatter_split=0 || exit 1
    RL_ENGINE_LIB=$V b ${cfg}_head_$rep $cfg || exit 1
  done
done
echo done
