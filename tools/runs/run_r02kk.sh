#!/bin/bash
# A/B: [T0, T1) re-derived after every changing chunk (nd) vs left stale in runs of detailed chunks
set -o pipefail
mkdir -p gpurun_out
ND=distributed-rate-limiter_amd/librl_engine_nd.so
for v in base nd; do
  if [ $v = nd ]; then export RL_ENGINE_LIB=$ND; else unset RL_ENGINE_LIB; fi
  timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_kk_$v.log 2>&1 || { echo "rd $v failed"; tail -5 gpurun_out/rd_kk_$v.log; exit 1; }
  echo "== $v"; grep -E "^batch" gpurun_out/rd_kk_$v.log
  for c in mixed_tenants zipf_1b sw_zipf; do
    timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b_kk_${v}_$c.log 2>&1 || { echo "bench $v $c failed"; tail -5 gpurun_out/b_kk_${v}_$c.log; exit 1; }
    tail -1 gpurun_out/b_kk_${v}_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $c', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'])"
  done
done
