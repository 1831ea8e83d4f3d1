#!/bin/bash
# same-box A/B: per-key chains on (in-tree build) vs off (-DRL_NO_CHAINS)
set -o pipefail
mkdir -p gpurun_out
NC=distributed-rate-limiter_amd/ab/librl_engine_nochain.so
for rep in 1 2; do
 for c in tb_uniform zipf_1b mixed_tenants; do
  for v in base nochain; do
   lib=""; [ $v = nochain ] && lib=$NC
   RL_ENGINE_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b_n_${c}_${v}_$rep.log 2>&1 || { echo "bench $c $v failed"; tail -5 gpurun_out/b_n_${c}_${v}_$rep.log; exit 1; }
   tail -1 gpurun_out/b_n_${c}_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v $rep', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'region %.3f'%d['stage_ms']['region'], 'total %.3f'%d['stage_ms']['total'])"
  done
 done
done
