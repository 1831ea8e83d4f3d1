#!/bin/bash
# A/B builds: 128K-request tiles (half the [bin][tile] counts), non-temporal upsweep loads; upsweep grid
set -o pipefail
mkdir -p gpurun_out
for cfg in sw_zipf tb_uniform; do
for v in base t256 ntup up8; do
  unset RL_ENGINE_LIB; args=""
  case $v in t256|ntup) export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/$v/librl_engine.so;; up8) args="--tune upsweep_per_cu=8";; esac
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --steps 6 $args > gpurun_out/b_s_${cfg}_$v.log 2>&1 || { echo "bench $cfg $v failed"; tail -5 gpurun_out/b_s_${cfg}_$v.log; exit 1; }
  tail -1 gpurun_out/b_s_${cfg}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $v', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('upsweep0','scan0','scatter0','upsweep1','scatter1','unpermute','region')})"
done; done
