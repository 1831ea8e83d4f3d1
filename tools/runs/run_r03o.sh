#!/bin/bash
# greedy scan without the SW rounds path (no spills); A/B hot chains at 2 waves/SIMD (175 VGPRs, no scratch)
set -o pipefail
mkdir -p gpurun_out
true
true
for cfg in sw_zipf zipf_1b mixed_tenants; do
for v in "base" "hw2"; do
  if [ $v = hw2 ]; then export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/hw2/librl_engine.so; else unset RL_ENGINE_LIB; fi
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --steps 6 > gpurun_out/b_o_${cfg}_$v.log 2>&1 || { echo "bench $cfg $v failed"; tail -5 gpurun_out/b_o_${cfg}_$v.log; exit 1; }
  tail -1 gpurun_out/b_o_${cfg}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $v', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('region','region_offsets','unpermute','scatter0','scatter1')})"
done; done
