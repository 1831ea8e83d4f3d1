#!/bin/bash
# round 6: token-bucket rounds, 3 (working tree) vs 6 (variants/s6) allows per key and round
set -o pipefail
mkdir -p gpurun_out
one() {  # rep cfg v
  if [ $3 = s6 ]; then export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/s6/librl_engine.so; else unset RL_ENGINE_LIB; fi
  timeout -k 10 200 python -u bench.py --config $2 --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $2 $3"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$1 $2 $3', round(d['ms_per_step'],3), 'region', s['region'], d['status'])"
}
for rep in 1 2; do
  for cfg in zipf_1b tb_uniform; do
    if [ $rep = 1 ]; then one $rep $cfg s3 && one $rep $cfg s6 || exit 1
    else one $rep $cfg s6 && one $rep $cfg s3 || exit 1; fi
  done
done
export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/s6/librl_engine.so
timeout -k 10 300 python -u tools/region_debug.py --config zipf_1b --batches 3 > gpurun_out/rdbg_r06x_z1b_s6.log 2>&1 || { echo "rdbg failed"; exit 1; }
grep -E "^batch 2|image regions|sparse regions" gpurun_out/rdbg_r06x_z1b_s6.log | tail -3 | cut -c1-210
echo done
