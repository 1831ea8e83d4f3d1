#!/bin/bash
# round 6 A/B on one box: partition tiles of 128K requests (kTileItems 256, variants/t256) vs
# 64K (base = HEAD)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in sw_zipf tb_uniform zipf_1b; do
    for v in base t256; do
      export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/$v/librl_engine.so
      timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $cfg $v"; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$rep $cfg $v', round(d['ms_per_step'],3), {k: round(v,3) for k,v in s.items() if k in ('upsweep0','scan0','scatter0','group','unpermute','region')}, d['status'])"
    done
  done
done
