#!/bin/bash
# round 6 A/B on one box: image regions keep expired slots as tombstones (working tree) vs the
# relink on every load (base = HEAD, variants/base)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in sw_zipf zipf_1b mixed_tenants; do
    for v in base new; do
      if [ $v = base ]; then export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so; else unset RL_ENGINE_LIB; fi
      timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $cfg $v"; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$rep $cfg $v', round(d['ms_per_step'],3), 'region', s['region'], 'scatter0', s['scatter0'], d['status'])"
    done
  done
done
