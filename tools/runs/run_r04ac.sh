#!/bin/bash
# same-box A/B: token bucket rounds then lane-serial (variant, in-tree lib) vs rounds only (base)
set -o pipefail
mkdir -p gpurun_out
BASE=$PWD/distributed-rate-limiter_amd/ab/librl_engine_base.so
for rep in 1 2; do
for v in var base; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
for c in zipf_1b tb_uniform mixed_tenants; do
timeout -k 10 300 python -u bench.py --config $c --steps 8 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r04ac.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04ac.log; exit 1; }
tail -1 gpurun_out/b_r04ac.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v $c', round(d['ms_per_step'],3), 'region', d['stage_ms']['region'])"
done
done
done
echo done
