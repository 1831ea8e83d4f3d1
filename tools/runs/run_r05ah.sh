#!/bin/bash
# round 5: TB walk view with 32-bit lane arithmetic (elapsed from 32 bits when it fits, expiry and
# bounds as lane indices): walk parity, same-box A/B (base = HEAD) on sw_zipf, mixed_tenants
# result: slower (mixed_tenants 12.57/12.63/12.65 -> 13.07/13.09/13.09 ms/step, region +0.45 ms): not kept
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_hot.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r05ah.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05ah.log | head -20; tail -30 gpurun_out/t_r05ah.log; exit 1; }
tail -1 gpurun_out/t_r05ah.log
BASE=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so
for cfg in mixed_tenants; do
for rep in 1 2 3; do
for v in base new; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05ah.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05ah.log; exit 1; }
tail -1 gpurun_out/b_r05ah.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg $v', round(d['ms_per_step'],3), 'offs', round(s.get('region_offsets'),3), 'region', round(s.get('region'),3), d['status'])"
done
done
done
unset RL_ENGINE_LIB
echo done
