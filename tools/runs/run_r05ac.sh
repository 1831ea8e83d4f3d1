#!/bin/bash
# round 5: walk table window of 4 views loaded together, no block prefetch (no load in flight
# across the loop back edges): walk parity, same-box A/B (base = HEAD) on sw_zipf, mixed_tenants
# result: mixed_tenants region 7.26/7.26 -> 7.00/7.23 ms but ms/step 12.65/12.69 -> 12.81/12.77; sw_zipf unchanged: no clear gain, not kept
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_hot.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r05ac.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05ac.log | head -20; tail -30 gpurun_out/t_r05ac.log; exit 1; }
tail -1 gpurun_out/t_r05ac.log
BASE=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so
for cfg in sw_zipf mixed_tenants; do
for rep in 1 2; do
for v in base new; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05ac.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05ac.log; exit 1; }
tail -1 gpurun_out/b_r05ac.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg $v', round(d['ms_per_step'],3), 'offs', round(s.get('region_offsets'),3), 'region', round(s.get('region'),3), d['status'])"
done
done
done
unset RL_ENGINE_LIB
echo done
