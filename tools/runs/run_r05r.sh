#!/bin/bash
# round 5: chains at 2 waves per SIMD (256 VGPRs, 96 B scratch) instead of 1 (296 incl. AGPRs),
# so two normal-region waves fit beside a chain instead of one: walk parity, same-box A/B
# (base = HEAD) on sw_zipf, mixed_tenants
# result: sw_zipf 13.00/12.98 (base) vs 13.01/13.02; mixed_tenants 14.16/14.21 vs 15.16/15.18 (region +0.9 ms): not kept
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_hot.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r05r.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05r.log | head -20; tail -30 gpurun_out/t_r05r.log; exit 1; }
tail -1 gpurun_out/t_r05r.log
BASE=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so
for cfg in sw_zipf mixed_tenants; do
for rep in 1 2; do
for v in base new; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05r.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05r.log; exit 1; }
tail -1 gpurun_out/b_r05r.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg $v', round(d['ms_per_step'],3), 'offs', round(s.get('region_offsets'),3), 'region', round(s.get('region'),3), d['status'])"
done
done
done
unset RL_ENGINE_LIB
echo done
