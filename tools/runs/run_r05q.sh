#!/bin/bash
# round 5: chains launched right after the hot summaries (before region order / solo), so their
# one-SIMD waves are dispatched ahead of the normal regions: hot / walk / config parity, sw_zipf
# timeline, same-box A/B (base = HEAD) on sw_zipf, zipf_1b, mixed_tenants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_hot.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r05q.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05q.log | head -20; tail -30 gpurun_out/t_r05q.log; exit 1; }
tail -1 gpurun_out/t_r05q.log
timeout -k 10 300 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_r05q_sw_zipf.txt 2>&1 || { echo "region_debug failed"; exit 1; }
grep -E "^batch|quantile 1.0|latest" gpurun_out/rd_r05q_sw_zipf.txt | cut -c1-250
BASE=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so
for cfg in sw_zipf zipf_1b mixed_tenants; do
for rep in 1 2; do
for v in base new; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05q.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05q.log; exit 1; }
tail -1 gpurun_out/b_r05q.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg $v', round(d['ms_per_step'],3), 'offs', round(s.get('region_offsets'),3), 'region', round(s.get('region'),3), d['status'])"
done
done
done
unset RL_ENGINE_LIB
echo done
