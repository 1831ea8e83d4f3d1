#!/bin/bash
# round 5: chain pass 2 (other keys of a hot region) with 8 chunks in flight instead of 4:
# parity, same-box A/B (base = HEAD) on all four
# result: no gain (sw_zipf region 3.24-3.32 -> 3.41-3.44 ms, others unchanged): not kept
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_walk.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r05ai.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05ai.log | head -20; tail -30 gpurun_out/t_r05ai.log; exit 1; }
tail -1 gpurun_out/t_r05ai.log
BASE=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so
for cfg in sw_zipf zipf_1b tb_uniform mixed_tenants; do
for rep in 1 2; do
for v in base new; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05ai.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05ai.log; exit 1; }
tail -1 gpurun_out/b_r05ai.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg $v', round(d['ms_per_step'],3), 'region', round(s.get('region'),3), d['status'])"
done
done
done
unset RL_ENGINE_LIB
echo done
