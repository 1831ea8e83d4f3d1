#!/bin/bash
# round 5: the walk common path (find, verdicts, allow) as an inner loop of its own
# (register-allocator weights): walk parity, same-box A/B (base = HEAD) on sw_zipf, mixed_tenants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_hot.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r05s.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05s.log | head -20; tail -30 gpurun_out/t_r05s.log; exit 1; }
tail -1 gpurun_out/t_r05s.log
BASE=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so
for cfg in sw_zipf mixed_tenants; do
for rep in 1 2; do
for v in base new; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05s.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05s.log; exit 1; }
tail -1 gpurun_out/b_r05s.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg $v', round(d['ms_per_step'],3), 'offs', round(s.get('region_offsets'),3), 'region', round(s.get('region'),3), d['status'])"
done
done
done
unset RL_ENGINE_LIB
echo done
