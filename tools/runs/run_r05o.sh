#!/bin/bash
# round 5: hot chains: debug counters in LDS instead of scalars
# result: no gain (base 14.23/14.22 ms/step vs LDS counters 14.53/14.60); not kept
# same-box A/B on mixed_tenants (base = HEAD)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_hot.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r05o.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05o.log | head -20; tail -30 gpurun_out/t_r05o.log; exit 1; }
tail -1 gpurun_out/t_r05o.log
BASE=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so
for rep in 1 2; do
for v in base new; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --config mixed_tenants --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05o.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05o.log; exit 1; }
tail -1 gpurun_out/b_r05o.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('mixed $v', round(d['ms_per_step'],3), 'region', round(s.get('region'),3), d['status'])"
done
done
unset RL_ENGINE_LIB
echo done
