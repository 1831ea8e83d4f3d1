#!/bin/bash
# round 5: hot-chain allow walk — parity (walk tests, hot + config suites), then mixed_tenants /
# sw_zipf / zipf_1b bench lines with the walk on and off (rl_tune walk=0), same box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_walk.py -x -v --timeout 240 --timeout-method thread > gpurun_out/t_r05c_walk.log 2>&1 || { echo "walk tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05c_walk.log | head -20; tail -30 gpurun_out/t_r05c_walk.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r05c_walk.log | tail -1
timeout -k 10 700 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r05c_hot.log 2>&1 || { echo "hot/config tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r05c_hot.log | head -20; tail -30 gpurun_out/t_r05c_hot.log; exit 1; }
tail -1 gpurun_out/t_r05c_hot.log
for cfg in mixed_tenants zipf_1b sw_zipf; do
for w in 1 0; do
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline --tune walk=$w > gpurun_out/b_r05c.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05c.log; exit 1; }
tail -1 gpurun_out/b_r05c.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg walk=$w', round(d['ms_per_step'],3), 'region', s.get('region'), 'offs', s.get('region_offsets'), 'fill', s.get('hot_fill'), d['status'])"
done
done
echo done
