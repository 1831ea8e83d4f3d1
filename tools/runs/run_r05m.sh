#!/bin/bash
# round 5: walk verdicts filled by their own k_hot_fill instance (the plain fill back at 25-36
# VGPRs): walk / hot parity, then the four bench configs without extras
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_hot.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r05m.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05m.log | head -20; tail -30 gpurun_out/t_r05m.log; exit 1; }
tail -1 gpurun_out/t_r05m.log
for cfg in sw_zipf zipf_1b mixed_tenants tb_uniform; do
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05m.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05m.log; exit 1; }
tail -1 gpurun_out/b_r05m.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg', round(d['ms_per_step'],3), {k:round(v,3) for k,v in s.items() if isinstance(v,float)}, d['status'])"
done
echo done
