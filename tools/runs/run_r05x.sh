#!/bin/bash
# round 5: persistent k_regions grid (region_per_cu workgroups per CU looping over the dispatch
# order) vs one workgroup per region (region_per_cu=0): parity (parity / configs / hot / growth
# tests), then same-box A/B on all four configs
# result: slower everywhere (mixed 12.39/12.59 -> 14.64/14.56 at 12 per CU, 16.1 at 14; zipf_1b 9.07 -> 10.33; sw_zipf 13.20 -> 14.23): not kept
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_hot.py tests/test_gpu_walk.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r05x.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05x.log | head -20; tail -30 gpurun_out/t_r05x.log; exit 1; }
tail -1 gpurun_out/t_r05x.log
for cfg in mixed_tenants zipf_1b sw_zipf tb_uniform; do
for rep in 1 2; do
for rp in 0 12 14; do
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline --tune region_per_cu=$rp > gpurun_out/b_r05x.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05x.log; exit 1; }
tail -1 gpurun_out/b_r05x.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg region_per_cu=$rp', round(d['ms_per_step'],3), 'region', round(s.get('region'),3), d['status'])"
done
done
done
echo done
