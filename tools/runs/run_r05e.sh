#!/bin/bash
# round 5: allow walk, third version (register-block verdicts, remaining-0 and group verdicts): parity of the walk
# tests, region timelines of mixed_tenants with the walk on / off, bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_walk.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r05e_walk.log 2>&1 || { echo "walk tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05e_walk.log | head -20; tail -30 gpurun_out/t_r05e_walk.log; exit 1; }
tail -1 gpurun_out/t_r05e_walk.log
for w in 1 0; do
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 3 --tune walk=$w > gpurun_out/rd_r05e_mixed_w$w.txt 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_r05e_mixed_w$w.txt; exit 1; }
grep -E "^batch|WALK" gpurun_out/rd_r05e_mixed_w$w.txt | head -12
done
for cfg in mixed_tenants sw_zipf; do
for w in 1 0; do
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline --tune walk=$w > gpurun_out/b_r05e.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05e.log; exit 1; }
tail -1 gpurun_out/b_r05e.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg walk=$w', round(d['ms_per_step'],3), 'region', s.get('region'), 'offs', s.get('region_offsets'), 'fill', s.get('hot_fill'), d['status'])"
done
done
echo done
