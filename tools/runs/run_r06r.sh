#!/bin/bash
# round 6 A/B on one box: hot chains as two-wave workgroups (pass 2 beside pass 1,
# rl_tune chain_split) vs one wave; parity of the split first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hot.py -x -v --timeout 120 --timeout-method thread -k "chain_split or two_keys or every_region" > gpurun_out/t_r06r.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r06r.log | head; tail -20 gpurun_out/t_r06r.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r06r.log | tail -1
for rep in 1 2; do
  for cfg in sw_zipf zipf_1b mixed_tenants; do
    for v in 0 1; do
      timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline --tune chain_split=$v > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $cfg $v"; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$rep $cfg split=$v', round(d['ms_per_step'],3), 'region', s['region'], 'scatter0', s['scatter0'], d['status'])"
    done
  done
done
for v in 0 1; do
  timeout -k 10 200 python -u tools/region_debug.py --config sw_zipf --batches 3 --tune chain_split=$v > gpurun_out/rdbg_r06r_sw_$v.log 2>&1 || { echo "rdbg failed"; exit 1; }
done
echo done
