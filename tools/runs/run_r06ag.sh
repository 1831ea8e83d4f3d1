#!/bin/bash
# round 6: two-wave hot chains on by default — the whole GPU suite, then region stage A/B
# (chain_split 1 vs 0) alternating, three reps on sw_zipf, one on zipf_1b / mixed_tenants
set -o pipefail
mkdir -p gpurun_out/r06ag
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06ag/gpu_suite.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/r06ag/gpu_suite.log | head -20; tail -20 gpurun_out/r06ag/gpu_suite.log; exit 1; }
grep -E "passed|failed" gpurun_out/r06ag/gpu_suite.log | tail -1
one() {  # rep cfg v
  timeout -k 10 200 python -u bench.py --config $2 --steps 10 --warmup 3 --no-extra --no-cpu-baseline --tune chain_split=$3 > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $2 $3"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$1 $2 split=$3', round(d['ms_per_step'],3), 'region', s['region'], 'scatter0', s['scatter0'], d['status'])"
}
one 1 sw_zipf 1 && one 1 sw_zipf 0 && one 2 sw_zipf 0 && one 2 sw_zipf 1 && one 3 sw_zipf 1 && one 3 sw_zipf 0 || exit 1
one 1 zipf_1b 1 && one 1 zipf_1b 0 && one 1 mixed_tenants 1 && one 1 mixed_tenants 0 || exit 1
echo done
