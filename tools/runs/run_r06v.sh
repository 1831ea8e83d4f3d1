#!/bin/bash
# round 6: the allow walk keeps its block verdicts as LDS state-log indices (working tree; first
# try: verdicts stored straight to the summaries) vs the
# round-5 register block (base = HEAD, variants/base): walk parity, region debug, bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_hot.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_r06v.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r06v.log | head; tail -20 gpurun_out/t_r06v.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r06v.log | tail -1
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 3 > gpurun_out/rdbg_r06v_mixed.log 2>&1 || { echo "rdbg failed"; exit 1; }
grep "batch" gpurun_out/rdbg_r06v_mixed.log
one() {  # rep cfg v
  if [ $3 = base ]; then export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so; else unset RL_ENGINE_LIB; fi
  timeout -k 10 200 python -u bench.py --config $2 --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $2 $3"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$1 $2 $3', round(d['ms_per_step'],3), 'region', s['region'], d['status'])"
}
for rep in 1 2; do
  for cfg in mixed_tenants sw_zipf; do
    if [ $rep = 1 ]; then one $rep $cfg base && one $rep $cfg new || exit 1
    else one $rep $cfg new && one $rep $cfg base || exit 1; fi
  done
done
echo done
