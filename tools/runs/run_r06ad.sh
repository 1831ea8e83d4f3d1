#!/bin/bash
# round 6: wave min / max by DPP + readlane instead of ds_bpermute shuffles (k_hot_summ's chunk
# summaries, wave_apply's window reference) — working tree vs base = HEAD (variants/base)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hot.py tests/test_gpu_walk.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r06ad.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r06ad.log | head; tail -20 gpurun_out/t_r06ad.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r06ad.log | tail -1
one() {  # rep cfg v
  if [ $3 = base ]; then export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so; else unset RL_ENGINE_LIB; fi
  timeout -k 10 200 python -u bench.py --config $2 --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $2 $3"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$1 $2 $3', round(d['ms_per_step'],3), 'offsets', s.get('region_offsets'), 'region', s['region'], 'scatter0', s['scatter0'], d['status'])"
}
for rep in 1 2; do
  for cfg in sw_zipf zipf_1b mixed_tenants; do
    if [ $rep = 1 ]; then one $rep $cfg base && one $rep $cfg new || exit 1
    else one $rep $cfg new && one $rep $cfg base || exit 1; fi
  done
done
echo done
