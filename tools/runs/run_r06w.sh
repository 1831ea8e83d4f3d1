#!/bin/bash
# round 6: token-bucket rounds decide up to 3 allows per key and round (working tree) vs one
# (base = HEAD, variants/base): TB parity first, then region debug and bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hot.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r06w.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r06w.log | head; tail -20 gpurun_out/t_r06w.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r06w.log | tail -1
for v in base new; do
  if [ $v = base ]; then export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so; else unset RL_ENGINE_LIB; fi
  timeout -k 10 300 python -u tools/region_debug.py --config zipf_1b --batches 3 > gpurun_out/rdbg_r06w_z1b_$v.log 2>&1 || { echo "rdbg failed"; exit 1; }
  grep -E "^batch 2|image regions|sparse regions" gpurun_out/rdbg_r06w_z1b_$v.log | cut -c1-200
done
one() {  # rep cfg v
  if [ $3 = base ]; then export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so; else unset RL_ENGINE_LIB; fi
  timeout -k 10 200 python -u bench.py --config $2 --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $2 $3"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$1 $2 $3', round(d['ms_per_step'],3), 'region', s['region'], d['status'])"
}
for rep in 1 2; do
  for cfg in zipf_1b tb_uniform mixed_tenants sw_zipf; do
    if [ $rep = 1 ]; then one $rep $cfg base && one $rep $cfg new || exit 1
    else one $rep $cfg new && one $rep $cfg base || exit 1; fi
  done
done
echo done
