#!/bin/bash
# 8-wave tiles + packed per-wave counts: full GPU suite, same-box A/B vs the plain 8-wave build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_p.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/t_p.log | head -20; tail -30 gpurun_out/t_p.log; exit 1; }
tail -1 gpurun_out/t_p.log
for rep in 1 2; do
 for v in base t512; do
   lib=""; [ $v = t512 ] && lib=distributed-rate-limiter_amd/ab/librl_engine_t512.so
   RL_ENGINE_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_p_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/b_p_${v}_$rep.log; exit 1; }
   tail -1 gpurun_out/b_p_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $rep', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.02})"
 done
done
for c in mixed_tenants zipf_1b sw_zipf; do
  timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b_p_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/b_p_$c.log; exit 1; }
  tail -1 gpurun_out/b_p_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.3})"
done
