#!/bin/bash
# same-box A/B: 4-wave tiles (in-tree) vs 8-wave tiles (RL_TILE_THREADS=512, older source)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
 for v in base t512; do
   lib=""; [ $v = t512 ] && lib=distributed-rate-limiter_amd/ab/librl_engine_t512.so
   RL_ENGINE_LIB=$lib timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/b_o_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/b_o_${v}_$rep.log; exit 1; }
   tail -1 gpurun_out/b_o_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $rep', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.02})"
 done
done
