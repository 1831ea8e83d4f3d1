#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
 for v in "" "--tune bin_shift=3"; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $v > gpurun_out/b_t_$rep.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_t_$rep.log; exit 1; }
  tail -1 gpurun_out/b_t_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $rep', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.1})"
 done
done
