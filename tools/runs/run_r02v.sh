#!/bin/bash
# persistent region walk A/B (waves per CU), with a parity check on batch 0 for each arm
set -o pipefail
mkdir -p gpurun_out
for c in zipf_1b mixed_tenants tb_uniform; do
 for w in 0 12 16; do
  timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --cpu-sample 8388608 --tune region_walk=$w > gpurun_out/b_v_${c}_$w.log 2>&1 || { echo "bench $c $w failed"; tail -5 gpurun_out/b_v_${c}_$w.log; exit 1; }
  tail -1 gpurun_out/b_v_${c}_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c walk=$w', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], d['parity'][:9], {k:v for k,v in d['stage_ms'].items() if v>0.5})"
 done
done
