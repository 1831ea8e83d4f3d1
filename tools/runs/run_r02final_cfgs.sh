#!/bin/bash
# end-of-round: every bench config on the final build (one line each)
set -o pipefail
mkdir -p gpurun_out
for c in sw_zipf zipf_1b mixed_tenants tb_uniform; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bf_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/bf_$c.log; exit 1; }
  tail -1 gpurun_out/bf_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], d.get('parity'))"
done
