#!/bin/bash
# the other bench configs on the final build: mixed_tenants and zipf_1b lines (driver-style, no
# stage events in the timed steps)
set -o pipefail
mkdir -p gpurun_out/final
for c in mixed_tenants zipf_1b; do
timeout -k 10 500 python -u bench.py --config $c --steps 10 --warmup 3 --no-extra > gpurun_out/final/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/final/bench_$c.log; exit 1; }
tail -1 gpurun_out/final/bench_$c.log > gpurun_out/final/bench_$c.json
python -c "
import json; d=json.load(open('gpurun_out/final/bench_$c.json')); print('$c', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'), d['stage_ms'])"
done
echo done
