#!/bin/bash
# sparse_max sweep on zipf_1b and mixed_tenants (same box)
set -o pipefail
mkdir -p gpurun_out
for c in zipf_1b; do
for v in 96 48 160 256 96; do
timeout -k 10 300 python -u bench.py --config $c --steps 8 --warmup 3 --no-extra --no-cpu-baseline --tune sparse_max=$v > gpurun_out/b_r04ab.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04ab.log; exit 1; }
tail -1 gpurun_out/b_r04ab.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$c sparse_max=$v', round(d['ms_per_step'],3), 'region', d['stage_ms']['region'])"
done
done
echo done
