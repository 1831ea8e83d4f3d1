#!/bin/bash
# same-box sweep of the persistent grids' workgroups per CU on the default line (sw_zipf)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for t in "" "--tune unpermute_per_cu=2" "--tune scatter_per_cu=2" "--tune upsweep_per_cu=8"; do
timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --no-extra --no-cpu-baseline $t > gpurun_out/b_r04ad.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04ad.log; exit 1; }
tail -1 gpurun_out/b_r04ad.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('[$t]', round(d['ms_per_step'],3), 'up0', s['upsweep0'], 'sc0', s['scatter0'], 'sc1', s['scatter1'], 'unp', s['unpermute'])"
done
done
echo done
