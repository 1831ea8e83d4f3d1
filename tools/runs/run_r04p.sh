#!/bin/bash
# region wave phases (load / stream / write-back) for sw_zipf and zipf_1b; unpermute_mid XCD map
set -o pipefail
mkdir -p gpurun_out
for c in sw_zipf zipf_1b; do
timeout -k 10 300 python -u tools/region_debug.py --config $c --batches 2 > gpurun_out/rd_${c}_r04p.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_${c}_r04p.log; exit 1; }
grep -E "^batch 1|regions [0-9]+: mean|quantile 1.0" gpurun_out/rd_${c}_r04p.log | tail -4
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/b_r04p.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04p.log; exit 1; }
tail -1 gpurun_out/b_r04p.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('%.3e'%d['value'], d['ms_per_step'], d['stage_ms'])"
echo done
