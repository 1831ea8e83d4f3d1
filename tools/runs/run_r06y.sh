#!/bin/bash
# round 6: why sw_zipf's scatter0 moves 3.6-4.4 ms between runs of identical code: the same
# process back to back, after a pause, after another config
set -o pipefail
mkdir -p gpurun_out
one() {  # tag cfg
  timeout -k 10 200 python -u bench.py --config $2 --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $2"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$1 $2', round(d['ms_per_step'],3), 'scatter0', s['scatter0'], 'group', s.get('group'), 'unpermute', s.get('unpermute'), 'region', s['region'])"
}
one a sw_zipf && one b sw_zipf && one c sw_zipf || exit 1
sleep 30
one d-after-30s sw_zipf || exit 1
one e tb_uniform && one f-after-tb sw_zipf || exit 1
one g zipf_1b && one h-after-z1b sw_zipf || exit 1
rocm-smi --showtemp --showpower --showclocks > gpurun_out/smi_r06y.txt 2>&1 || true
echo done
