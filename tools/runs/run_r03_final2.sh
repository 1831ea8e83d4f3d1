#!/bin/bash
# round-3 final evidence (2/2): every bench config, rocprofv3 trace + PMC of tb_uniform, zipf_1b,
# mixed_tenants, region timelines
set -o pipefail
mkdir -p gpurun_out
for cfg in sw_zipf tb_uniform zipf_1b mixed_tenants; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra > gpurun_out/b_G_${cfg}.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/b_G_${cfg}.log; exit 1; }
  tail -1 gpurun_out/b_G_${cfg}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'])"
done
bash tools/profile.sh r03F_tb_uniform --config tb_uniform --steps 3 --warmup 1 --no-cpu-baseline --no-extra || exit 1
bash tools/profile.sh r03F_zipf_1b --config zipf_1b --steps 3 --warmup 1 --no-cpu-baseline --no-extra || exit 1
bash tools/profile.sh r03F_mixed_tenants --config mixed_tenants --steps 3 --warmup 1 --no-cpu-baseline --no-extra || exit 1
timeout -k 10 200 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_F_sw_zipf.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_F_mixed.log 2>&1 || exit 1
echo done
