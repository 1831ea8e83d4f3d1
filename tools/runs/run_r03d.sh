#!/bin/bash
# dynamic upsweep LDS; A/B split_hot (1: chains on a side stream, 0: one launch, chains first) x region_order on every config
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_d.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_d.log | head -20; tail -20 gpurun_out/t_d.log; exit 1; }
tail -1 gpurun_out/t_d.log
for cfg in sw_zipf zipf_1b mixed_tenants tb_uniform; do
for v in "S1 --tune split_hot=1" "S0 --tune split_hot=0" "S1O0 --tune split_hot=1 --tune region_order=0"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --steps 6 "$@" > gpurun_out/b_d_${cfg}_$tag.log 2>&1 || { echo "bench $cfg $tag failed"; tail -5 gpurun_out/b_d_${cfg}_$tag.log; exit 1; }
  tail -1 gpurun_out/b_d_${cfg}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done; done
