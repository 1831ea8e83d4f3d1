#!/bin/bash
# routing with upsweep-stored digits + 2-choice route table; A/B of route / region_order / split_hot on sw_zipf
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_c.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_c.log | head -20; tail -20 gpurun_out/t_c.log; exit 1; }
tail -1 gpurun_out/t_c.log
for v in "A" "B --tune route=0" "C --tune region_order=0" "D --tune split_hot=0" "E --tune route=0 --tune region_order=0"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra "$@" > gpurun_out/b_c_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/b_c_$tag.log; exit 1; }
  tail -1 gpurun_out/b_c_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
timeout -k 10 200 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_c.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_c.log; exit 1; }
grep -E "batch|quantile 1.0" gpurun_out/rd_c.log
