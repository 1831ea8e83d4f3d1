#!/bin/bash
# second dominant key per hot region (3-wave chains), fused group summaries + per-group fill; order_prefix (smallest regions dispatched first, then largest-first) x split_hot
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_e.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_e.log | head -20; tail -20 gpurun_out/t_e.log; exit 1; }
tail -1 gpurun_out/t_e.log
for cfg in sw_zipf zipf_1b; do
for v in "P0 --tune order_prefix=0" "P4k --tune order_prefix=4096" "P16k --tune order_prefix=16384" "S0 --tune split_hot=0"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --steps 6 "$@" > gpurun_out/b_e_${cfg}_$tag.log 2>&1 || { echo "bench $cfg $tag failed"; tail -5 gpurun_out/b_e_${cfg}_$tag.log; exit 1; }
  tail -1 gpurun_out/b_e_${cfg}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'region', round(d['stage_ms']['region'],2))"
done; done
timeout -k 10 200 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_e.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_e.log; exit 1; }
grep -E "batch|quantile 1.0" gpurun_out/rd_e.log
