#!/bin/bash
# sliding-window greedy scan in wave_apply (vs rounds, sw_rounds=1): full GPU suite + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_k.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_k.log | head -20; tail -20 gpurun_out/t_k.log; exit 1; }
tail -1 gpurun_out/t_k.log
for cfg in sw_zipf zipf_1b mixed_tenants; do
for v in "scan" "rounds --tune sw_rounds=1"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --steps 6 "$@" > gpurun_out/b_k_${cfg}_$tag.log 2>&1 || { echo "bench $cfg $tag failed"; tail -5 gpurun_out/b_k_${cfg}_$tag.log; exit 1; }
  tail -1 gpurun_out/b_k_${cfg}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('region','region_offsets','unpermute','scatter0')})"
done; done
timeout -k 10 200 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_k.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_k.log; exit 1; }
grep -E "batch|quantile 1.0|latest|normal: sum" gpurun_out/rd_k.log
