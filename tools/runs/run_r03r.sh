#!/bin/bash
# two-key hot regions: 3-wave workgroups (chain3 1) or single waves running both keys' passes (chain3 0)
set -o pipefail
mkdir -p gpurun_out
RL_TUNE="chain3=0" timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_r.log | head -20; tail -20 gpurun_out/t_r.log; exit 1; }
tail -1 gpurun_out/t_r.log
for cfg in sw_zipf zipf_1b mixed_tenants; do
for v in "C3 --tune chain3=1" "C1 --tune chain3=0"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --steps 6 "$@" > gpurun_out/b_r_${cfg}_$tag.log 2>&1 || { echo "bench $cfg $tag failed"; tail -5 gpurun_out/b_r_${cfg}_$tag.log; exit 1; }
  tail -1 gpurun_out/b_r_${cfg}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('region','region_offsets','unpermute','scatter0')})"
done; done
