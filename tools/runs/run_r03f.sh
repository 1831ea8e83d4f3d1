#!/bin/bash
# full GPU suite + smoke + default bench (with cpu baseline and extras) + region timeline + sw_zipf profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_f.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_f.log; exit 1; }
tail -1 gpurun_out/smoke_f.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_f.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_f.log | head -20; tail -20 gpurun_out/t_f.log; exit 1; }
tail -1 gpurun_out/t_f.log
timeout -k 10 400 python -u bench.py > gpurun_out/b_f.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_f.log; exit 1; }
tail -1 gpurun_out/b_f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'), '%.3e'%d['cpu_baseline']['value'], 'tb', '%.3e'%d['tb_uniform']['value'], d['tb_uniform']['parity'], 'config1', d['config1']['parity'], '%.3e'%d['config1']['engine_value'])"
timeout -k 10 200 python -u tools/region_debug.py --config sw_zipf --batches 3 > gpurun_out/rd_f.log 2>&1 || { echo "region_debug failed"; tail -5 gpurun_out/rd_f.log; exit 1; }
grep -E "batch|quantile 1.0|latest" gpurun_out/rd_f.log
bash tools/profile.sh r03f_sw_zipf --steps 3 --warmup 1 --no-cpu-baseline --no-extra || exit 1
for v in "SC1 --tune scatter_per_cu=1" "SC2 --tune scatter_per_cu=2" "SC3 --tune scatter_per_cu=3"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra --steps 6 "$@" > gpurun_out/b_f_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/b_f_$tag.log; exit 1; }
  tail -1 gpurun_out/b_f_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
