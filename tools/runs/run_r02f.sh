#!/bin/bash
# round-2 checkpoint: smoke, full GPU suite, default bench (+cpu baseline), large-config benches,
# then the rocprofv3 kernel-trace + PMC profile of the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_f.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_f.log; exit 1; }
tail -1 gpurun_out/smoke_f.log
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/t_f.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/t_f.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/b_f_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_f_default.log; exit 1; }
tail -1 gpurun_out/b_f_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'))"
for c in sw_zipf mixed_tenants zipf_1b; do
  timeout -k 10 300 python -u bench.py --config $c --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/b_f_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/b_f_$c.log; exit 1; }
  tail -1 gpurun_out/b_f_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.1})"
done
bash tools/profile.sh r02f_tb_uniform --steps 3 --warmup 1 --no-cpu-baseline
