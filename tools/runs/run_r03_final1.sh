#!/bin/bash
# round-3 final evidence (1/2): smoke, full GPU suite, default bench (sw_zipf + tb_uniform + config1,
# CPU baseline, parity), rocprofv3 trace + PMC of sw_zipf
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_F.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_F.log; exit 1; }
tail -1 gpurun_out/smoke_F.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t_F.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_F.log | head -20; tail -20 gpurun_out/t_F.log; exit 1; }
tail -1 gpurun_out/t_F.log
timeout -k 10 400 python -u bench.py > gpurun_out/b_F.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_F.log; exit 1; }
tail -1 gpurun_out/b_F.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'), 'cpu %.3e'%d['cpu_baseline']['value'], 'tb', '%.3e'%d['tb_uniform']['value'], d['tb_uniform']['parity'], 'config1', d['config1']['parity'], '%.3e'%d['config1']['engine_value'])"
bash tools/profile.sh r03F_sw_zipf --steps 3 --warmup 1 --no-cpu-baseline --no-extra || exit 1
