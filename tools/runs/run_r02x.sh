#!/bin/bash
# round-2 final evidence: smoke, full GPU suite, default bench (+cpu baseline, config 1),
# rocprofv3 trace + PMC of tb_uniform and the large configs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_x.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_x.log; exit 1; }
tail -1 gpurun_out/smoke_x.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/t_x.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/t_x.log | head; exit 1; }
tail -1 gpurun_out/t_x.log
timeout -k 10 400 python -u bench.py > gpurun_out/b_x_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_x_default.log; exit 1; }
tail -1 gpurun_out/b_x_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'), '%.3e'%d['cpu_baseline']['value'])"
bash tools/profile.sh r02x_tb_uniform --steps 3 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r02x_mixed_tenants --config mixed_tenants --steps 2 --warmup 1 --no-cpu-baseline || exit 1
