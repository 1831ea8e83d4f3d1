#!/bin/bash
# end-of-round check on the clean build: smoke, full GPU suite, default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_final.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/t_final.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/t_final.log | head; exit 1; }
tail -1 gpurun_out/t_final.log
timeout -k 10 400 python -u bench.py > gpurun_out/b_final.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_final.log; exit 1; }
tail -1 gpurun_out/b_final.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], 'traffic', d['roofline']['traffic'], d.get('parity'), d['cpu_baseline']['cpu_model'], '%.3e'%d['config1']['engine_value'])"
