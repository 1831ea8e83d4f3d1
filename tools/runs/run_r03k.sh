#!/bin/bash
# end-of-round check on the final defaults (split scatter, split unpermute for two-pass batches):
# smoke, full GPU suite, default bench line, the other configs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_K.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_K.log; exit 1; }
tail -1 gpurun_out/smoke_K.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t_K.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_K.log | head -20; tail -20 gpurun_out/t_K.log; exit 1; }
tail -1 gpurun_out/t_K.log
timeout -k 10 400 python -u bench.py > gpurun_out/b_K.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_K.log; exit 1; }
tail -1 gpurun_out/b_K.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'), 'cpu %.3e'%d['cpu_baseline']['value'], 'tb', '%.3e'%d['tb_uniform']['value'], d['tb_uniform']['parity'], 'config1', d['config1']['parity'], '%.3e'%d['config1']['engine_value'])"
for cfg in zipf_1b mixed_tenants; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-extra --stage-timing > gpurun_out/b_K_${cfg}.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/b_K_${cfg}.log; exit 1; }
  tail -1 gpurun_out/b_K_${cfg}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k:round(v,2) for k,v in s.items()})"
done
echo done
