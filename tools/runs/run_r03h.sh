#!/bin/bash
# round-3 evidence after the split scatter: smoke, full GPU suite, default bench (sw_zipf + tb_uniform + config1,
# CPU baseline, parity), rocprofv3 trace + PMC of sw_zipf
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_H.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_H.log; exit 1; }
tail -1 gpurun_out/smoke_H.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t_H.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_H.log | head -20; tail -20 gpurun_out/t_H.log; exit 1; }
tail -1 gpurun_out/t_H.log
timeout -k 10 400 python -u bench.py > gpurun_out/b_H.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_H.log; exit 1; }
tail -1 gpurun_out/b_H.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'), 'cpu %.3e'%d['cpu_baseline']['value'], 'tb', '%.3e'%d['tb_uniform']['value'], d['tb_uniform']['parity'], 'config1', d['config1']['parity'], '%.3e'%d['config1']['engine_value'])"
bash tools/profile.sh r03H_sw_zipf --steps 3 --warmup 1 --no-cpu-baseline --no-extra || exit 1
V=distributed-rate-limiter_amd/variants/sd8/librl_engine.so
RL_TUNE=unpermute_split=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_hot.py > gpurun_out/t_h_un.log 2>&1 && echo "unpermute_split tests: $(tail -1 gpurun_out/t_h_un.log)" || { tail -20 gpurun_out/t_h_un.log; exit 1; }
for rep in 1 2; do
  for v in d4 d8 un; do
    T=""
    if [ $v = d8 ]; then export RL_ENGINE_LIB=$V; else unset RL_ENGINE_LIB; fi
    if [ $v = un ]; then T="--tune unpermute_split=1"; fi
    for cfg in sw_zipf tb_uniform; do
      timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-extra --stage-timing $T > gpurun_out/b_h_${v}_${cfg}_$rep.log 2>&1 || { tail -5 gpurun_out/b_h_${v}_${cfg}_$rep.log; exit 1; }
      tail -1 gpurun_out/b_h_${v}_${cfg}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$v $cfg', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'sc0 %.3f sc1 %.3f un %.3f'%(s['scatter0'], s['scatter1'], s['unpermute']))"
    done
  done
done
unset RL_ENGINE_LIB
echo done
