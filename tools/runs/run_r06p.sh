#!/bin/bash
# round 6: partition tile size chosen per batch (128K requests for >= 3 x 2^26, else 64K):
# two-pass parity tests, then a same-box A/B against variants/base (64K always)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r06p.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_r06p.log; exit 1; }
tail -1 gpurun_out/t_r06p.log
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export RL_ENGINE_LIB=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so; else unset RL_ENGINE_LIB; fi
    timeout -k 10 200 python -u bench.py --config sw_zipf --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $v"; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$rep sw_zipf $v', round(d['ms_per_step'],3), {k: round(v,3) for k,v in s.items() if k in ('upsweep0','scan0','scatter0','group','unpermute','region')}, d['status'])"
  done
done
