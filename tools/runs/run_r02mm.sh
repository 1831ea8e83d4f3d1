#!/bin/bash
# A/B: hot chains prefetch the next chunk the walk will read (pf, default) vs only chunk c + 1 (nopf)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_mm.log 2>&1 || { echo "tests failed"; tail -15 gpurun_out/t_mm.log; exit 1; }
tail -1 gpurun_out/t_mm.log
for v in pf nopf; do
  if [ $v = nopf ]; then export RL_ENGINE_LIB=distributed-rate-limiter_amd/librl_engine_nopf.so; else unset RL_ENGINE_LIB; fi
  timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_mm_$v.log 2>&1 || { echo "rd $v failed"; tail -5 gpurun_out/rd_mm_$v.log; exit 1; }
  echo "== $v"; grep -E "^batch 5" -A2 gpurun_out/rd_mm_$v.log
  for c in mixed_tenants zipf_1b sw_zipf; do
    timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b_mm_${v}_$c.log 2>&1 || { echo "bench $v $c failed"; exit 1; }
    tail -1 gpurun_out/b_mm_${v}_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $c', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'])"
  done
done
