#!/bin/bash
# sparse regions: new parity tests, full GPU suite, then sparse_max sweep on the large-table configs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_sparse.log 2>&1 || { echo "sparse tests failed"; tail -30 gpurun_out/t_sparse.log; exit 1; }
tail -2 gpurun_out/t_sparse.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
for c in mixed_tenants zipf_1b; do
  for sm in 0 48 96 192; do
    timeout -k 10 300 python -u bench.py --config $c --steps 4 --warmup 2 --no-cpu-baseline --tune sparse_max=$sm > gpurun_out/b_sp_${c}_$sm.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/b_sp_${c}_$sm.log; exit 1; }
    tail -1 gpurun_out/b_sp_${c}_$sm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c sm=$sm', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], {k:v for k,v in d['stage_ms'].items() if v>0.3})"
  done
done
