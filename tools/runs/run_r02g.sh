#!/bin/bash
# sparse-templated region kernel: parity subset, default bench, stage ablations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sparse.py tests/test_gpu_hot.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_g.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_g.log; exit 1; }
tail -1 gpurun_out/t_g.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_g.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_g.log; exit 1; }
tail -1 gpurun_out/b_g.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], {k:v for k,v in d['stage_ms'].items() if v>0.02})"
timeout -k 10 300 python -u tools/ablate.py --rounds 5 --variants "ablate=0/ablate=16/ablate=4/ablate=1/ablate=2/ablate=8/ablate=2,scatter_per_cu=2/ablate=1,scatter_per_cu=2/ablate=256/ablate=512/ablate=1024/ablate=65536" > gpurun_out/abl_g.log 2>&1 || { echo "ablate failed"; tail -5 gpurun_out/abl_g.log; exit 1; }
cat gpurun_out/abl_g.log | tail -20
