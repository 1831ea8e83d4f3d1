#!/bin/bash
# round 6: walk fix (reset-only chunks), RL_E_INTERNAL, router empty-round status fold, walk
# tables allocated on demand: walk / router / hot GPU tests, then the mixed_tenants line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_router_cpp.py tests/test_gpu_hot.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r06a.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|CHECK" gpurun_out/t_r06a.log | head -20; tail -30 gpurun_out/t_r06a.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r06a.log | tail -1
timeout -k 10 300 python -u bench.py --config mixed_tenants --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r06a.json 2> gpurun_out/b_r06a.err || { echo "bench failed"; tail -20 gpurun_out/b_r06a.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/b_r06a.json'))
print('mixed', d['value'], d['ms_per_step'], d['status'], d['stage_ms'], d['hbm_footprint_gb'])
"
echo done
