#!/bin/bash
# round 5: GPU suite after the walk inner loop and the early chain launch,
# smoke, default bench line with extras
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r05t.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r05t.log | head -20; tail -30 gpurun_out/t_r05t.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r05t.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05t.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r05t.log; exit 1; }
tail -1 gpurun_out/smoke_r05t.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_r05t.json 2> gpurun_out/b_r05t.err || { echo "bench failed"; tail -20 gpurun_out/b_r05t.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/b_r05t.json'))
print('default', d['value'], d['ms_per_step'], d['parity'], d['hbm_footprint_gb'])
for k in ('tb_uniform','zipf_1b','mixed_tenants'):
    x=d[k]; print(k, x['value'], x['ms_per_step'], x['parity'], {a:b['io_frac'] for a,b in x['roofline']['kernels'].items()})
print({a:b['io_frac'] for a,b in d['roofline']['kernels'].items()})
"
echo done
