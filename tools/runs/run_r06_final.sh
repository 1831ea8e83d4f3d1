#!/bin/bash
# round-6 closing check: GPU suite, smoke, default bench line, 2-rank rehearsal (router stats), mixed
# timeline (6 batches)
set -o pipefail
mkdir -p gpurun_out/r06_final
O=gpurun_out/r06_final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" $O/gpu_suite.log | head -20; tail -20 $O/gpu_suite.log; exit 1; }
grep -E "passed|failed" $O/gpu_suite.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench_default.json
python -c "
import json; d=json.load(open('$O/bench_default.json'))
print('default', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], d.get('parity'))
for x in ('tb_uniform','zipf_1b','mixed_tenants'): print(x, '%.3e'%d[x]['value'], 'ms %.3f'%d[x]['ms_per_step'], d[x]['parity'][:40])
print('config1', d['config1']['parity'], '%.3e'%d['config1']['engine_value'], '%.3e'%d['config1']['cpu_port_value'])"
RL_BENCH_REHEARSE=1 MASTER_ADDR=127.0.0.1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 5 --warmup 2 --config zipf_1b --batch 16777216 > $O/rehearse.log 2>&1 || { echo "rehearsal failed"; tail -20 $O/rehearse.log; exit 1; }
grep "^{" $O/rehearse.log | tail -1 > $O/rehearse_zipf_1b.json
python -c "import json; d=json.load(open('$O/rehearse_zipf_1b.json')); print('rehearsal', d['router'])"
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > $O/region_debug_mixed.txt 2>&1 || { echo "region_debug failed"; tail -20 $O/region_debug_mixed.txt; exit 1; }
grep -E "^batch" $O/region_debug_mixed.txt | tail -2
echo done
