#!/bin/bash
# round 5: split unpermute with 16 rounds of positions and 8 of gathers in flight (was 8 / 4):
# the gathers are latency-bound (~2.6 TB/s, 56% of wave cycles waiting). Parity of the
# partition / config tests, same-box A/B (base = HEAD) on sw_zipf, tb_uniform, zipf_1b
# result: sw_zipf unpermute 2.20/2.23 (base) vs 2.27/2.27, zipf_1b 1.13/1.13 vs 1.16/1.15: not kept
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r05v.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05v.log | head -20; tail -30 gpurun_out/t_r05v.log; exit 1; }
tail -1 gpurun_out/t_r05v.log
BASE=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so
for cfg in sw_zipf tb_uniform zipf_1b; do
for rep in 1 2; do
for v in base new; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05v.log; exit 1; }
tail -1 gpurun_out/b_r05v.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg $v', round(d['ms_per_step'],3), 'unpermute', round(s.get('unpermute'),3), d['status'])"
done
done
done
unset RL_ENGINE_LIB
echo done
