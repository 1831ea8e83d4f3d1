#!/bin/bash
# same-box A/B: split scatter with 8 loader rounds in flight (RL_SPLIT_DEPTH=8) vs 4
set -o pipefail
mkdir -p gpurun_out
VAR=$PWD/distributed-rate-limiter_amd/ab/librl_engine_sd8.so
for rep in 1 2 3; do
for v in base var; do
if [ $v = var ]; then export RL_ENGINE_LIB=$VAR; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r04ae.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r04ae.log; exit 1; }
tail -1 gpurun_out/b_r04ae.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$v', round(d['ms_per_step'],3), 'sc0', s['scatter0'], 'sc1', s['scatter1'])"
done
done
unset RL_ENGINE_LIB
echo done
