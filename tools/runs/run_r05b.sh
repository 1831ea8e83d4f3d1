#!/bin/bash
# round 5: scatter ranker by LDS representative match (vs wave_match ballots): parity of the
# partition-heavy tests, then same-box A/B of the bench lines (base = HEAD's code)
set -o pipefail
mkdir -p gpurun_out
: parity done in the previous call

BASE=$PWD/distributed-rate-limiter_amd/variants/base/librl_engine.so
for cfg in sw_zipf tb_uniform; do
for rep in 1 2 3; do
for v in base new; do
if [ $v = base ]; then export RL_ENGINE_LIB=$BASE; else unset RL_ENGINE_LIB; fi
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/b_r05b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05b.log; exit 1; }
tail -1 gpurun_out/b_r05b.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg $v', round(d['ms_per_step'],3), 'sc0', s.get('scatter0'), 'sc1', s.get('scatter1'), 'up0', s.get('upsweep0'))"
done
done
done
unset RL_ENGINE_LIB
echo done
